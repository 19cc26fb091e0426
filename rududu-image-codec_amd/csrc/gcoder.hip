// gcoder.hip -- the serial .ric coder on the GPU: one wave per stream.
//
// The .ric payload is one adaptive range-coder stream with a raw-bit FIFO
// multiplexed into it (CMuxCodec, src/lib/muxcodec.*); its state crosses every
// band, so a stream is inherently sequential.  What is
// parallel is the set of streams: a batch holds many independent frames.  Each
// frame's stream runs on one wave:
//  * every piece of coder state is wave-uniform: the compiler keeps it in
//    SGPRs and runs the coder on the scalar unit (SALU + scalar branches);
//  * the 16-context adaptive models (CBitCodec, CGeomCodec, k_mean) and the
//    small format tables live one context per lane of a VGPR ("lane arrays"),
//    read with v_readlane and written with a lane-select;
//  * the 64 lanes are the wave's load engine: they fetch the next 64 block
//    records and the next groups of block coefficients (4 blocks x 16 lanes)
//    ahead of the scalar walk, so the walk reads registers, not memory;
//  * stores (the coded bytes, decoded coefficients) go out from lane 0 as
//    vector stores.
// Output is byte-identical to the host coder (encoder.cpp / entropy.cpp),
// i.e. to the reference's tree<encode> / pred<encode> / CMuxCodec.
#include <hip/hip_runtime.h>
#include <cstdint>

#include "ric_types.h"
#include "symbols.h"
#include "coder_tables.h"
#include "gcoder.h"

namespace ric {

#include "huff_tables.inc"

namespace {

using namespace tables;

#define GC_DI __device__ __forceinline__
// global-address-space views (plain loads/stores, not flat ones that also
// count against the LDS counter)
#define GAS __attribute__((address_space(1)))
template <typename T> GC_DI const GAS T* gld(const T* p) { return (const GAS T*)p; }
template <typename T> GC_DI GAS T* gst(T* p) { return (GAS T*)p; }
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

GC_DI uint32_t lane_id() { return __lane_id(); }
// lane arrays: element i of a per-wave array held in lane i of a VGPR
GC_DI uint32_t lget(uint32_t a, uint32_t i) { return __builtin_amdgcn_readlane(a, i); }
GC_DI uint32_t lset(uint32_t a, uint32_t i, uint32_t x) { return lane_id() == i ? x : a; }

// ---------------------------------------------------------------- tables
// Per-lane constants of the models, built once per wave.
struct GTabs {
	uint32_t geo_ks;     // lane i < 25: kGeoK[i] | kGeoShift[i] << 8
	uint32_t geo_thr;    // lane s in 1..10: kGeoThres[s - 1] | kGeoThres[s] << 16
	uint32_t bit_thr;    // lane s in 0..9: kBitThres[s] | kBitThres[s + 1] << 16
	GC_DI void init()
	{
		const uint32_t l = lane_id();
		geo_ks = l < 25 ? (uint32_t)kGeoK[l] | (uint32_t)kGeoShift[l] << 8 : 0;
		geo_thr = (l >= 1 && l <= 10) ? (uint32_t)kGeoThres[l - 1] | (uint32_t)kGeoThres[l] << 16 : 0;
		bit_thr = l <= 9 ? (uint32_t)kBitThres[l] | (uint32_t)kBitThres[l + 1] << 16 : 0;
	}
};

// ------------------------------------------------------------ the encoder
// Coded bytes go to a ring in LDS and leave for HBM in 1 KiB pieces (all 64
// lanes, 16-byte stores) once no reservation slot points into them: single
// byte stores would each hold the vector-memory counter the walk's prefetch
// loads are waited on with.
constexpr uint32_t kRing = 16384;       // bytes of LDS per wave
constexpr uint32_t kFlush = 1024;
__shared__ __attribute__((aligned(16))) uint8_t g_ring[kRing];
__shared__ uint16_t g_huff[16 * 16 + 17 * 17];  // kHuff_HIGH rows, then kHuff_LOW rows
__shared__ uint32_t g_coef[64 * 16];             // the current chunk's coefficients, 16 per block

// CMuxCodec encoder state.  Byte positions are offsets from `out`; the four
// reservation slots of the carry-less coder (last[], muxcodec.cpp:63-74) are a
// FIFO q0..q3: normalize_enc writes the front one and appends p.
struct GEnc {
	uint8_t* out;
	uint32_t cap;
	uint32_t range, low, ebits;
	uint64_t ebuf;
	uint32_t p, reserved;            // reserved == 0: none (offset 0 is never a slot)
	uint32_t q0, q1, q2, q3;
	uint32_t ovf;                    // 1: past cap, 2: ring overrun
	uint32_t flushed;                // bytes [0, flushed) are in HBM
	uint32_t hdr0, hdr1, hdr2;       // the 9-byte .ric header (ric.cpp:142-152)

	GC_DI void put(uint32_t slot, uint32_t v)
	{
		if (slot < cap) {
			if (lane_id() == 0) g_ring[slot & (kRing - 1)] = (uint8_t)v;
		} else {
			ovf |= 1;
		}
	}
	// copy ring bytes [flushed, upto) (upto a multiple of 16, or the end) to HBM
	GC_DI void flush_to(uint32_t upto)
	{
		if (flushed == 0 && upto > 0) {
			// the header overwrites the coder's two leading bytes (out + 7, + 8)
			if (lane_id() == 0) {
				uint32_t* r = (uint32_t*)g_ring;
				r[0] = hdr0; r[1] = hdr1;
				g_ring[8] = (uint8_t)hdr2;
			}
		}
		const uint32_t l = lane_id();
		for (uint32_t b = flushed; b < upto; b += 64 * 16) {
			const uint32_t o = b + l * 16;
			if (o < upto && o + 16 <= ((cap + 15) & ~15u)) {
				const u32x4 v = *(const u32x4*)(g_ring + (o & (kRing - 1)));
				*gst((u32x4*)(out + o)) = v;
			}
		}
		flushed = upto;
	}
	// Called between chunks of blocks (never inside the block walk: a vector
	// store in that loop makes the compiler drain every load in flight before
	// it).  The ring must have held every byte since the last call: a chunk
	// that wrote more than the ring holds (a pathological stream) is flagged.
	GC_DI void maybe_flush()
	{
		if (p - flushed > kRing - 64) ovf |= 2;
		uint32_t lw = reserved ? (reserved < q0 ? reserved : q0) : q0;
		if (lw - flushed >= kFlush) {
			lw &= ~(kFlush - 1);
			flush_to(lw);
		}
	}
	GC_DI void raw_byte(uint32_t b)
	{
		if (!reserved) put(p++, b);
		else { put(reserved, b); reserved = 0; }
	}
	GC_DI void drain()                                   // emptyBuffer, muxcodec.cpp:536-548
	{
		while (ebits >= 8) {
			ebits -= 8;
			raw_byte((uint32_t)(ebuf >> ebits) & 255u);
		}
	}
	GC_DI void norm()                                    // normalize_enc, muxcodec.cpp:63-74
	{
		drain();                                         // flushBuffer<false>: complete bytes,
		if (ebits > 0 && !reserved) reserved = p++;      // then reserve the partial one
		do {
			put(q0, low >> 24);
			if (((low + range - 1) ^ low) >= 0x01000000u) range = (0u - low) & 4095u;
			q0 = q1; q1 = q2; q2 = q3; q3 = p++;
			range <<= 8;
			low <<= 8;
		} while (range <= 4096u);
	}
	GC_DI void bin(uint32_t freq, uint32_t bit)         // codeBin, muxcodec.h:156-163
	{
		if (range <= 4096u) norm();
		const uint32_t t = (range * freq) >> 12;
		low += t & (0u - bit);
		range = t + ((range - 2 * t) & (0u - bit));
	}
	GC_DI void bits(uint32_t v, uint32_t len)           // bitsCode, 64-bit FIFO (entropy.h)
	{
		if (ebits + len > 64) drain();
		ebuf = (ebuf << len) | v;
		ebits += len;
	}
	GC_DI void init(uint8_t* o, uint32_t c, uint32_t base)   // init_encoder at out + base
	{
		out = o; cap = c;
		low = 0; range = 1u << 16;
		ebits = 0; ebuf = 0;
		reserved = 0;
		q0 = base; q1 = base + 1; q2 = base + 2; q3 = base + 3;
		p = base + 4;
		ovf = c < base + 4 ? 1u : 0u;
		flushed = 0;
	}
	GC_DI uint32_t end()                                 // endCoding, muxcodec.cpp:87-106
	{
		drain();
		if (ebits > 0) {                                 // flushBuffer<true>: the last partial byte
			raw_byte((uint32_t)(ebuf << (8 - ebits)) & 255u);
			ebits = 0;
		}
		if (range <= 4096u) norm();
		const uint32_t last_out = 0x200 | 'W';
		if ((low & 4095u) > (last_out & 4095u)) low += 4096u;
		low = (low & ~4095u) | (last_out & 4095u);
		put(q0, low >> 24);
		put(q1, (low >> 16) & 255u);
		put(q2, (low >> 8) & 255u);
		put(q3, low & 255u);
		if (p > cap) ovf |= 1;
		if (!ovf) flush_to((p + 15) & ~15u);
		return p;
	}
};

// CBitCodec (16 contexts): lane c = freq | shift << 16 | mps << 24
struct GBit {
	uint32_t st;
	GC_DI void init() { st = 2048u; }
	GC_DI void code(GEnc& e, const GTabs& T, uint32_t sym, uint32_t c)   // bitcodec.h:52-60, 81-92
	{
		const uint32_t v = lget(st, c);
		uint32_t freq = v & 0xFFFFu, sh = (v >> 16) & 0xFFu, mps = v >> 24;
		const uint32_t s = sym ^ mps;
		e.bin(freq, s ^ 1);
		freq = (freq + (s << (9 - sh)) - (freq >> (3 + sh))) & 0xFFFFu;
		const uint32_t th = lget(T.bit_thr, sh), t0 = th & 0xFFFFu, t1 = th >> 16;
		if (((freq - t1) & 0xFFFFu) > t0 - t1) {
			if (freq > t0) {
				if (sh == 0) { mps ^= 1; freq = 4096u - freq; sh = 1; }
				else sh--;
			} else if (sh < 9) sh++;
		}
		st = lset(st, c, freq | sh << 16 | mps << 24);
	}
};

// One CGeomCodec context in scalars (geomcodec.h:41-57, 88-97): freq, idx.
struct GGeoCtx {
	uint32_t freq, idx;
	GC_DI void load(uint32_t arr, uint32_t c) { const uint32_t v = lget(arr, c); freq = v & 0xFFFFu; idx = v >> 16; }
	GC_DI uint32_t packed() const { return freq | idx << 16; }
	// magnitude - 1 (unary + k raw bits) then, if SIGNED, one raw sign bit:
	// the remainder and the sign as one chunk
	template <bool SIGNED>
	GC_DI void code(GEnc& e, const GTabs& T, uint32_t sym, uint32_t sign)
	{
		const uint32_t ks = lget(T.geo_ks, idx), k = ks & 0xFFu, s = ks >> 8;
		const uint32_t f = freq;
		uint32_t fr = freq;
		for (uint32_t l = sym >> k; l > 0; l--) {
			e.bin(f, 1);
			fr -= fr >> (3 + s);
		}
		e.bin(f, 0);
		if (SIGNED) e.bits(((sym & ((1u << k) - 1)) << 1) | sign, k + 1);
		else if (k > 0) e.bits(sym & ((1u << k) - 1), k);
		fr = (fr + ((4096u - fr) >> (3 + s))) & 0xFFFFu;
		const uint32_t th = lget(T.geo_thr, s), t0 = th & 0xFFFFu, t1 = th >> 16;
		if (((fr - t0) & 0xFFFFu) > t1 - t0) {
			if (fr < t0) { if (idx < 24) idx++; }
			else if (idx > 0) idx--;
			if (idx >= 9) fr = 2048;
		}
		freq = fr;
	}
};

GC_DI uint32_t geo_init_lane(const uint8_t* kinit)          // setCtx, geomcodec.cpp:31-41
{
	const uint32_t c = lane_id() & 15;
	const uint32_t idx = kinit[c];
	const uint32_t f = idx >= 9 ? 2048u : (uint32_t)((kGeoThres[idx - 1] + kGeoThres[idx]) >> 1);
	return f | idx << 16;
}

// taboo code, n = 2 (initTaboo / tabooCode, muxcodec.cpp:113-129, 210-240):
// nb[] is the Fibonacci run 1, 1, 2, 3, ...; sum[] its prefix sums.
GC_DI void taboo_code(GEnc& e, uint32_t nbv)
{
	const uint32_t l = lane_id();
	uint32_t fa = 1, fb = 1, sm = 0;
	for (uint32_t i = 0; i < 32; i++) {                 // lane l: nb[l], sum[l]
		const uint32_t cur = i < 2 ? 1u : fa + fb;
		if (i >= 2) { fa = fb; fb = cur; }
		sm += cur;
		if (i == l) break;
	}
	const uint32_t nbl = l < 2 ? 1u : fb, suml = sm;
	const uint32_t nt = 2;
	int i = 0, len;
	uint32_t r = 0, nb = nbv;
	while (lget(suml, (uint32_t)i) <= nb) i++;
	if (i == 0) { e.bits(0, nt); return; }
	len = i; i--;
	nb -= lget(suml, (uint32_t)i);
	while (i > (int)nt) {
		const uint32_t k = (uint32_t)i - nt + 1;
		uint32_t cnt = lget(nbl, k), j = 0;
		while (nb >= cnt) { j++; cnt += lget(nbl, k + j); }
		nb -= cnt - lget(nbl, k + j);
		j = nt - j;
		r = (r << j) | 1;
		i -= (int)j;
	}
	if (i == (int)nt) nb++;
	r = ((((r << i) | (nb & ((1u << i) - 1))) << 1) | 1) << nt;
	e.bits(r, (uint32_t)len + nt);
}

// CBandCodec::pred<encode> (LL DPCM), bandcodec.cpp:62-104.  The residuals and
// contexts of a 64-coefficient run of a row are computed by the lanes; the
// scalar walk codes them in order.
template <typename C>
GC_DI void pred_enc(GEnc& e, const GTabs& T, const GBandDesc& B, const char* arena)
{
	static constexpr uint8_t ginit[16] = {9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,15};
	const GAS C* c = gld((const C*)(arena + B.off));
	const long st = B.pitch;
	const int dx = B.dx, dy = B.dy;
	uint32_t geo = geo_init_lane(ginit);
	const uint32_t l = lane_id();
	for (int j = 0; j < dy; j++) {
		const GAS C* row = c + (long)j * st;
		for (int x0 = 0; x0 < dx; x0 += 64) {
			const int i = x0 + (int)l;
			uint32_t sym = 0, ctx = 15;
			if (i < dx) {
				const int cur = row[i];
				if (j == 0) {
					sym = i == 0 ? (uint32_t)s2u(cur) : (uint32_t)s2u(cur - row[i - 1]);
				} else if (i == 0) {
					sym = (uint32_t)s2u(cur - row[-st]);
				} else {
					const int w = row[i - 1], n = row[i - st], nw = row[i - 1 - st];
					const int a = w - nw, bb = n - nw;
					int var = bitlen((uint32_t)((a < 0 ? -a : a) + (bb < 0 ? -bb : bb)));
					if (var > 15) var = 15;
					ctx = (uint32_t)var;
					sym = (uint32_t)s2u(cur - w - n + nw);
				}
			}
			const int nx = dx - x0 < 64 ? dx - x0 : 64;
			for (int q = 0; q < nx; q++) {
				const uint32_t s = lget(sym, (uint32_t)q);
				if (j == 0 && x0 + q == 0) { taboo_code(e, s); continue; }
				const uint32_t cx = lget(ctx, (uint32_t)q);
				GGeoCtx g;
				g.load(geo, cx);
				g.code<false>(e, T, s, 0);
				geo = lset(geo, cx, g.packed());
			}
			e.maybe_flush();
		}
	}
}

// The lanes' fetch of one group of 4 blocks (scan positions s0..s0+3): lane
// 16 j + i gets coefficient i of block j, i in the block's own raster order
// over its w x h corner (the record's mask bits).  One aligned dword load per
// lane whatever the band type (no type-divergent loads into one register): a
// short band's value is the half selected by bit g of *half, taken when the
// chunk is staged (unpack_coef).
GC_DI uint32_t fetch_group(const char* band, int is_int, long st, int dx, int dy, int nblk, int s0, int g,
                           uint32_t& half)
{
	const int l = (int)lane_id();
	const int s = s0 + (l >> 4), i = l & 15;
	uint32_t v = 0;
	if (s < nblk) {
		int bx, by;
		scan_block(s, dx, dy, bx, by);
		const int w = dx - bx * 4 < 4 ? dx - bx * 4 : 4, h = dy - by * 4 < 4 ? dy - by * 4 : 4;
		if (i < w * h) {
			const int r = w == 4 ? i >> 2 : i / w, q = i - r * w;
			const long e = (long)(by * 4 + r) * st + bx * 4 + q;
			const long byte = is_int ? e * 4 : e * 2;
			v = *gld((const uint32_t*)(band + (byte & ~3l)));
			half |= (uint32_t)((byte >> 1) & 1) << g;
		}
	}
	return v;
}
GC_DI uint32_t unpack_coef(uint32_t v, int is_int, uint32_t half, int g)
{
	return is_int ? v : (v >> (((half >> g) & 1) * 16)) & 0xFFFFu;
}

// The lanes' fetch of the records of scan positions s0..s0+63.
struct RecChunk {
	uint32_t lo, hi, pin;
};
GC_DI RecChunk fetch_recs(const uint64_t* rec, const uint8_t* pin, int dx, int dy, int nblk, int s0)
{
	const int s = s0 + (int)lane_id();
	RecChunk r{0, 0, 0};
	if (s < nblk) {
		int bx, by;
		scan_block(s, dx, dy, bx, by);
		const long k = (long)by * ((dx + 3) >> 2) + bx;
		const uint64_t v = gld(rec)[k];
		r.lo = (uint32_t)v; r.hi = (uint32_t)(v >> 32);
		r.pin = pin ? gld(pin)[k] : 0u;
	}
	return r;
}

// The coefficients of one block: unary + raw remainder + sign each, one
// geometric context (CGeomCodec::code, geomcodec.h:41-57; block_enum's
// coefficient loop, bandcodec.cpp:392-401).
GC_DI void code_coefs(GEnc& e, const GTabs& T, uint32_t& geo, uint32_t gc, uint32_t mask, uint32_t cv, uint32_t cb)
{
	GGeoCtx g;
	g.load(geo, gc);
	while (mask) {
		const uint32_t i = (uint32_t)__builtin_ctz(mask);
		mask &= mask - 1;
		const uint32_t u = lget(cv, cb + i);
		g.code<true>(e, T, (u >> 1) - 1, u & 1);
	}
	geo = lset(geo, gc, g.packed());
}

// CBandCodec::tree<encode> over the GPU block records (encoder.cpp
// tree_rec_fast; bandcodec.cpp:484-589 with block_enum :346-478).  high: the
// finest level (HIGH tables); par: the band has a parent level.
GC_DI void tree_enc(GEnc& e, const GTabs& T, const GBandDesc& B, const char* arena)
{
	const bool high = B.high, par = B.has_pin;
	const uint64_t* rec = (const uint64_t*)(arena + B.rec_off);
	const uint8_t* pin = par ? (const uint8_t*)(arena + B.pin_off) : nullptr;
	const char* band = arena + B.off;
	const int is_int = B.is_int;
	const long st = B.pitch;
	const int dx = B.dx, dy = B.dy;
	const int nblk = ((dx + 3) >> 2) * ((dy + 3) >> 2);
	const uint32_t l = lane_id();
	// CGeomCodec init {5,9,9,...,10,10,10,11} (bandcodec.cpp:487)
	const uint32_t gidx = l == 0 ? 5u : (l < 12 ? 9u : (l < 15 ? 10u : 11u));
	uint32_t geo = (gidx >= 9 ? 2048u : (uint32_t)((kGeoThres[gidx - 1] + kGeoThres[gidx]) >> 1)) | gidx << 16;
	GBit tree, bord;
	tree.init(); bord.init();
	// k_mean init 2,3,4,5,8,11,13,14,15,... << 10 (bandcodec.cpp:488-489)
	uint32_t kmean = l < 8 ? (uint32_t)((l < 4 ? l + 2 : (l == 4 ? 8 : (l == 5 ? 11 : (l == 6 ? 13 : 14)))) << 10)
	                       : 15u << 10;
	const uint32_t hbase = high ? 0u : 256u, hrow = high ? 16u : 17u;
	const uint32_t hoff = high ? 0xFFFFFFFFu : 0u;      // HIGH tables index k - 1
	// Chunks of 64 blocks in scan order.  The loads of chunk c + 1 (records,
	// 16 groups of 4 blocks' coefficients) are issued when chunk c starts and
	// consumed a whole chunk later, in one wait; chunk c's coefficients then
	// sit in LDS (g_coef), one 16-lane row per block.
	RecChunk rn = fetch_recs(rec, pin, dx, dy, nblk, 0);
	uint32_t cn[16], half = 0;
	RIC_UNROLL
	for (int g = 0; g < 16; g++) cn[g] = fetch_group(band, is_int, st, dx, dy, nblk, 4 * g, g, half);
	for (int s0 = 0; s0 < nblk; s0 += 64) {
		const RecChunk rc = rn;
		RIC_UNROLL
		for (int g = 0; g < 16; g++) g_coef[g * 64 + l] = unpack_coef(cn[g], is_int, half, g);
		if (s0 + 64 < nblk) {
			rn = fetch_recs(rec, pin, dx, dy, nblk, s0 + 64);
			half = 0;
			RIC_UNROLL
			for (int g = 0; g < 16; g++) cn[g] = fetch_group(band, is_int, st, dx, dy, nblk, s0 + 64 + 4 * g, g, half);
		}
		const int nj = nblk - s0 < 64 ? nblk - s0 : 64;
		for (int j = 0; j < nj; j++) {
			const uint32_t li = (uint32_t)j;
			const uint64_t r = (uint64_t)lget(rc.lo, li) | (uint64_t)lget(rc.hi, li) << 32;
			const uint32_t ins = BlockRec::insig(r);
			const uint32_t mask = BlockRec::mask(r);
			if (BlockRec::edge(r)) {
				bord.code(e, T, ins, 0);
				if (ins) continue;
				e.bits(BlockRec::raw(r), BlockRec::rawlen(r));
				const uint32_t cv = g_coef[j * 16 + (l & 15)];
				code_coefs(e, T, geo, BlockRec::gctx(r), mask, cv, 0);
			} else {
				uint32_t ctx = 15;
				if (par) {
					const uint32_t pi = lget(rc.pin, li);
					if (BlockRec::pin_prop(pi)) continue;
					ctx = BlockRec::pin_ctx(pi);
				}
				tree.code(e, T, ins, ctx);
				if (ins) continue;
				const uint32_t cv = g_coef[j * 16 + (l & 15)];
				const uint32_t k = BlockRec::k(r);
				const uint32_t km = lget(kmean, ctx);
				const uint32_t idx = (km + (1u << 9)) >> 10;
				const uint32_t h = g_huff[hbase + idx * hrow + k + hoff];
				const uint32_t rl = BlockRec::rawlen(r);
				e.bits(((h >> 5) << rl) | BlockRec::raw(r), (h & 31) + rl);
				code_coefs(e, T, geo, k - 1, mask, cv, 0);
				const uint32_t kk = high ? k - 1 : k;
				kmean = lset(kmean, ctx, (km + (kk << 7) - (km >> 3)) & 0xFFFFu);
			}
		}
		e.maybe_flush();
	}
}

// One frame's stream per workgroup (one wave): the reference's CompressImage
// coding order (src/ric/ric.cpp:157-176 -> CWavelet2D::CodeBand,
// src/lib/wavelet2d.cpp:150-177): the coarsest LL, then every level coarse to
// fine, V, H, D.  The .ric file goes to out + f * ostride: the 9-byte header
// (ric.cpp:142-152) then the payload; the coder buffer starts at out + 7 and
// the header overwrites its two dropped leading bytes (as ric_codec).
__global__ void __launch_bounds__(64) k_gc_encode(const GEncArgs* __restrict__ ap)
{
	const GEncArgs& a = *ap;
	const int f = blockIdx.x;
	const char* arena = a.arena + (size_t)f * a.astride;
	uint8_t* out = a.out + (size_t)f * a.ostride;
	for (int i = (int)threadIdx.x; i < 16 * 16 + 17 * 17; i += 64)
		g_huff[i] = i < 256 ? kHuff_HIGH[i >> 4][i & 15] : kHuff_LOW[(i - 256) / 17][(i - 256) % 17];
	__syncthreads();
	const int32_t status = *gld((const int32_t*)(arena + a.status_off));
	GTabs T;
	T.init();
	GEnc e;
	e.init(out, (uint32_t)a.cap, 7);
	e.hdr0 = 'R' | 'U' << 8 | 'D' << 16 | (uint32_t)'2' << 24;
	e.hdr1 = (uint32_t)(a.w & 0xFFFF) | (uint32_t)(a.h & 0xFFFF) << 16;
	e.hdr2 = (uint32_t)((a.q & 31) | ((a.trans & 3) << 6));
	if (a.ll.is_int) pred_enc<int32_t>(e, T, a.ll, arena);
	else pred_enc<int16_t>(e, T, a.ll, arena);
	for (int b = 0; b < a.nb; b++) tree_enc(e, T, a.b[b], arena);
	const uint32_t end = e.end();
	uint32_t rc = 0;
	if (status) rc = 2;                                  // a fused kernel's ring timeout
	else if (e.ovf & 2) rc = 3;                          // the LDS ring overran (pathological stream)
	else if (e.ovf) rc = 1;
	if (lane_id() == 0) {
		gst(a.res)[2 * f] = rc ? 0u : end;               // file length = 9 + (end - 7) - 2
		gst(a.res)[2 * f + 1] = rc;
	}
}

}  // namespace

int launch_gc_encode(const GEncArgs* dev_args, int nframes, hipStream_t st)
{
	if (nframes <= 0) return 0;
	hipLaunchKernelGGL(k_gc_encode, dim3(nframes), dim3(64), 0, st, dev_args);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace ric
