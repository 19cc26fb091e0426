// encoder.cpp -- the serial .ric band encoder over GPU block records, with the
// range-coder / raw-bit FIFO state held in registers (a local EncCore).
// Restates CBandCodec::tree<encode> (src/lib/bandcodec.cpp:484-589), CBitCodec
// / CGeomCodec code (src/lib/bitcodec.h:52-60, geomcodec.h:41-57) and CMuxCodec
// codeBin / bitsCode / normalize_enc / flushBuffer (src/lib/muxcodec.h:156-231,
// muxcodec.cpp:63-74, 536-570).  Output is byte-identical to the reference's tree<encode>.
#include "entropy.h"
#include "coder_tables.h"
#include "symbols.h"
#include "host_pool.h"
#include <atomic>
#include <memory>

namespace ric {

#include "huff_tables.inc"

namespace {

using namespace tables;

#define RIC_AI __attribute__((always_inline)) inline

// Measurement builds only (tests/native ENC_STATS): event counts of the
// serial pass by kind, and RIC_ENC_NO_RAW, which drops every raw-bit write
// (wrong output; the time of the pass without its raw-bit half).
#ifdef RIC_ENC_STATS
}  // namespace
uint64_t g_enc_stats[8];   // bins, sign bits, remainder bits, huffman bits, enum/edge raw bits, raw calls
namespace {
#define RIC_STAT(i, n) (g_enc_stats[i] += (n))
#else
#define RIC_STAT(i, n) ((void)0)
#endif

struct EncCore {
	Mux::EncState s;
	explicit EncCore(const Mux::EncState& st) : s(st) {}

	RIC_AI void put(uint8_t* slot, uint8_t v) { if (__builtin_expect(slot < s.limit, 1)) *slot = v; else s.ovf = true; }
	RIC_AI void norm()                                    // normalize_enc, muxcodec.cpp:63-74
	{
		// flushBuffer<false>: every complete raw byte first, then reserve the partial one
		while (s.ebits >= 8) {
			s.ebits -= 8;
			const uint8_t b = (uint8_t)(s.ebuf >> s.ebits);
			if (!s.reserved) put(s.p++, b); else { put(s.reserved, b); s.reserved = nullptr; }
		}
		if (s.ebits > 0 && !s.reserved) s.reserved = s.p++;
		do {
			put(s.last[s.outcount++ & 3], (uint8_t)(s.low >> 24));
			if (((s.low + s.range - 1) ^ s.low) >= 0x01000000u) s.range = (0u - s.low) & 4095u;
			s.last[(s.outcount + 3) & 3] = s.p++;
			s.range <<= 8;
			s.low <<= 8;
		} while (s.range <= 4096u);
	}
	RIC_AI void drain()                                   // emptyBuffer, muxcodec.cpp:536-548
	{
		while (s.ebits >= 8) {
			s.ebits -= 8;
			const uint8_t b = (uint8_t)(s.ebuf >> s.ebits);
			if (!s.reserved) put(s.p++, b); else { put(s.reserved, b); s.reserved = nullptr; }
		}
	}
	RIC_AI void bin(uint32_t freq, uint32_t bit)           // codeBin, muxcodec.h:156-163
	{
		RIC_STAT(0, 1);
		if (__builtin_expect(s.range <= 4096u, 0)) norm();
		const uint32_t t = (s.range * freq) >> 12;
		s.low = bit ? s.low + t : s.low;
		s.range = bit ? s.range - t : t;
	}
	RIC_AI void bits(uint32_t v, uint32_t len)             // bitsCode (64-bit FIFO, see entropy.h)
	{
		RIC_STAT(5, 1);
#ifdef RIC_ENC_NO_RAW
		return;
#endif
		if (__builtin_expect(s.ebits + len > 64, 0)) drain();
		s.ebuf = (s.ebuf << len) | v;
		s.ebits += len;
	}
};

// The modelling half alone: the same calls as EncCore, recorded as events
// for a later serial replay (replay_events).  One 64-bit event per bin, with
// the raw bits that follow it up to the next bin (raw bits never move across
// a bin: only a bin can normalise, and a normalisation is what places them):
//   bit 0 the bin's symbol, bits 1-13 its freq, bit 14 a bin is present (else
//   the event only carries raw bits: a band's leading raw field, or bits past
//   32 after one bin), bits 16-21 the raw length (<= 32), bits 32-63 the raw
//   value.
struct EvCore {
	EvBuf* buf;
	uint64_t* p;
	uint64_t* end;
	uint64_t cur = 0;                 // the event being built (0: none)
	uint32_t rlen = 0;
	explicit EvCore(EvBuf& b) : buf(&b)
	{
		if (b.cap < 4096) b.grow(4096);
		p = b.p;
		end = b.p + b.cap;
	}
	__attribute__((noinline)) void grow()
	{
		const size_t used = (size_t)(p - buf->p);
		buf->grow(buf->cap * 2);
		p = buf->p + used;
		end = buf->p + buf->cap;
	}
	RIC_AI void emit()
	{
		if (__builtin_expect(p == end, 0)) grow();
		*p++ = cur;
	}
	RIC_AI void bin(uint32_t freq, uint32_t bit)
	{
		if (cur) emit();
		cur = (uint64_t)((freq << 1) | bit | (1u << 14));
		rlen = 0;
	}
	static constexpr uint64_t kRawOnly = 4096u << 1;      // freq 4096, symbol 0, no bin: the identity
	RIC_AI void append(uint32_t v, uint32_t len)             // rlen + len <= 32
	{
		const uint64_t raw = ((cur >> 32) << len) | v;
		rlen += len;
		cur = (cur & 0xFFFFu) | ((uint64_t)rlen << 16) | (raw << 32);
	}
	RIC_AI void bits(uint32_t v, uint32_t len)
	{
		if (!cur) { cur = kRawOnly; rlen = 0; }
		if (__builtin_expect(rlen + len > 32, 0)) {
			// fill this event to 32 bits; the rest starts a raw-only event
			const uint32_t a = 32 - rlen, b = len - a;
			if (a) append(v >> b, a);
			emit();
			cur = kRawOnly;
			rlen = 0;
			v &= b >= 32 ? 0xFFFFFFFFu : (1u << b) - 1u;
			len = b;
		}
		append(v, len);
	}
	size_t finish()
	{
		if (cur) emit();
		cur = 0;
		return (size_t)(p - buf->p);
	}
};

struct BitE {                                             // CBitCodec::code
	uint16_t freq[16];
	uint8_t shift[16], mps[16];
	BitE() { for (int i = 0; i < 16; i++) { freq[i] = 2048; shift[i] = 0; mps[i] = 0; } }
	template <typename Core>
	RIC_AI void code(Core& e, uint32_t sym, int c)
	{
		const uint32_t s = sym ^ mps[c];
		e.bin(freq[c], s ^ 1);
		const int sh = shift[c];
		freq[c] = (uint16_t)(freq[c] + (s << (9 - sh)) - (freq[c] >> (3 + sh)));
		if ((uint16_t)(freq[c] - kBitThres[sh + 1]) > kBitThres[sh] - kBitThres[sh + 1]) {
			if (freq[c] > kBitThres[sh]) {
				if (sh == 0) { mps[c] ^= 1; freq[c] = (uint16_t)(4096 - freq[c]); shift[c] = 1; }
				else shift[c]--;
			} else if (sh < 9) shift[c]++;
		}
	}
};

struct GeoE {                                             // CGeomCodec::code
	uint16_t freq[16];
	uint8_t idx[16];
	explicit GeoE(const uint8_t* kinit)
	{
		for (int c = 0; c < 16; c++) {
			idx[c] = kinit[c];
			freq[c] = idx[c] >= 9 ? 2048 : (uint16_t)((kGeoThres[idx[c] - 1] + kGeoThres[idx[c]]) >> 1);
		}
	}
	// magnitude - 1 then the raw sign bit (remainder and sign as one chunk)
	template <typename Core>
	RIC_AI void code_signed(Core& e, uint32_t sym, uint32_t sign, int c)
	{
		const uint32_t k = kGeoK[idx[c]], f = freq[c];
		const int s = kGeoShift[idx[c]];
		for (uint32_t l = sym >> k; l > 0; l--) {
			e.bin(f, 1);
			freq[c] -= freq[c] >> (3 + s);
		}
		e.bin(f, 0);
		RIC_STAT(1, 1); RIC_STAT(2, k);
		e.bits(((sym & ((1u << k) - 1)) << 1) | sign, k + 1);
		freq[c] += (4096 - freq[c]) >> (3 + s);
		if ((uint16_t)(freq[c] - kGeoThres[s - 1]) > kGeoThres[s] - kGeoThres[s - 1]) {
			if (freq[c] < kGeoThres[s - 1]) { if (idx[c] < 24) idx[c]++; }
			else if (idx[c] > 0) idx[c]--;
			if (idx[c] >= 9) freq[c] = 2048;
		}
	}
};

// One CGeomCodec context in registers for the run of a block's magnitudes
// (they share one context): no model reload after every band access.
struct GeoRegE {
	// the context's idx-dependent parameters kept ready (k, the adaptation
	// shift, its two thresholds), reloaded only when idx moves
	uint32_t freq, idx, k, sh, th0, span;
	RIC_AI void params()
	{
		const int s = kGeoShift[idx];
		k = kGeoK[idx]; sh = 3 + s;
		th0 = kGeoThres[s - 1]; span = (uint32_t)(kGeoThres[s] - kGeoThres[s - 1]);
	}
	RIC_AI void load(const GeoE& g, int c) { freq = g.freq[c]; idx = g.idx[c]; params(); }
	RIC_AI void store(GeoE& g, int c) const { g.freq[c] = (uint16_t)freq; g.idx[c] = (uint8_t)idx; }
	template <typename Core>
	RIC_AI void code_signed(Core& e, uint32_t sym, uint32_t sign)   // GeoE::code_signed
	{
		const uint32_t f = freq;
		uint32_t fr = freq;
		for (uint32_t l = sym >> k; l > 0; l--) {
			e.bin(f, 1);
			fr -= fr >> sh;
		}
		e.bin(f, 0);
		RIC_STAT(1, 1); RIC_STAT(2, k);
		e.bits(((sym & ((1u << k) - 1)) << 1) | sign, k + 1);
		fr = (uint16_t)(fr + ((4096 - fr) >> sh));
		if (__builtin_expect((uint16_t)(fr - th0) > span, 0)) {
			if (fr < th0) { if (idx < 24) idx++; }
			else if (idx > 0) idx--;
			if (idx >= 9) fr = 2048;
			params();
		}
		freq = fr;
	}
};

// CMP: the values come from the frame's compacted stream (compact.hip) in
// walk order -- *cp, advanced by every block's mask population, read or
// skipped -- instead of from the dense band.
template <typename Core, typename C, bool HIGH, bool PAR, bool CMP = false>
void tree_rec_core(Core& e, const uint64_t* rec, const uint8_t* pin, const BandView& b, const int16_t** cpp = nullptr)
{
	const int16_t* cp = CMP ? *cpp : nullptr;
	constexpr bool SH = sizeof(C) == 2;
	static const uint8_t ginit[16] = {5,9,9,9,9,9,9,9,9,9,9,9,10,10,10,11};   // bandcodec.cpp:487
	uint16_t kmean[16] = {2 << 10, 3 << 10, 4 << 10, 5 << 10, 8 << 10, 11 << 10, 13 << 10, 14 << 10,
	                      15 << 10, 15 << 10, 15 << 10, 15 << 10, 15 << 10, 15 << 10, 15 << 10, 15 << 10};
	GeoE g(ginit);
	BitE tree, bord;
	const C* band = (const C*)b.p;
	const long st = b.pitch;
	const int bw = (b.dx + 3) >> 2, bh = (b.dy + 3) >> 2, nfx = b.dx >> 2;
	for (int by = 0; by < bh; by++) {
		const C* row = band + (long)by * 4 * st;
		const long rb = (long)by * bw;
		for (int p = 0; p < bw; p++) {
			// serpentine scan (bandcodec.cpp:509-523); records are in raster order
			const int bx = !(by & 1) ? p : (nfx < bw ? (p == 0 ? nfx : nfx - p) : nfx - 1 - p);
			const uint64_t r = rec[rb + bx];
			const C* blk = row + bx * 4;
			const uint32_t ins = BlockRec::insig(r);
			uint32_t mask = BlockRec::mask(r);
			if (__builtin_expect(BlockRec::edge(r), 0)) {
				bord.code(e, ins, 0);
				if (ins) { if (CMP) cp += __builtin_popcount(mask); continue; }
				RIC_STAT(4, BlockRec::rawlen(r));
				e.bits(BlockRec::raw(r), BlockRec::rawlen(r));
				const int w = BlockRec::w(r), gc = BlockRec::gctx(r);
				while (mask) {
					const int i = __builtin_ctz(mask);
					mask &= mask - 1;
					const int v = CMP ? *cp++ : blk[(i / w) * st + (i % w)];
					g.code_signed(e, (uc<SH>(v) >> 1) - 1, v & 1, gc);
				}
			} else {
				int ctx = 15;
				if (PAR) {
					const uint32_t pi = pin[rb + bx];
					if (BlockRec::pin_prop(pi)) { if (CMP) cp += __builtin_popcount(mask); continue; }
					ctx = (int)BlockRec::pin_ctx(pi);
				}
				tree.code(e, ins, ctx);
				if (ins) { if (CMP) cp += __builtin_popcount(mask); continue; }
				const uint32_t k = BlockRec::k(r);
				const int idx = (kmean[ctx] + (1 << 9)) >> 10;
				const uint16_t h = HIGH ? kHuff_HIGH[idx][k - 1] : kHuff_LOW[idx][k];
				const uint32_t rl = BlockRec::rawlen(r);
				RIC_STAT(3, h & 31); RIC_STAT(4, rl);
				e.bits(((uint32_t)(h >> 5) << rl) | BlockRec::raw(r), (h & 31) + rl);
				const int gc = (int)k - 1;
				GeoRegE gr;
				gr.load(g, gc);
				while (mask) {
					const int i = __builtin_ctz(mask);
					mask &= mask - 1;
					const int v = CMP ? *cp++ : blk[(i >> 2) * st + (i & 3)];
					gr.code_signed(e, (uc<SH>(v) >> 1) - 1, v & 1);
				}
				gr.store(g, gc);
				const uint32_t kk = k - (HIGH ? 1 : 0);
				kmean[ctx] = (uint16_t)(kmean[ctx] + (kk << 7) - (kmean[ctx] >> 3));
			}
		}
	}
	if (CMP) *cpp = cp;
}

template <typename C, bool HIGH>
void tree_rec_disp(Mux& m, const uint64_t* rec, const uint8_t* pin, const BandView& b)
{
	EncCore e(m.enc_state());
	if (pin) tree_rec_core<EncCore, C, HIGH, true>(e, rec, pin, b);
	else tree_rec_core<EncCore, C, HIGH, false>(e, rec, pin, b);
	m.set_enc_state(e.s);
}

template <typename C, bool HIGH>
size_t tree_model_disp(EvBuf& ev, const uint64_t* rec, const uint8_t* pin, const BandView& b)
{
	EvCore e(ev);
	if (pin) tree_rec_core<EvCore, C, HIGH, true>(e, rec, pin, b);
	else tree_rec_core<EvCore, C, HIGH, false>(e, rec, pin, b);
	return e.finish();
}

// the same over a compacted band's values
template <bool HIGH>
size_t tree_model_cmp(EvBuf& ev, const uint64_t* rec, const uint8_t* pin, const BandView& b, const int16_t* cv)
{
	EvCore e(ev);
	if (pin) tree_rec_core<EvCore, int16_t, HIGH, true, true>(e, rec, pin, b, &cv);
	else tree_rec_core<EvCore, int16_t, HIGH, false, true>(e, rec, pin, b, &cv);
	return e.finish();
}

}  // namespace

void tree_encode_records_fast(Mux& m, const uint64_t* rec, const uint8_t* pin, const BandView& b, bool high)
{
	if (b.is_int) { if (high) tree_rec_disp<int32_t, true>(m, rec, pin, b); else tree_rec_disp<int32_t, false>(m, rec, pin, b); }
	else { if (high) tree_rec_disp<int16_t, true>(m, rec, pin, b); else tree_rec_disp<int16_t, false>(m, rec, pin, b); }
}

void tree_encode_records_compact(Mux& m, const uint64_t* rec, const uint8_t* pin, const BandView& b, bool high,
                                 const int16_t** cp)
{
	EncCore e(m.enc_state());
	if (pin) {
		if (high) tree_rec_core<EncCore, int16_t, true, true, true>(e, rec, pin, b, cp);
		else tree_rec_core<EncCore, int16_t, false, true, true>(e, rec, pin, b, cp);
	} else {
		if (high) tree_rec_core<EncCore, int16_t, true, false, true>(e, rec, pin, b, cp);
		else tree_rec_core<EncCore, int16_t, false, false, true>(e, rec, pin, b, cp);
	}
	m.set_enc_state(e.s);
}

size_t tree_model_records(EvBuf& ev, const uint64_t* rec, const uint8_t* pin, const BandView& b, bool high)
{
	if (b.is_int) return high ? tree_model_disp<int32_t, true>(ev, rec, pin, b) : tree_model_disp<int32_t, false>(ev, rec, pin, b);
	return high ? tree_model_disp<int16_t, true>(ev, rec, pin, b) : tree_model_disp<int16_t, false>(ev, rec, pin, b);
}

size_t band_value_count(const uint64_t* rec, const BandView& b)
{
	const long n = (long)((b.dx + 3) >> 2) * ((b.dy + 3) >> 2);
	size_t c = 0;
	for (long i = 0; i < n; i++) c += (size_t)__builtin_popcount(BlockRec::mask(rec[i]));
	return c;
}

void replay_events(Mux& m, const uint64_t* ev, size_t n)
{
	EncCore e(m.enc_state());
	for (size_t i = 0; i < n; i++) {
		const uint64_t x = ev[i];
		const uint32_t lo = (uint32_t)x;
		// the bin (a raw-only event is the identity bin: freq 4096, symbol 0,
		// and no normalisation)
		if (__builtin_expect((lo >> 14) & (e.s.range <= 4096u), 0)) e.norm();
		const uint32_t freq = (lo >> 1) & 0x1FFFu, bit = lo & 1u;
		const uint32_t t = (e.s.range * freq) >> 12;
		e.s.low = bit ? e.s.low + t : e.s.low;
		e.s.range = bit ? e.s.range - t : t;
		const uint32_t len = (lo >> 16) & 63u;
		if (__builtin_expect(e.s.ebits + len > 64, 0)) e.drain();
		e.s.ebuf = (e.s.ebuf << len) | (uint32_t)(x >> 32);
		e.s.ebits += len;
	}
	m.set_enc_state(e.s);
}

void encode_bands_split(Mux& m, Pool& pool, std::vector<EvBuf>& bufs, const BandView& ll, const BandRecs* bands, int n)
{
	if ((int)bufs.size() < n) bufs.resize(n);
	std::vector<size_t> cnt(n, 0);
	std::unique_ptr<std::atomic<int>[]> done(new std::atomic<int>[n]);
	std::vector<int> big(n);
	for (int i = 0; i < n; i++) { done[i].store(0); big[i] = i; }
	std::stable_sort(big.begin(), big.end(), [&](int a, int b) {
		return (long)bands[a].v.dx * bands[a].v.dy > (long)bands[b].v.dx * bands[b].v.dy;
	});
	for (int k = 0; k < n; k++) {
		const int i = big[k];
		pool.submit([&, i] {
			const BandRecs& B = bands[i];
			if (B.cvals && !B.v.is_int)
				cnt[i] = B.high ? tree_model_cmp<true>(bufs[i], B.rec, B.pin, B.v, B.cvals)
				                : tree_model_cmp<false>(bufs[i], B.rec, B.pin, B.v, B.cvals);
			else
				cnt[i] = tree_model_records(bufs[i], B.rec, B.pin, B.v, B.high);
			done[i].store(1, std::memory_order_release);
		});
	}
	pred_encode(m, ll);
	for (int i = 0; i < n; i++) {
		while (!done[i].load(std::memory_order_acquire)) std::this_thread::yield();
		replay_events(m, bufs[i].p, cnt[i]);
	}
}

}  // namespace ric
