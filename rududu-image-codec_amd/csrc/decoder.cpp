// decoder.cpp -- the serial .ric band decoder with the range-decoder / raw-bit
// state held in registers (a local DecCore), restating the decode side of
// CBandCodec::tree / block_enum (src/lib/bandcodec.cpp:346-589), CGeomCodec /
// CBitCodec decode (src/lib/geomcodec.h:59-75, bitcodec.h:62-70) and CMuxCodec
// getBit / bitsDecode / huffDecode / enumDecode / maxDecode
// (src/lib/muxcodec.h:205-276, muxcodec.cpp:381-534).
//
// Bytes are consumed lazily in exactly the reference's order: raw-bit reads
// and range-decoder normalisations share one byte stream.  Differences are
// only in how the work is done: 16-bit enumerative codes are decoded by table
// (the combinatorial number system, k <= 8 after the complement), coefficient
// positions are visited by scanning set bits, and a geometric remainder and
// the sign bit that follows it are read as one (k + 1)-bit chunk (no range
// decoding happens between them, so the same bytes are read).
#include <cstdlib>
#include "entropy.h"
#include "coder_tables.h"

#include <cstring>
#include <vector>

namespace ric {

#include "huff_tables.inc"

namespace {

using namespace tables;

// The longest unary run of a valid stream: a `short` band stores the
// sign-magnitude 2|q| + sign in 16 bits, so |q| - 1 < 2^15; an `int` band
// (the coarsest level) is guarded at 2^20.  Past that a stream is corrupt and
// the run is cut: a hostile stream cannot keep the decoder spinning for long
// (the reference has no guard), and every valid stream decodes the same.
template <typename C> constexpr uint32_t kUnaryMax = sizeof(C) == 2 ? (1u << 15) : (1u << 20);

// binomials C(n, r) for n < 17
struct Binom {
	uint32_t c[17][17];
	Binom()
	{
		for (int n = 0; n < 17; n++)
			for (int r = 0; r < 17; r++) c[n][r] = r == 0 ? 1 : n == 0 ? 0 : c[n - 1][r - 1] + c[n - 1][r];
	}
};
const Binom kBin;

// 16-bit enumerative decode table: pattern of (k, code), k = 1..8
struct Enum16 {
	uint32_t off[9];
	std::vector<uint16_t> pat;
	Enum16()
	{
		uint32_t n = 0;
		for (int k = 1; k <= 8; k++) { off[k] = n; n += kBin.c[16][k]; }
		pat.assign(n, 0);
		for (uint32_t b = 1; b < 65536; b++) {
			const int k = __builtin_popcount(b);
			if (k > 8) continue;
			// enumCode, src/lib/muxcodec.cpp:352-359: code = sum C(n_j, j + 1)
			uint32_t code = 0, row = 0;
			for (int i = 0; i < 16; i++)
				if (b & (1u << i)) { code += kBin.c[i][row + 1]; row++; }
			pat[off[k] + code] = (uint16_t)b;
		}
	}
};
const Enum16 kEnum16;

// 8-bit first-level Huffman LUTs (sym << 8 | len; 0 = longer code)
struct HuffLutD {
	uint16_t lut[33][256];
	HuffLutD()
	{
		for (int t = 0; t < 33; t++) {
			const uint16_t* tab = t < 17 ? kHuff_LOW[t] : kHuff_HIGH[t - 17];
			const int n = t < 17 ? 17 : 16;
			for (int i = 0; i < 256; i++) {
				lut[t][i] = 0;
				for (int s = 0; s < n; s++) {
					const int len = tab[s] & 31;
					if (len <= 8 && (i >> (8 - len)) == (tab[s] >> 5)) { lut[t][i] = (uint16_t)((s << 8) | len); break; }
				}
			}
		}
	}
};
const HuffLutD kHuffLutD;

#define RIC_AI __attribute__((always_inline)) inline

// The decoder's cold state -- the code register (read only by the carry
// check of a normalisation), the stream limit and the overflow flag -- lives
// outside the register state, so the hot loop keeps range, low, the raw-bit
// buffer and the stream pointer in registers.  The rule this imposes: at most
// one DecCore per thread between its construction (from Mux::dec_state) and
// Mux::set_dec_state(d.state()) -- no nested or interleaved decodes on one
// thread (tree_dec is the only constructor and does not nest).  t_live
// enforces it: a second construction before state() aborts.
thread_local uint32_t t_code;
thread_local const uint8_t* t_limit;
thread_local bool t_ovf;
thread_local bool t_live;

struct DecCore {
	uint32_t range, low, nbits, buffer;
	const uint8_t* p;

	explicit DecCore(const Mux::DecState& s) : range(s.range), low(s.low), nbits(s.nbits), buffer(s.buffer), p(s.p)
	{
		if (t_live) abort();                                    // a nested decode on this thread (above)
		t_live = true;
		t_code = s.code; t_limit = s.limit; t_ovf = s.ovf;
	}
	Mux::DecState state() const { t_live = false; return {range, low, t_code, nbits, buffer, p, t_limit, t_ovf}; }

	RIC_AI uint8_t next()
	{
		const uint8_t b = *p;
		if (__builtin_expect(p < t_limit, 1)) p++; else t_ovf = true;
		return b;
	}
	RIC_AI void norm()                                         // normalize_dec, muxcodec.cpp:76-85
	{
		do {
			// the carry fix is rare: a predicted branch keeps t_code off the range chain
			const uint32_t code = t_code;
			if (__builtin_expect(((code - low + range - 1) ^ (code - low)) >= 0x01000000u, 0)) range = (low - code) & 4095u;
			const uint32_t b = next();
			low = (low << 8) | b;
			t_code = (code << 8) | b;
			range <<= 8;
		} while (range <= 4096u);
	}
	RIC_AI uint32_t get_bit(uint32_t freq)                       // getBit, muxcodec.h:205-213
	{
		if (__builtin_expect(range <= 4096u, 0)) norm();
		const uint32_t t = (range * freq) >> 12;
		const bool one = low >= t;                      // the same outcome, selects instead of masks
		low = one ? low - t : low;
		range = one ? range - t : t;
		return one;
	}
	RIC_AI void fill(uint32_t len)                               // fillBuffer, muxcodec.cpp:572-579
	{
		do {
			nbits += 8;
			buffer = (buffer << 8) | next();
		} while (nbits < len);
	}
	RIC_AI uint32_t bits(uint32_t len)                           // bitsDecode, muxcodec.h:233-239
	{
		if (nbits < len) fill(len);
		nbits -= len;
		return (buffer >> nbits) & ((1u << len) - 1);
	}
	RIC_AI uint32_t huff(int t, const uint16_t* tab, int n)      // huffDecode, muxcodec.h:256-276
	{
		const uint32_t c = (((buffer << 16) | ((uint32_t)p[0] << 8) | p[1]) >> nbits) & 0xFFFF;
		const uint32_t e = kHuffLutD.lut[t][c >> 8];
		uint32_t sym, len;
		if (__builtin_expect(e != 0, 1)) { sym = e >> 8; len = e & 0xFF; }
		else {
			sym = 0; len = tab[0] & 31;
			for (int s = 0; s < n; s++) {
				const uint32_t l = tab[s] & 31;
				if ((c >> (16 - l)) == (uint32_t)(tab[s] >> 5)) { sym = s; len = l; break; }
			}
		}
		p -= (int)(nbits - len) >> 3;
		if (__builtin_expect(p > t_limit, 0)) { p = t_limit; t_ovf = true; }
		if (nbits < len) buffer = p[-1];
		nbits = (nbits - len) & 7;
		return sym;
	}
	RIC_AI uint32_t enum_code(uint32_t k, uint32_t nmax)       // code part of enumDecode, muxcodec.cpp:391-393
	{
		const uint32_t lost = kCnkLost[nmax - 1][k - 1];
		uint32_t c = bits(kCnkLen[nmax - 1][k - 1] - 1);
		if (c >= lost) c = ((c << 1) | bits(1)) - lost;
		return c;
	}
	RIC_AI uint32_t enum16(uint32_t k)                          // enumDecode<16>
	{
		if (k > 8) {
			const uint32_t kk = 16 - k;
			const uint32_t c = enum_code(kk, 16);
			return ~(uint32_t)kEnum16.pat[kEnum16.off[kk] + (c < kBin.c[16][kk] ? c : 0)] & 0xFFFF;
		}
		const uint32_t c = enum_code(k, 16);
		return kEnum16.pat[kEnum16.off[k] + (c < kBin.c[16][k] ? c : 0)];
	}
	uint32_t enum_n(uint32_t k, uint32_t nmax)                  // enumDecode, muxcodec.cpp:381-405
	{
		int n = nmax - 1;
		uint32_t out = 0;
		if (k > ((nmax + 1) >> 1)) { k = nmax - k; out = (1u << nmax) - 1; }
		int row = (int)k - 1;
		uint32_t c = enum_code(k, nmax);
		while (row >= 0 && n >= 0) {
			const uint32_t v = kBin.c[n][row + 1];
			if (c >= v) { out ^= 1u << n; c -= v; row--; }
			n--;
		}
		return out;
	}
	uint32_t max_dec(uint32_t max)                              // maxDecode, muxcodec.cpp:526-534
	{
		uint32_t value = 0;
		const uint32_t len = bitlen(max), lost = (1u << len) - max - 1;
		if (len > 1) value = bits(len - 1);
		if (value >= lost) value = ((value << 1) | bits(1)) - lost;
		return value;
	}
};

struct BitM {                                                   // CBitCodec
	uint16_t freq[16];
	uint8_t shift[16], mps[16];
	BitM() { for (int i = 0; i < 16; i++) { freq[i] = 2048; shift[i] = 0; mps[i] = 0; } }
	RIC_AI uint32_t decode(DecCore& d, int c)
	{
		uint32_t sym = d.get_bit(freq[c]) ^ 1;
		const int sh = shift[c];
		freq[c] = (uint16_t)(freq[c] + (sym << (9 - sh)) - (freq[c] >> (3 + sh)));
		sym ^= mps[c];
		if ((uint16_t)(freq[c] - kBitThres[sh + 1]) > kBitThres[sh] - kBitThres[sh + 1]) {
			if (freq[c] > kBitThres[sh]) {
				if (sh == 0) { mps[c] ^= 1; freq[c] = (uint16_t)(4096 - freq[c]); shift[c] = 1; }
				else shift[c]--;
			} else if (sh < 9) shift[c]++;
		}
		return sym;
	}
};

struct GeoM {                                                   // CGeomCodec
	uint16_t freq[16];
	uint8_t idx[16];
	explicit GeoM(const uint8_t* kinit)
	{
		for (int c = 0; c < 16; c++) {
			idx[c] = kinit[c];
			freq[c] = idx[c] >= 9 ? 2048 : (uint16_t)((kGeoThres[idx[c] - 1] + kGeoThres[idx[c]]) >> 1);
		}
	}
	RIC_AI void adapt(int c, int s)
	{
		freq[c] += (4096 - freq[c]) >> (3 + s);
		if ((uint16_t)(freq[c] - kGeoThres[s - 1]) > kGeoThres[s] - kGeoThres[s - 1]) {
			if (freq[c] < kGeoThres[s - 1]) { if (idx[c] < 24) idx[c]++; }
			else if (idx[c] > 0) idx[c]--;
			if (idx[c] >= 9) freq[c] = 2048;
		}
	}
	// the signed coefficient: geometric magnitude - 1 then the raw sign bit.
	// LMAX: the longest unary run a valid stream can hold (see kUnaryMax)
	template <uint32_t LMAX>
	RIC_AI int decode_signed(DecCore& d, int c)
	{
		const uint32_t k = kGeoK[idx[c]], f = freq[c];
		const int s = kGeoShift[idx[c]];
		uint32_t l = 0;
		while (d.get_bit(f)) {
			freq[c] -= freq[c] >> (3 + s);
			if (++l > LMAX) break;                  // corrupt-stream guard
		}
		const uint32_t v = d.bits(k + 1);
		const uint32_t sym = (l << k) | (v >> 1);
		adapt(c, s);
		const int mag = (int)sym + 1;
		return (v & 1) ? -mag : mag;
	}
	RIC_AI uint32_t decode(DecCore& d, int c)
	{
		const uint32_t k = kGeoK[idx[c]], f = freq[c];
		const int s = kGeoShift[idx[c]];
		uint32_t l = 0;
		while (d.get_bit(f)) {
			freq[c] -= freq[c] >> (3 + s);
			if (++l > (1u << 20)) break;
		}
		if (k > 0) l = (l << k) | d.bits(k);
		adapt(c, s);
		return l;
	}
};

// One CGeomCodec context held in registers for the run of coefficients of a
// block (all of a block's magnitudes share one context): the model state is
// not re-read from memory after every coefficient store (a band store may
// alias the uint16_t model words for the compiler).
struct GeoReg {
	// the context's idx-dependent parameters kept ready (k, the adaptation
	// shift, its two thresholds), reloaded only when idx moves: the
	// coefficient-to-coefficient recurrence is then the frequency update
	// alone, not idx -> shift -> threshold loads (encoder.cpp GeoRegE)
	uint32_t freq, idx, k, sh, th0, span;
	RIC_AI void params()
	{
		const int s = kGeoShift[idx];
		k = kGeoK[idx]; sh = 3 + s;
		th0 = kGeoThres[s - 1]; span = (uint32_t)(kGeoThres[s] - kGeoThres[s - 1]);
	}
	RIC_AI void load(const GeoM& g, int c) { freq = g.freq[c]; idx = g.idx[c]; params(); }
	RIC_AI void store(GeoM& g, int c) const { g.freq[c] = (uint16_t)freq; g.idx[c] = (uint8_t)idx; }
	template <uint32_t LMAX>
	RIC_AI int decode_signed(DecCore& d)                         // GeoM::decode_signed
	{
		const uint32_t f = freq;
		uint32_t fr = freq, l = 0;
		while (d.get_bit(f)) {
			fr -= fr >> sh;
			if (++l > LMAX) break;                  // corrupt-stream guard
		}
		const uint32_t v = d.bits(k + 1);
		const uint32_t sym = (l << k) | (v >> 1);
		fr = (uint16_t)(fr + ((4096 - fr) >> sh));                  // adapt
		if (__builtin_expect((uint16_t)(fr - th0) > span, 0)) {
			if (fr < th0) { if (idx < 24) idx++; }
			else if (idx > 0) idx--;
			if (idx >= 9) fr = 2048;
			params();
		}
		freq = fr;
		const int mag = (int)sym + 1;
		return (v & 1) ? -mag : mag;
	}
};

template <typename P>
RIC_AI int max_len2_dec(const P* p, long st)                    // maxLen<2, decode>
{
	constexpr bool SH = sizeof(P) == 2;
	int mx = 0, mn = 0;
	for (int j = 0; j < 2; j++)
		for (int i = 0; i < 2; i++) {
			const int v = p[j * st + i];
			mx = v > mx ? v : mx;
			mn = v < mn ? v : mn;
		}
	mn = tr<SH>(-mn);
	return bitlen((uint32_t)(mn > mx ? mn : mx));
}

// The compacted output of a finest-level band (no children, so no marks):
// per block in walk order its mask of decoded positions (raster over its w
// columns), every 64 blocks the value count so far, and the values in walk
// order -- the layout k_cmp_expand (compact.hip) scatters back on the device.
struct CmpSink {
	uint16_t* mask;
	uint32_t* chunk_off;
	int16_t* vals;
	uint32_t nblk = 0, nval = 0;
	RIC_AI void block(uint32_t m)                              // after the block's values
	{
		if (!(nblk & 63)) chunk_off[nblk >> 6] = nval - (uint32_t)__builtin_popcount(m);
		mask[nblk++] = (uint16_t)m;
	}
};

template <typename C, bool HIGH, bool CMP = false>
RIC_AI int block_full_dec(DecCore& d, GeoM& g, C* blk, long st, int idx, CmpSink* cs = nullptr)
{
	constexpr bool SH = sizeof(C) == 2;
	const int t = HIGH ? 17 + idx : idx;
	const uint32_t k = HIGH ? d.huff(t, kHuff_HIGH[idx], 16) + 1 : d.huff(t, kHuff_LOW[idx], 17);
	uint32_t m = 0;
	if (HIGH || k != 0) {
		uint32_t sig = k != 16 ? d.enum16(k) : 0xFFFFu;
		const int gc = (int)k - 1;
		GeoReg r;
		r.load(g, gc);
		while (sig) {
			const int b = 31 - __builtin_clz(sig);      // bit 15 = raster position 0
			sig &= ~(1u << b);
			const int i = 15 - b;
			const C v = (C)tr<SH>(r.template decode_signed<kUnaryMax<C>>(d));
			if (CMP) { cs->vals[cs->nval++] = (int16_t)v; m |= 1u << i; }
			else blk[(i >> 2) * st + (i & 3)] = v;
		}
		r.store(g, gc);
	}
	if (CMP) cs->block(m);
	return (int)k - (HIGH ? 1 : 0);
}

// The coder state goes in and comes back by value: a DecCore whose address
// escapes into a call lives in memory, and tree_dec's loop would then load and
// store range / low through the stack on every bit.
template <typename C, bool HIGH, bool CMP = false>
__attribute__((noinline)) DecCore block_edge_dec(DecCore d, GeoM& g, C* blk, long st, int w, int h,
                                                 CmpSink* cs = nullptr)
{
	constexpr bool SH = sizeof(C) == 2;
	const uint32_t cnt = (uint32_t)(w * h);
	uint32_t k = HIGH ? d.max_dec(cnt - 1) + 1 : d.max_dec(cnt);
	if (k > cnt) k = cnt;                                       // corrupt-stream guard
	uint32_t m = 0;
	if (HIGH || k != 0) {
		uint32_t sig = k != cnt ? d.enum_n(k, cnt) : (1u << cnt) - 1;
		const int gc = kKConv2[kKConv1[cnt]][k - 1];
		for (int j = 0; j < h; j++)
			for (int i = 0; i < w; i++) {
				if (sig & (1u << (cnt - 1))) {
					const C v = (C)tr<SH>(g.template decode_signed<kUnaryMax<C>>(d, gc));
					if (CMP) { cs->vals[cs->nval++] = (int16_t)v; m |= 1u << (j * w + i); }
					else blk[j * st + i] = v;
				}
				sig <<= 1;
			}
	}
	if (CMP) cs->block(m);
	return d;
}

// CBandCodec::tree<decode>, src/lib/bandcodec.cpp:484-589
template <typename C, typename P, bool HIGH, bool CMP = false>
void tree_dec(Mux& m, const BandView& b, const BandView& par, bool has_child, CmpSink* cs = nullptr)
{
	constexpr bool SH = sizeof(C) == 2;
	static const uint8_t ginit[16] = {5,9,9,9,9,9,9,9,9,9,9,9,10,10,10,11};
	uint16_t kmean[16] = {2 << 10, 3 << 10, 4 << 10, 5 << 10, 8 << 10, 11 << 10, 13 << 10, 14 << 10,
	                      15 << 10, 15 << 10, 15 << 10, 15 << 10, 15 << 10, 15 << 10, 15 << 10, 15 << 10};
	DecCore d(m.dec_state());
	GeoM g(ginit);
	BitM tree, bord;
	const long st = b.pitch;
	const int dx = b.dx, dy = b.dy;
	P* pbase = (P*)par.p;
	const long pst = par.pitch;
	const int pdx = par.dx, pdy = par.dy;
	const C mark = (C)tr<SH>(has_child ? kInsignif : 0);
	C* band = (C*)b.p;
	// Clear() (:503) a stripe of rows at a time, just before its blocks are
	// decoded: the zeroed lines are still in cache when the coefficients land
	// (a whole-band clear first sends them to memory and reads them back)
	auto clear = [&](int j, int h) {
		if (!CMP)
			for (int r = 0; r < h; r++) memset(band + (j + r) * st, 0, sizeof(C) * dx);
	};

	// d passes through by value (a captured reference would put it in memory)
	auto edge = [&](DecCore d, C* c1, int i, int w, int h, P* pp, bool chk_row, int j) {
		if (pp && (i >> 1) < pdx && (!chk_row || (j >> 1) < pdy) && pp[i >> 1] == kInsignif) pp[i >> 1] = 0;
		if (!bord.decode(d, 0)) d = block_edge_dec<C, HIGH, CMP>(d, g, c1 + i, st, w, h, cs);
		else if (CMP) cs->block(0);
		return d;
	};

	int j = 0;
	for (; j + 4 <= dy; j += 4) {
		clear(j, 4);
		C* c1 = band + j * st;
		C* c2 = c1 + 2 * st;
		P* pp = pbase ? pbase + (long)(j >> 1) * pst : nullptr;
		int i = 0, bs = 4;
		if (j & 4) {
			bs = -4;
			i = dx & ~3;
			if (dx > i) d = edge(d, c1, i, dx - i, 4, pp, false, j);
			i += bs;
		}
		for (; i >= 0 && i + 4 <= dx; i += bs) {
			int ctx = 15;
			const int k = i >> 1;
			if (pp) {
				if (pp[k] == kInsignif) {
					pp[k] = 0;
					if (CMP) cs->block(0);                   // the finest level: mark == 0
					else c1[i] = c1[i + 2] = c2[i] = c2[i + 2] = mark;
					continue;
				}
				ctx = max_len2_dec<P>(pp + k, pst);
			}
			if (tree.decode(d, ctx)) {
				if (CMP) cs->block(0);
				else c1[i] = c1[i + 2] = c2[i] = c2[i + 2] = mark;
			} else {
				const int idx = (kmean[ctx] + (1 << 9)) >> 10;
				const int kk = block_full_dec<C, HIGH, CMP>(d, g, c1 + i, st, idx, cs);
				kmean[ctx] = (uint16_t)(kmean[ctx] + ((uint32_t)kk << 7) - (kmean[ctx] >> 3));
			}
		}
		if (i > 0 && i < dx) d = edge(d, c1, i, dx - i, 4, pp, false, j);
	}
	if (j < dy) {
		clear(j, dy - j);
		C* c1 = band + j * st;
		P* pp = pbase ? pbase + (long)(j >> 1) * pst : nullptr;
		const int h = dy - j;
		int i = 0, bs = 4;
		if (j & 4) {
			bs = -4;
			i = dx & ~3;
			if (dx > i) d = edge(d, c1, i, dx - i, h, pp, true, j);
			i += bs;
		}
		for (; i >= 0 && i + 4 <= dx; i += bs) {
			if (pp && (j >> 1) < pdy && pp[i >> 1] == kInsignif) pp[i >> 1] = 0;
			if (!bord.decode(d, 0)) d = block_edge_dec<C, HIGH, CMP>(d, g, c1 + i, st, 4, h, cs);
			else if (CMP) cs->block(0);
		}
		if (i > 0 && i < dx) d = edge(d, c1, i, dx - i, h, pp, true, j);
	}
	m.set_dec_state(d.state());
}

}  // namespace

uint32_t tree_decode_compact(Mux& m, const BandView& b, const BandView& par, uint16_t* mask, uint32_t* chunk_off,
                             int16_t* vals)
{
	CmpSink cs;
	cs.mask = mask; cs.chunk_off = chunk_off; cs.vals = vals;
	if (par.p && par.is_int) tree_dec<int16_t, int32_t, true, true>(m, b, par, false, &cs);
	else tree_dec<int16_t, int16_t, true, true>(m, b, par, false, &cs);
	return cs.nval;
}

void tree_decode_fast(Mux& m, const BandView& b, const BandView& par, bool high, bool has_child)
{
	const bool pint = par.p ? par.is_int : b.is_int;
	if (!b.is_int && !pint) {
		if (high) tree_dec<int16_t, int16_t, true>(m, b, par, has_child);
		else tree_dec<int16_t, int16_t, false>(m, b, par, has_child);
	} else if (!b.is_int) {
		if (high) tree_dec<int16_t, int32_t, true>(m, b, par, has_child);
		else tree_dec<int16_t, int32_t, false>(m, b, par, has_child);
	} else {
		if (high) tree_dec<int32_t, int32_t, true>(m, b, par, has_child);
		else tree_dec<int32_t, int32_t, false>(m, b, par, has_child);
	}
}

}  // namespace ric
