// symbols.h -- per-block symbolisation of the zerotree band scan
// (CBandCodec::tree<encode>, src/lib/bandcodec.cpp:484-589 and block_enum
// :346-478), as a pure function of the quantised bands so it can run one lane
// per 4x4 block on the GPU (symbols.hip).  The host then only runs the adaptive
// models and the range coder over the records (entropy.cpp).
//
// Facts used (all from the encoder side of tree()):
//  * A full block is skipped ("propagated") iff its parent anchor holds the
//    INSIGNIF marker when the band is scanned, i.e. iff the parent 4x4 block
//    containing (2*bx, 2*by) is a full block whose buildTree result was
//    insignificant (tree() copies that marker to all four anchors,
//    bandcodec.cpp:528-536).  Parent edge blocks never set anchors.
//  * The parent context maxLen<2,encode> starts from max = 0, so negative
//    marker values never contribute (bandcodec.cpp:330-340).
//  * A block is insignificant iff buildTree left the marker at its top-left.
// The record is split so the block-local part can be produced by the kernel
// that quantises the block, and the parent-dependent part by the kernel that
// quantises the parent level (the fused forward+quantiser, dwt.hip).
#pragma once
#include <cstdint>
#include "ric_types.h"

namespace ric {

// Two arrays per band, both in RASTER block order (index by * bw + bx); the
// host encoder walks them in the reference's serpentine scan order.
//
// rec (u64): what the block itself determines (written by whoever quantises
// the block: the fused forward+quantiser kernel, or k_blocks)
//  [0,16)  significance mask, bit i = raster position i inside the block
//  [16,32) precomputed raw bits (enumCode; maxCode + enumCode for edge blocks)
//  [32,37) their length
//  [37,42) k = non-zero count
//  46 edge, 47 insignificant
//  [49,53) geometric-coder context of the block's coefficients
//  [53,55) edge width - 1, [55,57) edge height - 1
// pin (u8): what the parent block determines (written by whoever quantises the
// PARENT level; absent for the coarsest level, whose blocks have no parent)
//  [0,5) tree context maxLen<2> of the parent 2x2 (bandcodec.cpp:324-344)
//  7     propagated: the parent is a full block left insignificant by
//        buildTree, so tree() skips this block (bandcodec.cpp:525-531).  Only
//        meaningful for full blocks (edge blocks never look at the parent).
struct BlockRec {
	static RIC_HD uint32_t mask(uint64_t r) { return (uint32_t)(r & 0xFFFF); }
	static RIC_HD uint32_t raw(uint64_t r) { return (uint32_t)((r >> 16) & 0xFFFF); }
	static RIC_HD uint32_t rawlen(uint64_t r) { return (uint32_t)((r >> 32) & 31); }
	static RIC_HD uint32_t k(uint64_t r) { return (uint32_t)((r >> 37) & 31); }
	static RIC_HD bool edge(uint64_t r) { return (r >> 46) & 1; }
	static RIC_HD bool insig(uint64_t r) { return (r >> 47) & 1; }
	static RIC_HD uint32_t gctx(uint64_t r) { return (uint32_t)((r >> 49) & 15); }
	static RIC_HD uint32_t w(uint64_t r) { return (uint32_t)((r >> 53) & 3) + 1; }
	static RIC_HD uint32_t h(uint64_t r) { return (uint32_t)((r >> 55) & 3) + 1; }
	static RIC_HD uint32_t pin_ctx(uint32_t p) { return p & 31; }
	static RIC_HD bool pin_prop(uint32_t p) { return (p >> 7) & 1; }
};

// format constants (src/lib/muxcodec.cpp:294-332, bandcodec.cpp:409-423)
struct SymTables {
	uint16_t cnk[8][16];
	uint8_t cnk_len[16][8];
	uint16_t cnk_lost[16][8];
	uint8_t kconv2[9][16];
	uint8_t kconv1[16];
};

#if defined(__HIPCC__)
#define RIC_TABLE_SPACE __constant__
#else
#define RIC_TABLE_SPACE
#endif

RIC_HD void enum_bits(const SymTables& T, uint32_t bits, uint32_t k, uint32_t nmax, uint32_t& code_out, uint32_t& len_out)
{
	// CMuxCodec::enumCode, src/lib/muxcodec.cpp:341-365 (bits: reference order)
	uint32_t code = 0, n = 0, row = 0;
	if (k > ((nmax + 1) >> 1)) { k = nmax - k; bits ^= (1u << nmax) - 1; }
	while (bits != 0) {
		if (bits & 1) { code += T.cnk[row][n]; row++; }
		n++;
		bits >>= 1;
	}
	const uint32_t lost = T.cnk_lost[nmax - 1][k - 1], len = T.cnk_len[nmax - 1][k - 1];
	if (code < lost) { code_out = code; len_out = len - 1; }
	else { code_out = code + lost; len_out = len; }
}

RIC_HD void max_bits(uint32_t value, uint32_t max, uint32_t& code_out, uint32_t& len_out)
{
	// CMuxCodec::maxCode, src/lib/muxcodec.cpp:516-524
	const uint32_t len = (uint32_t)bitlen(max), lost = (1u << len) - max - 1;
	if (value < lost) { code_out = value; len_out = len - 1; }
	else { code_out = value + lost; len_out = len; }
}

// enumCode of a full 16-coefficient mask by two table lookups (the device
// fast path): the code is a sum over set bits of C(n, rank + 1)
// (Cnk, src/lib/muxcodec.cpp:282-292, 341-365), split at bit 8 -- lo[] holds
// the sum over bits 0..7, hi[klo][] the sum over bits 8..15 after klo lower set
// bits.  Only k <= 8 is ever looked up (the reference complements larger k).
constexpr uint32_t binom_c(int n, int r)
{
	if (r < 0 || n < r) return 0;
	uint32_t c = 1;
	for (int i = 1; i <= r; i++) c = c * (uint32_t)(n - r + i) / (uint32_t)i;
	return c;
}
struct EnumSplit {
	uint16_t lo[256];
	uint16_t hi[9][256];
};
constexpr EnumSplit make_enum_split()
{
	EnumSplit e{};
	{
		for (int b = 0; b < 256; b++) {
			uint32_t c = 0;
			int r = 0;
			for (int n = 0; n < 8; n++)
				if ((b >> n) & 1) { c += binom_c(n, r + 1); r++; }
			e.lo[b] = (uint16_t)c;
			for (int klo = 0; klo <= 8; klo++) {
				uint32_t ch = 0;
				int rr = klo;
				for (int n = 0; n < 8; n++)
					if ((b >> n) & 1) { ch += binom_c(n + 8, rr + 1); rr++; }
				e.hi[klo][b] = rr <= 8 ? (uint16_t)ch : 0;
			}
		}
	}
	return e;
}

RIC_HD void enum16_split(const EnumSplit& E, const SymTables& T, uint32_t bits, uint32_t k, uint32_t& code_out,
                         uint32_t& len_out)
{
	if (k > 8) { k = 16 - k; bits ^= 0xFFFFu; }
	const uint32_t lo = bits & 255u;
	const uint32_t code = (uint32_t)E.lo[lo] + E.hi[popc32(lo)][bits >> 8];
	const uint32_t lost = T.cnk_lost[15][k - 1], len = T.cnk_len[15][k - 1];
	if (code < lost) { code_out = code; len_out = len - 1; }
	else { code_out = code + lost; len_out = len; }
}

// Scan position s of a band -> block (bx, by): serpentine rows, odd block rows
// right-to-left with the partial block first (bandcodec.cpp:509-523, 560-573).
RIC_HD void scan_block(int s, int dx, int dy, int& bx, int& by)
{
	const int bw = (dx + 3) >> 2, nfx = dx >> 2;
	by = s / bw;
	const int p = s - by * bw;
	if (!(by & 1)) bx = p;
	else if (nfx < bw) bx = p == 0 ? nfx : nfx - p;
	else bx = nfx - 1 - p;
}

RIC_HD uint32_t bitrev16(uint32_t m)
{
#if defined(__clang__)
	return __builtin_bitreverse32(m) >> 16;
#else
	uint32_t r = 0;
	for (int i = 0; i < 16; i++) r |= ((m >> i) & 1u) << (15 - i);
	return r;
#endif
}

// The block-local record of a full 4x4 block from its 16 final values (raster
// order, as the band holds them after buildTree: sign-magnitude, the INSIGNIF
// marker at [0] if insignificant).  block_enum's encoder side
// (bandcodec.cpp:346-403) with its raw bits precomputed.
// the record of a full block from its significance mask (bit i = raster
// position i) and whether its top-left holds the INSIGNIF marker
template <bool SPLIT>
RIC_HD uint64_t block_local_mask(const SymTables& T, const EnumSplit* E, uint32_t mask, bool insig, bool high)
{
	const uint64_t wh = ((uint64_t)3 << 53) | ((uint64_t)3 << 55);   // w = h = 4
	if (insig) return wh | (1ull << 47);
	const uint32_t k = popc32(mask);
	// enumCode wants the reference's bit order: first coefficient = MSB
	const uint32_t sig = bitrev16(mask);
	uint32_t raw = 0, rawlen = 0;
	if (SPLIT) {
		if (k != 0 && k != 16) enum16_split(*E, T, sig, k, raw, rawlen);
	} else if ((high || k != 0) && k != 16) {
		enum_bits(T, sig, k, 16, raw, rawlen);
	}
	const uint32_t gctx = k ? k - 1 : 0;
	return wh | mask | ((uint64_t)raw << 16) | ((uint64_t)rawlen << 32) | ((uint64_t)k << 37) | ((uint64_t)gctx << 49);
}
template <bool SPLIT>
RIC_HD uint64_t block_local_full_t(const SymTables& T, const EnumSplit* E, const int (&v)[16], bool high)
{
	uint32_t mask = 0;
	RIC_UNROLL
	for (int i = 0; i < 16; i++) mask |= (v[i] != 0 ? 1u : 0u) << i;
	return block_local_mask<SPLIT>(T, E, mask, v[0] == kInsignif, high);
}
RIC_HD uint64_t block_local_full(const SymTables& T, const int (&v)[16], bool high)
{
	return block_local_full_t<false>(T, nullptr, v, high);
}
RIC_HD uint64_t block_local_full(const SymTables& T, const EnumSplit& E, const int (&v)[16], bool high)
{
	return block_local_full_t<true>(T, &E, v, high);
}

// The block-local record of a partial (edge) block from its values held as
// v[4 * row + col], w x h valid: block_enum for edge blocks,
// bandcodec.cpp:405-478.
RIC_HD uint64_t block_local_edge(const SymTables& T, const int (&v)[16], int w, int h, bool high)
{
	uint64_t r = 0;
	const bool insig = v[0] == kInsignif;
	r |= (uint64_t)1 << 46;
	r |= (uint64_t)insig << 47;
	r |= (uint64_t)(w - 1) << 53;
	r |= (uint64_t)(h - 1) << 55;
	if (insig) return r;
	uint32_t mask = 0, sig = 0, k = 0;
	RIC_UNROLL
	for (int q = 0; q < 16; q++) {                 // raster order over the w x h corner
		const int j = q >> 2, i = q & 3;
		if (j >= h || i >= w) continue;
		sig <<= 1;
		if (v[q] != 0) { mask |= 1u << (j * w + i); sig |= 1; k++; }
	}
	const uint32_t cnt = (uint32_t)(w * h);
	uint32_t raw, rawlen;
	if (high) max_bits(k - 1, cnt - 1, raw, rawlen);
	else max_bits(k, cnt, raw, rawlen);
	if ((high || k != 0) && k != cnt) {
		uint32_t ec, el;
		enum_bits(T, sig, k, cnt, ec, el);
		raw = (raw << el) | ec;
		rawlen += el;
	}
	const uint32_t gctx = k ? T.kconv2[T.kconv1[cnt]][k - 1] : 0;
	r |= mask;
	r |= (uint64_t)raw << 16;
	r |= (uint64_t)rawlen << 32;
	r |= (uint64_t)k << 37;
	r |= (uint64_t)gctx << 49;
	return r;
}

// The block-local record of block (bx, by) of band `band` (type C, pitch st).
template <typename C>
RIC_HD uint64_t block_local(const SymTables& T, const C* band, long st, int dx, int dy, bool high, int bx, int by)
{
	const int x0 = bx * 4, y0 = by * 4;
	const int w = dx - x0 < 4 ? dx - x0 : 4, h = dy - y0 < 4 ? dy - y0 : 4;
	const C* blk = band + (long)y0 * st + x0;
	int v[16];
	RIC_UNROLL
	for (int i = 0; i < 16; i++) v[i] = ((i >> 2) < h && (i & 3) < w) ? (int)blk[(long)(i >> 2) * st + (i & 3)] : 0;
	if (w == 4 && h == 4) return block_local_full(T, v, high);
	return block_local_edge(T, v, w, h, high);
}

// maxLen<2, encode> (bandcodec.cpp:324-344) of a parent 2x2: max starts at 0,
// so the (negative) INSIGNIF marker never contributes.
template <bool PSH>
RIC_HD uint32_t pin_ctx_of(int a, int b, int c, int d)
{
	int mx = 0;
	mx = a > mx ? a : mx; mx = b > mx ? b : mx;
	mx = c > mx ? c : mx; mx = d > mx ? d : mx;
	return (uint32_t)bitlen(uc<PSH>(mx) >> 1) & 31;
}

// Parent info of block (bx, by) of a band whose parent band is `par` (type P).
// Facts used (encoder side of tree(), bandcodec.cpp:484-589):
//  * a full block is skipped ("propagated") iff the parent 4x4 block holding
//    (2*bx, 2*by) is a full block that buildTree left insignificant (tree()
//    copies that marker to all four anchors, :528-536); parent edge blocks
//    never set anchors;
//  * the tree context is maxLen of the parent 2x2 at (2*bx, 2*by).
template <typename P>
RIC_HD uint32_t parent_info(const P* par, long pst, int pdx, int pdy, int bx, int by)
{
	const int pbx = bx >> 1, pby = by >> 1;
	const bool pfull = pbx * 4 + 4 <= pdx && pby * 4 + 4 <= pdy;
	const bool prop = pfull && (int)par[(long)(pby * 4) * pst + pbx * 4] == kInsignif;
	const P* pp = par + (long)(by * 2) * pst + bx * 2;
	const uint32_t ctx = pin_ctx_of<sizeof(P) == 2>(pp[0], pp[1], pp[pst], pp[pst + 1]);
	return ctx | ((uint32_t)prop << 7);
}

#include "sym_tables.inc"
// host copy of the tables (the device copy lives in __constant__ memory, symbols.hip)
inline const SymTables& host_sym_tables()
{
	static const SymTables T = RIC_SYM_TABLES_INIT;
	return T;
}

}  // namespace ric
