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
#pragma once
#include <cstdint>
#include "ric_types.h"

namespace ric {

// record layout (u64)
//  [0,16)  significance mask, bit i = raster position i inside the block
//  [16,32) precomputed raw bits (enumCode; maxCode + enumCode for edge blocks)
//  [32,37) their length
//  [37,42) k = non-zero count
//  [42,46) tree context (full blocks)
//  46 edge, 47 insignificant, 48 propagated (skip)
//  [49,53) geometric-coder context of the block's coefficients
//  [53,55) edge width - 1, [55,57) edge height - 1
struct BlockRec {
	static RIC_HD uint32_t mask(uint64_t r) { return (uint32_t)(r & 0xFFFF); }
	static RIC_HD uint32_t raw(uint64_t r) { return (uint32_t)((r >> 16) & 0xFFFF); }
	static RIC_HD uint32_t rawlen(uint64_t r) { return (uint32_t)((r >> 32) & 31); }
	static RIC_HD uint32_t k(uint64_t r) { return (uint32_t)((r >> 37) & 31); }
	static RIC_HD uint32_t ctx(uint64_t r) { return (uint32_t)((r >> 42) & 15); }
	static RIC_HD bool edge(uint64_t r) { return (r >> 46) & 1; }
	static RIC_HD bool insig(uint64_t r) { return (r >> 47) & 1; }
	static RIC_HD bool prop(uint64_t r) { return (r >> 48) & 1; }
	static RIC_HD uint32_t gctx(uint64_t r) { return (uint32_t)((r >> 49) & 15); }
	static RIC_HD uint32_t w(uint64_t r) { return (uint32_t)((r >> 53) & 3) + 1; }
	static RIC_HD uint32_t h(uint64_t r) { return (uint32_t)((r >> 55) & 3) + 1; }
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

// The record of block (bx, by) of band `b` (element type C, pitch st), parent
// band `par` (type P) or null.
template <typename C, typename P>
RIC_HD uint64_t block_record(const SymTables& T, const C* band, long st, int dx, int dy,
                             const P* par, long pst, int pdx, int pdy, bool high, int bx, int by)
{
	constexpr bool SH = sizeof(C) == 2;
	const int x0 = bx * 4, y0 = by * 4;
	const int w = dx - x0 < 4 ? dx - x0 : 4, h = dy - y0 < 4 ? dy - y0 : 4;
	const bool edge = w < 4 || h < 4;
	const C* blk = band + (long)y0 * st + x0;
	uint64_t r = 0;
	uint32_t ctx = 15;
	if (!edge && par) {
		const int pbx = bx >> 1, pby = by >> 1;
		const bool pfull = pbx * 4 + 4 <= pdx && pby * 4 + 4 <= pdy;
		if (pfull && (int)par[(long)(pby * 4) * pst + pbx * 4] == kInsignif) return 1ull << 48;
		const P* pp = par + (long)(by * 2) * pst + bx * 2;
		int mx = 0;
		for (int j = 0; j < 2; j++)
			for (int i = 0; i < 2; i++) { int v = pp[j * pst + i]; mx = v > mx ? v : mx; }
		ctx = (uint32_t)bitlen(ucs(sizeof(P) == 2, mx) >> 1);
	}
	const bool insig = (int)blk[0] == kInsignif;
	r |= (uint64_t)ctx << 42;
	r |= (uint64_t)edge << 46;
	r |= (uint64_t)insig << 47;
	r |= (uint64_t)(w - 1) << 53;
	r |= (uint64_t)(h - 1) << 55;
	if (insig) return r;
	uint32_t mask = 0, sig = 0, k = 0;
	for (int j = 0; j < h; j++)
		for (int i = 0; i < w; i++) {
			const int v = blk[(long)j * st + i];
			sig <<= 1;
			if (v != 0) { mask |= 1u << (j * w + i); sig |= 1; k++; }
		}
	(void)SH;
	const uint32_t cnt = (uint32_t)(w * h);
	uint32_t raw = 0, rawlen = 0, gctx;
	if (!edge) {
		gctx = k ? k - 1 : 0;
		if ((high || k != 0) && k != 16) enum_bits(T, sig, k, 16, raw, rawlen);
	} else {
		uint32_t mc, ml;
		if (high) max_bits(k - 1, cnt - 1, mc, ml);
		else max_bits(k, cnt, mc, ml);
		raw = mc; rawlen = ml;
		if ((high || k != 0) && k != cnt) {
			uint32_t ec, el;
			enum_bits(T, sig, k, cnt, ec, el);
			raw = (raw << el) | ec;
			rawlen += el;
		}
		gctx = k ? T.kconv2[T.kconv1[cnt]][k - 1] : 0;
	}
	r |= mask;
	r |= (uint64_t)raw << 16;
	r |= (uint64_t)rawlen << 32;
	r |= (uint64_t)k << 37;
	r |= (uint64_t)gctx << 49;
	return r;
}

#include "sym_tables.inc"
// host copy of the tables (the device copy lives in __constant__ memory, symbols.hip)
inline const SymTables& host_sym_tables()
{
	static const SymTables T = RIC_SYM_TABLES_INIT;
	return T;
}

}  // namespace ric
