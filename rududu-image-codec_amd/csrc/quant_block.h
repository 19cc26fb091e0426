// quant_block.h -- the per-4x4-block RD quantiser of CBandCodec::buildTree
// (tsuqBlock, src/lib/bandcodec.cpp:159-237) on 16 coefficients held in
// registers, shared by the standalone quantiser (quant.hip k_quant_level) and
// the fused forward+quantiser (dwt.hip k_fwdq).
//
// The reference's stable insertion sort of the RD candidates followed by the
// suffix thresholding (bandcodec.cpp:115-127, 188-198) becomes a 16-key
// bitonic network on packed (key << 4 | 15 - index) words: a candidate
// survives iff its packed key is >= the smallest packed key whose sorted rank r
// fails `key < rd_thres[r + cnt]`.
#pragma once
#include <hip/hip_runtime.h>
#include "ric_types.h"

namespace ric {

template <bool SH>
__device__ __forceinline__ int quant_mag(int v, int iQ)
{
	// (tmp * iQuant + (1 << 15)) >> 16 with x86 wrap-around semantics
	int tmp = (int)(uc<SH>(v) >> 1);
	int q = (int)((uint32_t)tmp * (uint32_t)iQ + 32768u) >> 16;
	return tr<SH>((q << 1) | (v & 1));
}

__device__ __forceinline__ void sort16_desc(uint32_t (&s)[16])
{
#pragma unroll
	for (int k = 2; k <= 16; k <<= 1) {
#pragma unroll
		for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
			for (int i = 0; i < 16; i++) {
				int l = i ^ j;
				if (l > i) {
					uint32_t a = s[i], b = s[l];
					bool desc = (i & k) == 0;
					uint32_t hi = a > b ? a : b, lo = a > b ? b : a;
					s[i] = desc ? hi : lo;
					s[l] = desc ? lo : hi;
				}
			}
		}
	}
}

// tsuqBlock (RD), src/lib/bandcodec.cpp:159-213, on a full block v[16]
// (raster order).  thres = the band's rd_thres[16] (makeThres).  Leaves the
// quantised sign-magnitude values in v and returns the non-zero count.
// Branch-free: every lane runs the same instruction stream (selects, no
// divergent regions), so the 16 values stay in place in registers.
template <bool SH>
__device__ __forceinline__ int tsuq_full(int (&v)[16], int Q, int iQ, const int* thres)
{
	const int T0 = tr<SH>(Q >> 1);
	const uint32_t th0 = uc<SH>(thres[0]);
	int cnt = 0, ncand = 0;
	uint32_t key[16];
#pragma unroll
	for (int i = 0; i < 16; i++) {
		const int x = v[i];
		const bool dz = (uint32_t)(x + T0) <= (uint32_t)(2 * T0);     // dead zone
		const int u = tr<SH>(s2u_(x));
		const uint32_t uu = uc<SH>(u);
		const bool cand = !dz && uu < th0;                             // RD candidate
		key[i] = cand ? ((uu << 4) | (uint32_t)(15 - i)) : 0u;
		v[i] = dz ? 0 : (cand ? u : quant_mag<SH>(u, iQ));
		cnt += (!dz && !cand) ? 1 : 0;
		ncand += cand ? 1 : 0;
	}
	// no RD candidate in any active lane of the wave: no survivor, v and the
	// count stay as they are (same skip as tsuq_full_pk)
	if (__builtin_amdgcn_ballot_w64(ncand != 0) == 0) return cnt;
	uint32_t s[16];
#pragma unroll
	for (int i = 0; i < 16; i++) s[i] = key[i];
	sort16_desc(s);
	// the smallest sorted key whose rank r still passes (bandcodec.cpp:188-198)
	int ti[16];
	const int* tc = thres + cnt;           // cnt + r <= 15 wherever r < ncand
#pragma unroll
	for (int r = 0; r < 16; r++) ti[r] = tc[r];
	uint32_t thr = 0xFFFFFFFFu;
#pragma unroll
	for (int r = 0; r < 16; r++) {
		const int kv = tr<SH>((int)(s[r] >> 4));
		thr = (r < ncand && !(kv < ti[r])) ? s[r] : thr;
	}
	int surv = 0;
#pragma unroll
	for (int i = 0; i < 16; i++) {
		const bool keep = key[i] != 0 && key[i] >= thr;
		v[i] = key[i] == 0 ? v[i] : (keep ? tr<SH>(2 | (v[i] & 1)) : 0);
		surv += keep ? 1 : 0;
	}
	return cnt + surv;
}

// edge tsuqBlock, src/lib/bandcodec.cpp:215-237: the w x h top-left corner of
// v (row stride 4), plain dead-zone rounding, no RD.  Returns the count.
template <bool SH>
__device__ __forceinline__ int tsuq_edge(int (&v)[16], int wdt, int hgt, int Q, int iQ)
{
	const int T0 = tr<SH>((Q + ((Q - (Q >> 2)) >> 1)) >> 1);
	int cnt = 0;
#pragma unroll
	for (int i = 0; i < 16; i++) {
		const bool in = (i >> 2) < hgt && (i & 3) < wdt;
		const int x = v[i];
		const bool dz = (uint32_t)(x + T0) <= (uint32_t)(2 * T0);
		const int q = quant_mag<SH>(tr<SH>(s2u_(x)), iQ);
		v[i] = !in ? x : (dz ? 0 : q);
		cnt += (in && !dz) ? 1 : 0;
	}
	return cnt;
}

}  // namespace ric

namespace ric {

// ------------------------------------------------- packed 16-bit variant
// tsuqBlock (RD) on a full block of a `short` band held as 8 packed words,
// w[2 * row + h] = (v[4 * row + 2h], v[4 * row + 2h + 1]), two coefficients
// per v_pk_* instruction.  Same result as tsuq_full<true> whenever every rd
// threshold of the band lies in [1, 4095] (host-checked, pk_ok()): then the
// sort keys (value << 4 | 15 - index) fit 16 bits below the 0xFFFF sentinel,
// and a zero key (no candidate) never passes a threshold.
//   tpk[c * 8 + p] = (thres[c + p], thres[c + p + 8]), 0xFFFF past the end,
//   for c = the lane's significant count before RD (0..16).
typedef short v2s __attribute__((ext_vector_type(2)));
typedef unsigned short v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2s as_v2(uint32_t u) { return __builtin_bit_cast(v2s, u); }
__device__ __forceinline__ uint32_t as_u32(v2s v) { return __builtin_bit_cast(uint32_t, v); }

__device__ __forceinline__ v2u as_v2u(uint32_t x) { return __builtin_bit_cast(v2u, x); }
__device__ __forceinline__ uint32_t as_w(v2u x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ v2u splat2(uint32_t x) { return as_v2u((x & 0xFFFFu) * 0x10001u); }
// Packed 16-bit primitives as single instructions.  Inline asm keeps the
// instruction combiner from rewriting a saturating-sub + min mask idiom into
// per-half compares and selects (three times the instructions).
__device__ __forceinline__ v2u pk_sub_sat(v2u a, v2u b) { return __builtin_elementwise_sub_sat(a, b); }
__device__ __forceinline__ v2u pk_add_sat(v2u a, v2u b) { return __builtin_elementwise_add_sat(a, b); }
// 0xFFFF in each half where a > b (unsigned).  One opaque block: written in C
// the combiner turns the saturating-sub / min / negate idiom into per-half
// compares and selects (twice the instructions).
__device__ __forceinline__ v2u gt_mask(v2u a, v2u b)
{
	uint32_t r;
	asm("v_pk_sub_u16 %0, %1, %2 clamp\n\t"
	    "v_pk_min_u16 %0, %0, 1 op_sel_hi:[1,0]\n\t"
	    "v_pk_sub_u16 %0, 0, %0"
	    : "=&v"(r) : "v"(as_w(a)), "v"(as_w(b)));
	return as_v2u(r);
}
// 0xFFFF in each half where x != 0
__device__ __forceinline__ v2u nzmask(v2u x)
{
	uint32_t r;
	asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]\n\t"
	    "v_pk_sub_u16 %0, 0, %0"
	    : "=&v"(r) : "v"(as_w(x)));
	return as_v2u(r);
}
__device__ __forceinline__ v2u rot16(v2u x) { return as_v2u(__builtin_amdgcn_alignbit(as_w(x), as_w(x), 16)); }
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b)   // (m & a) | (~m & b)
{
	uint32_t r;
	asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
	return r;
}

__device__ __forceinline__ void cas_d(v2u& a, v2u& b)      // descending, both halves
{
	const v2u mx = __builtin_elementwise_max(a, b), mn = __builtin_elementwise_min(a, b);
	a = mx; b = mn;
}

// bitonic sort (all comparators of a stage share one direction: the "flip"
// form), descending; element i lives in R[i & 7], half i >> 3
__device__ __forceinline__ void sort16_pk(v2u (&R)[8])
{
	// k = 2
	cas_d(R[0], R[1]); cas_d(R[2], R[3]); cas_d(R[4], R[5]); cas_d(R[6], R[7]);
	// k = 4: flip i^3, then i^1
	cas_d(R[0], R[3]); cas_d(R[1], R[2]); cas_d(R[4], R[7]); cas_d(R[5], R[6]);
	cas_d(R[0], R[1]); cas_d(R[2], R[3]); cas_d(R[4], R[5]); cas_d(R[6], R[7]);
	// k = 8: flip i^7, then i^2, i^1
	cas_d(R[0], R[7]); cas_d(R[1], R[6]); cas_d(R[2], R[5]); cas_d(R[3], R[4]);
	cas_d(R[0], R[2]); cas_d(R[1], R[3]); cas_d(R[4], R[6]); cas_d(R[5], R[7]);
	cas_d(R[0], R[1]); cas_d(R[2], R[3]); cas_d(R[4], R[5]); cas_d(R[6], R[7]);
	// k = 16: flip i^15 pairs lo(R[p]) with hi(R[p^7])
#pragma unroll
	for (int p = 0; p < 4; p++) {
		const int q = 7 - p;
		const v2u y = rot16(R[q]);
		const uint32_t mx = as_w(__builtin_elementwise_max(R[p], y)), mn = as_w(__builtin_elementwise_min(R[p], y));
		R[p] = as_v2u(__builtin_amdgcn_perm(mn, mx, 0x07060100u));   // (mx.lo, mn.hi)
		R[q] = as_v2u(__builtin_amdgcn_perm(mn, mx, 0x05040302u));   // (mx.hi, mn.lo)
	}
	// then i^4, i^2, i^1
	cas_d(R[0], R[4]); cas_d(R[1], R[5]); cas_d(R[2], R[6]); cas_d(R[3], R[7]);
	cas_d(R[0], R[2]); cas_d(R[1], R[3]); cas_d(R[4], R[6]); cas_d(R[5], R[7]);
	cas_d(R[0], R[1]); cas_d(R[2], R[3]); cas_d(R[4], R[5]); cas_d(R[6], R[7]);
}

// returns the non-zero count; w is replaced by the quantised block
__device__ __forceinline__ int tsuq_full_pk(uint32_t (&w)[8], int Q, int iQ, int th0, const uint32_t* tpk)
{
	const int T0 = (int)(int16_t)(Q >> 1);
	const v2u T0v = splat2((uint32_t)T0), th0v = splat2((uint32_t)th0), z = {0, 0};
	v2u accB = z;
	v2u key[8];
#pragma unroll
	for (int j = 0; j < 8; j++) {
		const v2s x = as_v2(w[j]);
		const v2u ax = as_v2u(as_u32(__builtin_elementwise_max(x, (v2s){0, 0} - x)));   // |x| (0x8000 for -32768)
		const v2u sg = as_v2u(w[j]) >> (v2u){15, 15};
		const v2u u = ax + ax + sg;                                                // s2u_, wrapped to short
		const v2u mnz = gt_mask(ax, T0v);                                          // outside the dead zone
		const v2u mlt = gt_mask(th0v, u);                                          // below rd_thres[0]
		// quant_mag: ((u >> 1) * iQ + 32768) >> 16, then (q << 1) | sign
		const uint32_t uw = as_w(u);
		const uint32_t qlo = __umul24((uw & 0xFFFFu) >> 1, (uint32_t)iQ) + 32768u;
		const uint32_t qhi = __umul24(uw >> 17, (uint32_t)iQ) + 32768u;
		const v2u q = as_v2u(__builtin_amdgcn_perm(qhi, qlo, 0x07060302u));
		const v2u qv = q + q + sg;
		w[j] = bfi(as_w(mlt), as_w(u), as_w(qv)) & as_w(mnz);                       // 0 / candidate u / quantised
		const v2u idx = {(unsigned short)(15 - 2 * j), (unsigned short)(14 - 2 * j)};
		key[j] = as_v2u(as_w(u * (v2u){16, 16} + idx) & as_w(mnz & mlt));           // 0 unless RD candidate
		accB = accB - as_v2u(as_w(mnz) & ~as_w(mlt));                              // + 1 per quantised value
	}
	const uint32_t cnt = (uint32_t)accB.x + accB.y;
	// no RD candidate in any active lane of the wave (smooth areas): nothing
	// to sort, no survivor -- the result below would leave w and the count as
	// they are
	uint32_t anyk = 0;
#pragma unroll
	for (int j = 0; j < 8; j++) anyk |= as_w(key[j]);
	if (__builtin_amdgcn_ballot_w64(anyk != 0) == 0) return (int)cnt;
	// sort layout: R[p] = (key p, key p + 8)
	v2u R[8];
#pragma unroll
	for (int j = 0; j < 4; j++) {
		R[2 * j] = as_v2u(__builtin_amdgcn_perm(as_w(key[j + 4]), as_w(key[j]), 0x05040100u));
		R[2 * j + 1] = as_v2u(__builtin_amdgcn_perm(as_w(key[j + 4]), as_w(key[j]), 0x07060302u));
	}
	sort16_pk(R);
	// thr = the smallest sorted key s_r with (s_r >> 4) >= thres[r + cnt]
	// (the last passing rank, bandcodec.cpp:188-198); zero keys never pass
	const uint32_t* tc = tpk + cnt * 8;
	v2u t = {0xFFFF, 0xFFFF};
#pragma unroll
	for (int p = 0; p < 8; p++) {
		const v2u pen = gt_mask(as_v2u(tc[p]), R[p] >> (v2u){4, 4});
		t = __builtin_elementwise_min(t, pk_add_sat(R[p], pen));
	}
	t = __builtin_elementwise_min(t, rot16(t));                               // both halves = thr
	v2u accS = z;
#pragma unroll
	for (int j = 0; j < 8; j++) {
		const v2u keep = ~gt_mask(t, key[j]);                 // key >= thr (never for key 0)
		const uint32_t nv = as_w(keep) & ((w[j] & 0x00010001u) | 0x00020002u);  // survivor: magnitude 1
		w[j] = bfi(as_w(nzmask(key[j])), nv, w[j]);
		accS = accS - keep;
	}
	return (int)(cnt + accS.x + accS.y);
}

// host-side check that a band's thresholds qualify for tsuq_full_pk
inline bool pk_ok(const int* thres)
{
	for (int i = 0; i < 16; i++)
		if (thres[i] < 1 || thres[i] > 4095) return false;
	return true;
}

}  // namespace ric
