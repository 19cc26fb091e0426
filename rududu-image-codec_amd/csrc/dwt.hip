// dwt.hip -- forward / inverse integer lifting wavelet, one pyramid level per
// launch, hand-written for gfx950 (wave64).
//
// Restates CWavelet2D::Transform97/53/Haar and their inverses
// (src/lib/wavelet2d.cpp:320-855) as a streaming kernel:
//   * one wave owns a 256-column strip (4 adjacent columns per lane, 8-byte
//     loads/stores for s16) and a segment of S output rows;
//   * every input row is row-lifted in registers, the +-1 neighbours coming
//     from the adjacent lanes (__shfl_up/__shfl_down);
//   * the column lifting runs as a rolling row window in registers -- the
//     reference's own 6-row window (src/lib/wavelet2d.cpp:410-454) vectorised
//     over 4 columns per lane and 64 lanes;
//   * strips overlap by 4 columns (one halo lane per side), segments by 4 rows,
//     so every wave is independent (no LDS, no barriers).
// Band types follow the reference: `short` levels truncate at every store
// (tr<SH>), the int level does not.  The boundary formulas are the reference's
// start/tail cases (symmetric extension).
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <mutex>
#include <type_traits>
#include "ric_types.h"
#include "ric_kernels.h"
#include "quant_block.h"
#include "symbols.h"

namespace ric {

namespace {

constexpr int kLanes = 64;
constexpr int kCols = 4;                          // columns per lane
constexpr int kStripValid = (kLanes - 2) * kCols; // 248 valid output columns per wave
constexpr int kWavesPerBlock = 4;

// Bounds-checked loads are branch-free -- clamped addresses, then a select:
// a divergent vector-or-scalar branch makes the compiler drain every load at
// the join, one memory round trip per row.
// (the empty asm pins the load: otherwise it is sunk back under the condition)
__device__ __forceinline__ int pinned(int v) { asm("" : "+v"(v)); return v; }

template <typename T>
__device__ __forceinline__ void load4(const T* __restrict__ row, int x, int W, bool vec, int (&c)[4])
{
	(void)vec;
	int v[4];
#pragma unroll
	for (int j = 0; j < 4; j++) v[j] = (int)row[min(max(x + j, 0), W - 1)];
	asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));   // one wait for the four loads
#pragma unroll
	for (int j = 0; j < 4; j++) c[j] = (x + j >= 0 && x + j < W) ? v[j] : 0;
}

// store two consecutive band values (band columns bx, bx+1), bounded by dx
template <typename T>
__device__ __forceinline__ void store2(T* __restrict__ row, int bx, int dx, int a, int b)
{
	if (bx + 1 < dx) {
		if constexpr (sizeof(T) == 2) {
			*reinterpret_cast<uint32_t*>(row + bx) = (uint32_t)(uint16_t)a | ((uint32_t)(uint16_t)b << 16);
		} else {
			*reinterpret_cast<int2*>(row + bx) = make_int2(a, b);
		}
	} else if (bx < dx) {
		row[bx] = (T)a;
	}
}

template <typename T>
__device__ __forceinline__ void load2(const T* __restrict__ row, int bx, int dx, int& a, int& b)
{
	const int hi = dx > 0 ? dx - 1 : 0;
	int v0 = (int)row[min(max(bx, 0), hi)], v1 = (int)row[min(max(bx + 1, 0), hi)];
	asm volatile("" : "+v"(v0), "+v"(v1));   // one wait for both loads
	a = (bx >= 0 && bx < dx) ? v0 : 0;
	b = (bx + 1 >= 0 && bx + 1 < dx) ? v1 : 0;
}

// a register copy the compiler cannot fold away
__device__ __forceinline__ uint4 opaque_copy(const uint4& v)
{
	uint4 r;
	asm volatile("v_mov_b32 %0, %1" : "=v"(r.x) : "v"(v.x));
	asm volatile("v_mov_b32 %0, %1" : "=v"(r.y) : "v"(v.y));
	asm volatile("v_mov_b32 %0, %1" : "=v"(r.z) : "v"(v.z));
	asm volatile("v_mov_b32 %0, %1" : "=v"(r.w) : "v"(v.w));
	return r;
}

// Neighbour exchange across lanes with DPP wave shifts (GFX9 wave_shr:1 /
// wave_shl:1): one VALU op instead of an LDS-crossbar ds_bpermute.  Lane 0
// (resp. 63) has no source and reads 0; those are halo lanes.
__device__ __forceinline__ int from_left(int v)   // lane i <- lane i-1
{
	return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ int from_right(int v)  // lane i <- lane i+1
{
	return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xF, 0xF, true);
}

// ------------------------------------------------------------------ rows
// TransLine97, src/lib/wavelet2d.cpp:320-359, on 4 columns per lane.
// x = absolute column of c[0] (multiple of 4).
template <bool SH, bool EDGE>
__device__ __forceinline__ void row_fwd97(int (&c)[4], int x, int W)
{
	int t, lm, rn;
	lm = from_left(c[3]);                                    // P1 (even)
	if (EDGE && x == 0) c[0] = tr<SH>(c[0] - c[1] * 3);
	else if (EDGE && x == W - 1) c[0] = tr<SH>(c[0] - lm * 3);
	else { t = tr<SH>(lm + c[1]); c[0] = tr<SH>(c[0] - (t + (t >> 1))); }
	if (EDGE && x + 2 == W - 1) c[2] = tr<SH>(c[2] - c[1] * 3);
	else { t = tr<SH>(c[1] + c[3]); c[2] = tr<SH>(c[2] - (t + (t >> 1))); }
	rn = from_right(c[0]);                                  // U1 (odd)
	if (EDGE && x + 1 == W - 1) c[1] = tr<SH>(c[1] - (c[0] >> 3));
	else c[1] = tr<SH>(c[1] - ((c[0] + c[2]) >> 4));
	if (EDGE && x + 3 == W - 1) c[3] = tr<SH>(c[3] - (c[2] >> 3));
	else c[3] = tr<SH>(c[3] - ((c[2] + rn) >> 4));
	lm = from_left(c[3]);                                    // P2 (even)
	if (EDGE && x == 0) c[0] = tr<SH>(c[0] + 2 * mult08<SH>(c[1]));
	else if (EDGE && x == W - 1) c[0] = tr<SH>(c[0] + 2 * mult08<SH>(lm));
	else c[0] = tr<SH>(c[0] + mult08<SH>(lm + c[1]));
	if (EDGE && x + 2 == W - 1) c[2] = tr<SH>(c[2] + 2 * mult08<SH>(c[1]));
	else c[2] = tr<SH>(c[2] + mult08<SH>(c[1] + c[3]));
	rn = from_right(c[0]);                                  // U2 (odd)
	if (EDGE && x + 1 == W - 1) c[1] = tr<SH>(c[1] + (c[0] - (c[0] >> 4)));
	else { t = tr<SH>(c[0] + c[2]); c[1] = tr<SH>(c[1] + ((t >> 1) - (t >> 5))); }
	if (EDGE && x + 3 == W - 1) c[3] = tr<SH>(c[3] + (c[2] - (c[2] >> 4)));
	else { t = tr<SH>(c[2] + rn); c[3] = tr<SH>(c[3] + ((t >> 1) - (t >> 5))); }
}

// TransLine97I, src/lib/wavelet2d.cpp:361-405
template <bool SH, bool EDGE>
__device__ __forceinline__ void row_inv97(int (&c)[4], int x, int W)
{
	int t, lm, rn;
	rn = from_right(c[0]);                                  // U2^-1 (odd)
	if (EDGE && x + 1 == W - 1) c[1] = tr<SH>(c[1] - (c[0] - (c[0] >> 4)));
	else { t = tr<SH>(c[0] + c[2]); c[1] = tr<SH>(c[1] - ((t >> 1) - (t >> 5))); }
	if (EDGE && x + 3 == W - 1) c[3] = tr<SH>(c[3] - (c[2] - (c[2] >> 4)));
	else { t = tr<SH>(c[2] + rn); c[3] = tr<SH>(c[3] - ((t >> 1) - (t >> 5))); }
	lm = from_left(c[3]);                                    // P2^-1 (even)
	if (EDGE && x == 0) c[0] = tr<SH>(c[0] - 2 * mult08<SH>(c[1]));
	else if (EDGE && x == W - 1) c[0] = tr<SH>(c[0] - 2 * mult08<SH>(lm));
	else c[0] = tr<SH>(c[0] - mult08<SH>(lm + c[1]));
	if (EDGE && x + 2 == W - 1) c[2] = tr<SH>(c[2] - 2 * mult08<SH>(c[1]));
	else c[2] = tr<SH>(c[2] - mult08<SH>(c[1] + c[3]));
	rn = from_right(c[0]);                                  // U1^-1 (odd)
	if (EDGE && x + 1 == W - 1) c[1] = tr<SH>(c[1] + (c[0] >> 3));
	else c[1] = tr<SH>(c[1] + ((c[0] + c[2]) >> 4));
	if (EDGE && x + 3 == W - 1) c[3] = tr<SH>(c[3] + (c[2] >> 3));
	else c[3] = tr<SH>(c[3] + ((c[2] + rn) >> 4));
	lm = from_left(c[3]);                                    // P1^-1 (even)
	if (EDGE && x == 0) c[0] = tr<SH>(c[0] + c[1] * 3);
	else if (EDGE && x == W - 1) c[0] = tr<SH>(c[0] + lm * 3);
	else { t = tr<SH>(lm + c[1]); c[0] = tr<SH>(c[0] + (t + (t >> 1))); }
	if (EDGE && x + 2 == W - 1) c[2] = tr<SH>(c[2] + c[1] * 3);
	else { t = tr<SH>(c[1] + c[3]); c[2] = tr<SH>(c[2] + (t + (t >> 1))); }
}

// TransLine53, src/lib/wavelet2d.cpp:593-611
template <bool SH, bool EDGE>
__device__ __forceinline__ void row_fwd53(int (&c)[4], int x, int W)
{
	int lm = from_left(c[3]);                                // P (even)
	if (EDGE && x == 0) c[0] = tr<SH>(c[0] - c[1]);
	else if (EDGE && x == W - 1) c[0] = tr<SH>(c[0] - lm);
	else c[0] = tr<SH>(c[0] - ((lm + c[1]) >> 1));
	if (EDGE && x + 2 == W - 1) c[2] = tr<SH>(c[2] - c[1]);
	else c[2] = tr<SH>(c[2] - ((c[1] + c[3]) >> 1));
	int rn = from_right(c[0]);                              // U (odd)
	if (EDGE && x + 1 == W - 1) c[1] = tr<SH>(c[1] + (c[0] >> 1));
	else c[1] = tr<SH>(c[1] + ((c[0] + c[2]) >> 2));
	if (EDGE && x + 3 == W - 1) c[3] = tr<SH>(c[3] + (c[2] >> 1));
	else c[3] = tr<SH>(c[3] + ((c[2] + rn) >> 2));
}

// TransLine53I, src/lib/wavelet2d.cpp:613-634
template <bool SH, bool EDGE>
__device__ __forceinline__ void row_inv53(int (&c)[4], int x, int W)
{
	int rn = from_right(c[0]);                              // U^-1 (odd)
	if (EDGE && x + 1 == W - 1) c[1] = tr<SH>(c[1] - (c[0] >> 1));
	else c[1] = tr<SH>(c[1] - ((c[0] + c[2]) >> 2));
	if (EDGE && x + 3 == W - 1) c[3] = tr<SH>(c[3] - (c[2] >> 1));
	else c[3] = tr<SH>(c[3] - ((c[2] + rn) >> 2));
	int lm = from_left(c[3]);                                // P^-1 (even)
	if (EDGE && x == 0) c[0] = tr<SH>(c[0] + c[1]);
	else if (EDGE && x == W - 1) c[0] = tr<SH>(c[0] + lm);
	else c[0] = tr<SH>(c[0] + ((lm + c[1]) >> 1));
	if (EDGE && x + 2 == W - 1) c[2] = tr<SH>(c[2] + c[1]);
	else c[2] = tr<SH>(c[2] + ((c[1] + c[3]) >> 1));
}

// TransLineHaar(I), src/lib/wavelet2d.cpp:766-786 (an odd last column is untouched)
template <bool SH>
__device__ __forceinline__ void row_fwdhaar(int (&c)[4], int x, int W)
{
	if (x + 1 < W) { c[0] = tr<SH>(c[0] - c[1]); c[1] = tr<SH>(c[1] + (c[0] >> 1)); }
	if (x + 3 < W) { c[2] = tr<SH>(c[2] - c[3]); c[3] = tr<SH>(c[3] + (c[2] >> 1)); }
}
template <bool SH>
__device__ __forceinline__ void row_invhaar(int (&c)[4], int x, int W)
{
	if (x + 1 < W) { c[1] = tr<SH>(c[1] - (c[0] >> 1)); c[0] = tr<SH>(c[0] + c[1]); }
	if (x + 3 < W) { c[3] = tr<SH>(c[3] - (c[2] >> 1)); c[2] = tr<SH>(c[2] + c[3]); }
}

template <int TRANS, bool SH, bool EDGE>
__device__ __forceinline__ void row_fwd(int (&c)[4], int x, int W)
{
	if constexpr (TRANS == CDF97) row_fwd97<SH, EDGE>(c, x, W);
	else if constexpr (TRANS == CDF53) row_fwd53<SH, EDGE>(c, x, W);
	else row_fwdhaar<SH>(c, x, W);
}
template <int TRANS, bool SH, bool EDGE>
__device__ __forceinline__ void row_inv(int (&c)[4], int x, int W)
{
	if constexpr (TRANS == CDF97) row_inv97<SH, EDGE>(c, x, W);
	else if constexpr (TRANS == CDF53) row_inv53<SH, EDGE>(c, x, W);
	else row_invhaar<SH>(c, x, W);
}

#define FOR4 _Pragma("unroll") for (int j = 0; j < 4; j++)

// ------------------------------------------------------- row I/O helpers
template <typename T> struct Raw4;
template <> struct Raw4<int16_t> { using type = uint2; };   // 4 x s16
template <> struct Raw4<int32_t> { using type = int4; };    // 4 x i32
template <typename T> struct Raw2;
template <> struct Raw2<int16_t> { using type = uint32_t; }; // 2 x s16
template <> struct Raw2<int32_t> { using type = int2; };     // 2 x i32

template <typename T>
__device__ __forceinline__ typename Raw4<T>::type pack4(const int (&c)[4])
{
	if constexpr (sizeof(T) == 2) {
		return make_uint2((uint32_t)(uint16_t)c[0] | ((uint32_t)c[1] << 16),
		                  (uint32_t)(uint16_t)c[2] | ((uint32_t)c[3] << 16));
	} else {
		return make_int4(c[0], c[1], c[2], c[3]);
	}
}
template <typename T>
__device__ __forceinline__ void unpack4(const typename Raw4<T>::type& r, int (&c)[4])
{
	if constexpr (sizeof(T) == 2) {
		c[0] = (int16_t)(r.x & 0xffff); c[1] = (int)r.x >> 16;
		c[2] = (int16_t)(r.y & 0xffff); c[3] = (int)r.y >> 16;
	} else {
		c[0] = r.x; c[1] = r.y; c[2] = r.z; c[3] = r.w;
	}
}
template <typename T>
__device__ __forceinline__ void unpack2(const typename Raw2<T>::type& r, int& a, int& b)
{
	if constexpr (sizeof(T) == 2) { a = (int16_t)(r & 0xffff); b = (int)r >> 16; }
	else { a = r.x; b = r.y; }
}

// columns x..x+3 of one row; CHK = bounds/alignment-checked element loads
template <typename T, bool CHK>
__device__ __forceinline__ typename Raw4<T>::type load_row4(const T* __restrict__ row, int x, int W, bool vec)
{
	if constexpr (!CHK) {
		return *reinterpret_cast<const typename Raw4<T>::type*>(row + x);
	} else {
		int c[4];
		load4(row, x, W, vec, c);
		return pack4<T>(c);
	}
}
// band columns bx, bx+1; CHK = bounded by dx (and bx >= 0)
template <typename T, bool CHK>
__device__ __forceinline__ typename Raw2<T>::type load_band2(const T* __restrict__ row, int bx, int dx)
{
	if constexpr (!CHK) {
		return *reinterpret_cast<const typename Raw2<T>::type*>(row + bx);
	} else {
		int a, b;
		load2(row, bx, dx, a, b);
		if constexpr (sizeof(T) == 2) return (uint32_t)(uint16_t)a | ((uint32_t)b << 16);
		else return make_int2(a, b);
	}
}
template <typename T, bool CHK>
__device__ __forceinline__ void store_band2(T* __restrict__ row, int bx, int dx, int a, int b)
{
	if constexpr (!CHK) {
		if constexpr (sizeof(T) == 2)
			*reinterpret_cast<uint32_t*>(row + bx) = (uint32_t)(uint16_t)a | ((uint32_t)b << 16);
		else
			*reinterpret_cast<int2*>(row + bx) = make_int2(a, b);
	} else {
		store2(row, bx, dx, a, b);
	}
}

// Segment height: waves own S output rows plus 4 halo rows each side, all
// loaded up front (S + 8 rows in registers), so a wave pays one memory
// latency instead of one per row pair.

// ------------------------------------------------ packed s16 9/7 lifting
// `short` levels of the 9/7 transform compute in packed 16-bit lanes
// (v_pk_* ops): every reference store to a `short` is a wrap to 16 bits, so
// mod-2^16 arithmetic is exact; the one step whose sum the reference keeps in
// `int` before shifting (U1, `(a + b) >> 4`) uses an exact halving add.
// A lane's 4 columns x..x+3 are held as E = (x, x+2) and O = (x+1, x+3), so
// both the row steps (neighbours via one DPP shift + one alignbit) and the
// column steps (elementwise between rows) are 2-wide, and the de-interleaved
// band words D/H/V/L are E/O of even/odd rows as they stand.
// v2s, as_v2, as_u32: quant_block.h
// (a & m) | (b & ~m): per-16-bit-half select
__device__ __forceinline__ v2s sel(uint32_t m, v2s a, v2s b) { return as_v2((as_u32(a) & m) | (as_u32(b) & ~m)); }
// (lm, c1): the odd left neighbours of E = (c0, c2); lm = left lane's c3
__device__ __forceinline__ v2s left_odd(v2s o)
{
	return as_v2(__builtin_amdgcn_alignbit(as_u32(o), (uint32_t)from_left((int)as_u32(o)), 16));
}
// (c2, rn): the even right neighbours of O = (c1, c3); rn = right lane's c0
__device__ __forceinline__ v2s right_even(v2s e)
{
	return as_v2(__builtin_amdgcn_alignbit((uint32_t)from_right((int)as_u32(e)), as_u32(e), 16));
}
// floor((a + b) / 16) of two shorts, exactly (the sum may need 17 bits)
__device__ __forceinline__ v2s avg16(v2s a, v2s b)
{
	v2s h = (a >> 1) + (b >> 1) + as_v2(as_u32(a) & as_u32(b) & 0x00010001u);
	return h >> 3;
}
__device__ __forceinline__ v2s mult08p(v2s a)     // CWavelet2D::mult08 on short
{
	a = a - (a >> 2);
	a = a + (a >> 4);
	return a + (a >> 8);
}
// CWavelet2D::mult08 on a SUM: the template deduces C = int (mult08(i[1] +
// i[3]), src/lib/wavelet2d.cpp:336, 344, 353, 372, 381, 443, 548, ...), so the
// sum keeps its 17th bit and the steps run in int; only mult08 of a single
// element runs on short.  mult08p of the 16-bit wrapped sum s' = s - 65536 w
// is exact in 16 bits (no step wraps for |s'| <= 32768) and equals the int
// result minus 52428 w (every step divides the wrap exactly: 65536 / 4,
// 49152 / 16, 52224 / 256), so a wrapped add is corrected by +-52428.
__device__ __forceinline__ v2s mult08x(v2s a, v2s b)
{
	const v2s s = a + b;
	const uint32_t ov = ~(as_u32(a) ^ as_u32(b)) & (as_u32(a) ^ as_u32(s));   // sign bits: the add wrapped
	const v2s m = as_v2(ov) >> 15;                                          // -1 where it did
	const v2s sg = a >> 15;                                                  // -1: wrapped downwards
	const v2s c = (as_v2(0xCCCCCCCCu) ^ sg) - sg;                            // +52428 / -52428 (mod 2^16)
	return mult08p(s) + as_v2(as_u32(c) & as_u32(m));
}
// X: the exact form; !X: the plain 16-bit sum, for a level whose input range
// keeps every such sum within 16 bits (level 0 of 8-bit pixels: |x| <= 2048
// bounds the argument by 12902, the l1 norm of its linear map times 2048)
template <bool X> __device__ __forceinline__ v2s m08s(v2s a, v2s b) { return X ? mult08x(a, b) : mult08p(a + b); }
__device__ __forceinline__ v2s mul3(v2s a) { return a + a + a; }

// per-lane boundary masks (16-bit halves) for the row steps
struct EdgeMasks {
	uint32_t eL;     // even element without a left neighbour (column 0)
	uint32_t eR;     // even element without a right neighbour (column W-1 even)
	uint32_t oR;     // odd element without a right neighbour (column W-1 odd)
	uint32_t eAny;
};
__device__ __forceinline__ EdgeMasks edge_masks(int x, int W)
{
	EdgeMasks m;
	m.eL = x == 0 ? 0x0000ffffu : 0u;
	m.eR = (x == W - 1 ? 0x0000ffffu : 0u) | (x + 2 == W - 1 ? 0xffff0000u : 0u);
	m.oR = (x + 1 == W - 1 ? 0x0000ffffu : 0u) | (x + 3 == W - 1 ? 0xffff0000u : 0u);
	m.eAny = m.eL | m.eR;
	return m;
}

struct PRow { v2s e, o; };

__device__ __forceinline__ PRow prow_from_u2(uint2 u)
{
	PRow r;
	r.e = as_v2(__builtin_amdgcn_perm(u.y, u.x, 0x05040100u));   // (c0, c2)
	r.o = as_v2(__builtin_amdgcn_perm(u.y, u.x, 0x07060302u));   // (c1, c3)
	return r;
}
__device__ __forceinline__ uint2 prow_to_u2(const PRow& r)
{
	const uint32_t e = as_u32(r.e), o = as_u32(r.o);
	return make_uint2(__builtin_amdgcn_perm(o, e, 0x05040100u),   // (c0, c1)
	                  __builtin_amdgcn_perm(o, e, 0x07060302u));  // (c2, c3)
}

// TransLine97 (src/lib/wavelet2d.cpp:320-359) on packed columns
template <bool EDGE>
__device__ __forceinline__ void row_fwd97p(PRow& r, const EdgeMasks& m)
{
	v2s E = r.e, O = r.o;
	v2s OL = left_odd(O);                                   // P1 (even)
	v2s t = OL + O;
	v2s s = t + (t >> 1);
	if (EDGE) s = sel(m.eAny, mul3(sel(m.eL, O, OL)), s);
	E = E - s;
	v2s ER = right_even(E);                                 // U1 (odd)
	v2s a = avg16(E, ER);
	if (EDGE) a = sel(m.oR, E >> 3, a);
	O = O - a;
	OL = left_odd(O);                                       // P2 (even)
	v2s mm = mult08x(OL, O);
	if (EDGE) { v2s me = mult08p(sel(m.eL, O, OL)); mm = sel(m.eAny, me + me, mm); }
	E = E + mm;
	ER = right_even(E);                                     // U2 (odd)
	t = E + ER;
	v2s d = (t >> 1) - (t >> 5);
	if (EDGE) d = sel(m.oR, E - (E >> 4), d);
	O = O + d;
	r.e = E; r.o = O;
}

// TransLine97I (src/lib/wavelet2d.cpp:361-405) on packed columns
template <bool EDGE>
__device__ __forceinline__ void row_inv97p(PRow& r, const EdgeMasks& m)
{
	v2s E = r.e, O = r.o;
	v2s ER = right_even(E);                                 // U2^-1 (odd)
	v2s t = E + ER;
	v2s d = (t >> 1) - (t >> 5);
	if (EDGE) d = sel(m.oR, E - (E >> 4), d);
	O = O - d;
	v2s OL = left_odd(O);                                   // P2^-1 (even)
	v2s mm = mult08x(OL, O);
	if (EDGE) { v2s me = mult08p(sel(m.eL, O, OL)); mm = sel(m.eAny, me + me, mm); }
	E = E - mm;
	ER = right_even(E);                                     // U1^-1 (odd)
	v2s a = avg16(E, ER);
	if (EDGE) a = sel(m.oR, E >> 3, a);
	O = O + a;
	OL = left_odd(O);                                       // P1^-1 (even)
	t = OL + O;
	v2s s = t + (t >> 1);
	if (EDGE) s = sel(m.eAny, mul3(sel(m.eL, O, OL)), s);
	E = E + s;
	r.e = E; r.o = O;
}

// Two independent rows (the pair e, e+1) stepped together, statement by
// statement, so every dependent packed op has an independent neighbour to
// issue against (the schedule alone does not interleave them).
template <bool EDGE>
__device__ __forceinline__ void row_fwd97p2(PRow& r, PRow& q, const EdgeMasks& m)
{
	v2s E = r.e, O = r.o, F = q.e, P = q.o;
	v2s OL = left_odd(O), PL = left_odd(P);                 // P1 (even)
	v2s t = OL + O, u = PL + P;
	v2s s = t + (t >> 1), s2 = u + (u >> 1);
	if (EDGE) { s = sel(m.eAny, mul3(sel(m.eL, O, OL)), s); s2 = sel(m.eAny, mul3(sel(m.eL, P, PL)), s2); }
	E = E - s; F = F - s2;
	v2s ER = right_even(E), FR = right_even(F);             // U1 (odd)
	v2s a = avg16(E, ER), b = avg16(F, FR);
	if (EDGE) { a = sel(m.oR, E >> 3, a); b = sel(m.oR, F >> 3, b); }
	O = O - a; P = P - b;
	OL = left_odd(O); PL = left_odd(P);                     // P2 (even)
	v2s mm = mult08x(OL, O), mm2 = mult08x(PL, P);
	if (EDGE) {
		v2s me = mult08p(sel(m.eL, O, OL)), me2 = mult08p(sel(m.eL, P, PL));
		mm = sel(m.eAny, me + me, mm); mm2 = sel(m.eAny, me2 + me2, mm2);
	}
	E = E + mm; F = F + mm2;
	ER = right_even(E); FR = right_even(F);                 // U2 (odd)
	t = E + ER; u = F + FR;
	v2s d = (t >> 1) - (t >> 5), d2 = (u >> 1) - (u >> 5);
	if (EDGE) { d = sel(m.oR, E - (E >> 4), d); d2 = sel(m.oR, F - (F >> 4), d2); }
	O = O + d; P = P + d2;
	r.e = E; r.o = O; q.e = F; q.o = P;
}

template <bool EDGE>
__device__ __forceinline__ void row_inv97p2(PRow& r, PRow& q, const EdgeMasks& m)
{
	v2s E = r.e, O = r.o, F = q.e, P = q.o;
	v2s ER = right_even(E), FR = right_even(F);             // U2^-1 (odd)
	v2s t = E + ER, u = F + FR;
	v2s d = (t >> 1) - (t >> 5), d2 = (u >> 1) - (u >> 5);
	if (EDGE) { d = sel(m.oR, E - (E >> 4), d); d2 = sel(m.oR, F - (F >> 4), d2); }
	O = O - d; P = P - d2;
	v2s OL = left_odd(O), PL = left_odd(P);                 // P2^-1 (even)
	v2s mm = mult08x(OL, O), mm2 = mult08x(PL, P);
	if (EDGE) {
		v2s me = mult08p(sel(m.eL, O, OL)), me2 = mult08p(sel(m.eL, P, PL));
		mm = sel(m.eAny, me + me, mm); mm2 = sel(m.eAny, me2 + me2, mm2);
	}
	E = E - mm; F = F - mm2;
	ER = right_even(E); FR = right_even(F);                 // U1^-1 (odd)
	v2s a = avg16(E, ER), b = avg16(F, FR);
	if (EDGE) { a = sel(m.oR, E >> 3, a); b = sel(m.oR, F >> 3, b); }
	O = O + a; P = P + b;
	OL = left_odd(O); PL = left_odd(P);                     // P1^-1 (even)
	t = OL + O; u = PL + P;
	v2s s = t + (t >> 1), s2 = u + (u >> 1);
	if (EDGE) { s = sel(m.eAny, mul3(sel(m.eL, O, OL)), s); s2 = sel(m.eAny, mul3(sel(m.eL, P, PL)), s2); }
	E = E + s; F = F + s2;
	r.e = E; r.o = O; q.e = F; q.o = P;
}

// ---------------------------------------------------------- forward level
template <typename TI, typename TO>
struct FwdArgs {
	const TI* src; long sp;   // input plane + pitch (elements)
	int W, H;
	TO* d[4]; long p[4];      // D, H, V, L outputs + pitches
	int nseg, vec, nofast;
};

// One wave: columns x..x+3 per lane of a 256-column strip, output rows
// [y0, y0+S).  FAST = interior strip of an aligned plane and a segment whose
// halo rows are all inside the image: no boundary formula and no bounds check
// can apply, so every condition below folds at compile time.
template <int TRANS, typename TI, typename TO, int S, bool FAST>
__device__ __forceinline__ void fwd_seg(const FwdArgs<TI, TO>& a, int x, int lane, int y0)
{
	constexpr bool SH = sizeof(TO) == 2;
	constexpr bool EDGE = !FAST;
	const int W = a.W, H = a.H;
	const bool out_lane = lane >= 1 && lane <= kLanes - 2 && (FAST || x < W);
	const int bx = x >> 1;
	auto emit = [&](int y, const int (&r)[4]) {
		if (!FAST && (y < y0 || y >= y0 + S || y >= H)) return;
		if (!out_lane) return;
		const int by = y >> 1;
		if (!(y & 1)) {
			store_band2<TO, EDGE>(a.d[BD] + (long)by * a.p[BD], bx, (W + 1) >> 1, r[0], r[2]);
			store_band2<TO, EDGE>(a.d[BH] + (long)by * a.p[BH], bx, W >> 1, r[1], r[3]);
		} else {
			store_band2<TO, EDGE>(a.d[BV] + (long)by * a.p[BV], bx, (W + 1) >> 1, r[0], r[2]);
			store_band2<TO, EDGE>(a.d[BL] + (long)by * a.p[BL], bx, W >> 1, r[1], r[3]);
		}
	};

	if constexpr (TRANS == HAAR) {
		// TransformHaar, src/lib/wavelet2d.cpp:788-819: complete row pairs only
		for (int e = y0; e < y0 + S && e + 1 < H; e += 2) {
			int r0[4], r1[4];
			unpack4<TI>(load_row4<TI, true>(a.src + (long)e * a.sp, x, W, a.vec != 0), r0);
			unpack4<TI>(load_row4<TI, true>(a.src + (long)(e + 1) * a.sp, x, W, a.vec != 0), r1);
			FOR4 { r0[j] = tr<SH>(r0[j]); r1[j] = tr<SH>(r1[j]); }
			row_fwd<TRANS, SH, true>(r0, x, W);
			row_fwd<TRANS, SH, true>(r1, x, W);
			FOR4 { r0[j] = tr<SH>(r0[j] - r1[j]); r1[j] = tr<SH>(r1[j] + (r0[j] >> 1)); }
			emit(e, r0); emit(e + 1, r1);
		}
	} else {
		constexpr int R = S + 8;                 // input rows y0-4 .. y0+S+3
		using RT = typename Raw4<TI>::type;
		RT raw[R];
		if constexpr (FAST) {
#pragma unroll
			for (int i = 0; i < R; i++) raw[i] = load_row4<TI, false>(a.src + (long)(y0 - 4 + i) * a.sp, x, W, a.vec != 0);
		} else {
			// batches of 16 rows: every element of the batch (clamped row and
			// columns) is loaded before one pin per 4 rows, then the rows and
			// columns outside the image are zeroed -- one memory round trip per
			// batch (a pin or a select right after each load waits for it)
			const int xc[4] = {min(max(x, 0), W - 1), min(max(x + 1, 0), W - 1), min(max(x + 2, 0), W - 1),
			                   min(max(x + 3, 0), W - 1)};
			constexpr int RB = 16;
#pragma unroll
			for (int i0 = 0; i0 < R; i0 += RB) {
				int ev[RB][4];
#pragma unroll
				for (int i = 0; i < RB; i++) {
					if (i0 + i >= R) break;
					const TI* row = a.src + (long)min(max(y0 - 4 + i0 + i, 0), H - 1) * a.sp;
#pragma unroll
					for (int j = 0; j < 4; j++) ev[i][j] = (int)row[xc[j]];
				}
#pragma unroll
				for (int i = 0; i < RB; i += 4) {
					if (i0 + i >= R) break;
					asm volatile("" : "+v"(ev[i][0]), "+v"(ev[i][1]), "+v"(ev[i][2]), "+v"(ev[i][3]),
					                  "+v"(ev[i + 1][0]), "+v"(ev[i + 1][1]), "+v"(ev[i + 1][2]), "+v"(ev[i + 1][3]),
					                  "+v"(ev[i + 2][0]), "+v"(ev[i + 2][1]), "+v"(ev[i + 2][2]), "+v"(ev[i + 2][3]),
					                  "+v"(ev[i + 3][0]), "+v"(ev[i + 3][1]), "+v"(ev[i + 3][2]), "+v"(ev[i + 3][3]));
				}
#pragma unroll
				for (int i = 0; i < RB; i++) {
					if (i0 + i >= R) break;
					const int y = y0 - 4 + i0 + i;
					const bool in = y >= 0 && y < H;
					int c[4];
#pragma unroll
					for (int j = 0; j < 4; j++) c[j] = in && x + j >= 0 && x + j < W ? ev[i][j] : 0;
					raw[i0 + i] = pack4<TI>(c);
				}
			}
		}
		int w0[4] = {0, 0, 0, 0}, w1[4] = {0, 0, 0, 0}, w2[4] = {0, 0, 0, 0};
		int w3[4] = {0, 0, 0, 0}, w4[4], w5[4] = {0, 0, 0, 0};
#pragma unroll
		for (int i = 0; i < R; i += 2) {
			const int e = y0 - 4 + i;            // the window's newest even row
			if (!FAST && (e < 0 || e >= H)) continue;
			unpack4<TI>(raw[i], w4);
			FOR4 w4[j] = tr<SH>(w4[j]);
			row_fwd<TRANS, SH, EDGE>(w4, x, W);
			if (FAST || e + 1 < H) {
				unpack4<TI>(raw[i + 1], w5);
				FOR4 w5[j] = tr<SH>(w5[j]);
				row_fwd<TRANS, SH, EDGE>(w5, x, W);
			}
			if constexpr (TRANS == CDF97) {
				// P1 at e, U1 at e-1, P2 at e-2, U2 at e-3 (src/lib/wavelet2d.cpp:425-454)
				if (!FAST && e == 0) { FOR4 w4[j] = tr<SH>(w4[j] - w5[j] * 3); }
				else if (!FAST && e == H - 1) { FOR4 w4[j] = tr<SH>(w4[j] - w3[j] * 3); }
				else { FOR4 { int t = tr<SH>(w3[j] + w5[j]); w4[j] = tr<SH>(w4[j] - (t + (t >> 1))); } }
				if (FAST || e >= 1) { FOR4 w3[j] = tr<SH>(w3[j] - ((w2[j] + w4[j]) >> 4)); }
				if (!FAST && e == 2) { FOR4 w2[j] = tr<SH>(w2[j] + 2 * mult08<SH>(w3[j])); }
				else if (FAST || e >= 4) { FOR4 w2[j] = tr<SH>(w2[j] + mult08<false>(w1[j] + w3[j])); }
				if (FAST || e >= 4) { FOR4 { int t = tr<SH>(w0[j] + w2[j]); w1[j] = tr<SH>(w1[j] + ((t >> 1) - (t >> 5))); } }
			} else {
				// P at e, U at e-1 (src/lib/wavelet2d.cpp:654-668)
				if (!FAST && e == 0) { FOR4 w4[j] = tr<SH>(w4[j] - w5[j]); }
				else if (!FAST && e == H - 1) { FOR4 w4[j] = tr<SH>(w4[j] - w3[j]); }
				else { FOR4 w4[j] = tr<SH>(w4[j] - ((w3[j] + w5[j]) >> 1)); }
				if (FAST || e >= 1) { FOR4 w3[j] = tr<SH>(w3[j] + ((w2[j] + w4[j]) >> 2)); }
			}
			if (!FAST || i >= 8) { emit(e - 4, w0); emit(e - 3, w1); }
			FOR4 { w0[j] = w2[j]; w1[j] = w3[j]; w2[j] = w4[j]; w3[j] = w5[j]; }
		}
		if (!FAST && y0 + S + 4 >= H) {
			// window now holds rows e-2 .. e+1 of the last pair e
			if (!(H & 1)) {
				if constexpr (TRANS == CDF97) {      // src/lib/wavelet2d.cpp:476-491
					FOR4 w3[j] = tr<SH>(w3[j] - (w2[j] >> 3));
					FOR4 w2[j] = tr<SH>(w2[j] + mult08<false>(w1[j] + w3[j]));
					FOR4 { int t = tr<SH>(w0[j] + w2[j]); w1[j] = tr<SH>(w1[j] + ((t >> 1) - (t >> 5))); }
					FOR4 w3[j] = tr<SH>(w3[j] + (w2[j] - (w2[j] >> 4)));
				} else {                              // src/lib/wavelet2d.cpp:685-691
					FOR4 w3[j] = tr<SH>(w3[j] + (w2[j] >> 1));
				}
				emit(H - 4, w0); emit(H - 3, w1); emit(H - 2, w2); emit(H - 1, w3);
			} else {
				if constexpr (TRANS == CDF97) {      // src/lib/wavelet2d.cpp:456-475
					FOR4 w2[j] = tr<SH>(w2[j] + 2 * mult08<SH>(w1[j]));
					FOR4 { int t = tr<SH>(w0[j] + w2[j]); w1[j] = tr<SH>(w1[j] + ((t >> 1) - (t >> 5))); }
				}
				emit(H - 3, w0); emit(H - 2, w1); emit(H - 1, w2);
			}
		}
	}
}

// Forward 9/7 level, short -> short, packed (same schedule as fwd_seg).
template <int S, bool FAST>
__device__ __forceinline__ void fwd97p_seg(const FwdArgs<int16_t, int16_t>& a, int x, int lane, int y0)
{
	constexpr bool EDGE = !FAST;
	const int W = a.W, H = a.H;
	const EdgeMasks m = edge_masks(x, W);
	const bool out_lane = lane >= 1 && lane <= kLanes - 2 && (FAST || x < W);
	const int bx = x >> 1;
	const int dxE = (W + 1) >> 1, dxO = W >> 1;
	auto st2 = [&](int16_t* row, int dx, v2s v) {
		const uint32_t u = as_u32(v);
		if (FAST || bx + 1 < dx) *reinterpret_cast<uint32_t*>(row + bx) = u;
		else if (bx < dx) row[bx] = (int16_t)(u & 0xffff);
	};
	auto emit = [&](int y, const PRow& r) {
		if (!FAST && (y < y0 || y >= y0 + S || y >= H)) return;
		if (!out_lane) return;
		const long by = y >> 1;
		if (!(y & 1)) { st2(a.d[BD] + by * a.p[BD], dxE, r.e); st2(a.d[BH] + by * a.p[BH], dxO, r.o); }
		else { st2(a.d[BV] + by * a.p[BV], dxE, r.e); st2(a.d[BL] + by * a.p[BL], dxO, r.o); }
	};
	// FAST: the output band rows advance by one pitch per row pair
	int16_t* pD = a.d[BD] + (long)(y0 >> 1) * a.p[BD];
	int16_t* pH = a.d[BH] + (long)(y0 >> 1) * a.p[BH];
	int16_t* pV = a.d[BV] + (long)(y0 >> 1) * a.p[BV];
	int16_t* pL = a.d[BL] + (long)(y0 >> 1) * a.p[BL];
	auto emit_pair = [&](const PRow& r0, const PRow& r1) {
		if (out_lane) {
			*reinterpret_cast<uint32_t*>(pD + bx) = as_u32(r0.e);
			*reinterpret_cast<uint32_t*>(pH + bx) = as_u32(r0.o);
			*reinterpret_cast<uint32_t*>(pV + bx) = as_u32(r1.e);
			*reinterpret_cast<uint32_t*>(pL + bx) = as_u32(r1.o);
		}
		pD += a.p[BD]; pH += a.p[BH]; pV += a.p[BV]; pL += a.p[BL];
	};
	// Input rows y0-4 .. y0+S+3 stream through a ring of 2*PF registers:
	// the loads of pair p+PF are issued before pair p is lifted, and the loop
	// body (PF pairs) stays small enough to live in the instruction cache.
	// (S = 2, k_fwdq_gen: the 5 pairs in one pass)
	constexpr int NP = (S + 8) / 2, PF = NP % 4 == 0 ? 4 : NP;
	// Border waves: a slot holds the raw elements of clamped columns of a
	// clamped row, loaded unconditionally and masked when the slot is taken (a
	// select or a pin right after a load is waited for at once: one memory
	// round trip per element).  Rows outside the image are never consumed:
	// pairs with e < 0 or e >= H are skipped, and row e + 1 >= H is unused.
	struct FRaw { int c0, c1, c2, c3; };
	using Slot = typename std::conditional<FAST, uint2, FRaw>::type;
	Slot ring[2 * PF];
	const int16_t* rp = a.src + (long)(y0 - 4) * a.sp;   // wave-uniform row pointer
	int yl = y0 - 4;
	const int xc0 = min(max(x, 0), W - 1), xc1 = min(max(x + 1, 0), W - 1);
	const int xc2 = min(max(x + 2, 0), W - 1), xc3 = min(max(x + 3, 0), W - 1);
	const uint32_t cm0 = (x >= 0 && x < W ? 0xFFFFu : 0u) | (x + 1 >= 0 && x + 1 < W ? 0xFFFF0000u : 0u);
	const uint32_t cm1 = (x + 2 >= 0 && x + 2 < W ? 0xFFFFu : 0u) | (x + 3 >= 0 && x + 3 < W ? 0xFFFF0000u : 0u);
	auto load_next = [&](Slot& dst) {
		if constexpr (FAST) {
			dst = load_row4<int16_t, false>(rp, x, W, true);
		} else {
			const int16_t* r = a.src + (long)min(max(yl, 0), H - 1) * a.sp;
			dst.c0 = r[xc0]; dst.c1 = r[xc1]; dst.c2 = r[xc2]; dst.c3 = r[xc3];
		}
		rp += a.sp; yl++;
	};
	auto take = [&](const Slot& r) -> PRow {
		if constexpr (FAST) {
			return prow_from_u2(r);
		} else {
			return prow_from_u2(make_uint2(((uint32_t)(uint16_t)r.c0 | ((uint32_t)r.c1 << 16)) & cm0,
			                               ((uint32_t)(uint16_t)r.c2 | ((uint32_t)r.c3 << 16)) & cm1));
		}
	};
#pragma unroll
	for (int j = 0; j < 2 * PF; j++) load_next(ring[j]);
	const v2s z = {0, 0};
	PRow w0 = {z, z}, w1 = {z, z}, w2 = {z, z}, w3 = {z, z}, w4 = {z, z}, w5 = {z, z};
#pragma unroll 1
	for (int it = 0; it < NP / PF; it++) {
#pragma unroll
	for (int k = 0; k < PF; k++) {
		const int i = 2 * (it * PF + k);
		const int e = y0 - 4 + i;
		// unpack the slot first, so its registers are free for the refill
		// (a refill into fresh registers would need a copy at the back-edge,
		// and that copy waits for the load)
		const PRow n0 = take(ring[2 * k]), n1 = take(ring[2 * k + 1]);
		if (it + 1 < NP / PF) { load_next(ring[2 * k]); load_next(ring[2 * k + 1]); }
		if (!FAST && (e < 0 || e >= H)) continue;
		w4 = n0;
		if (FAST || e + 1 < H) { w5 = n1; row_fwd97p2<EDGE>(w4, w5, m); }
		else row_fwd97p<EDGE>(w4, m);
		// P1 at e, U1 at e-1, P2 at e-2, U2 at e-3 (src/lib/wavelet2d.cpp:425-454)
		if (!FAST && e == 0) { w4.e -= mul3(w5.e); w4.o -= mul3(w5.o); }
		else if (!FAST && e == H - 1) { w4.e -= mul3(w3.e); w4.o -= mul3(w3.o); }
		else {
			v2s te = w3.e + w5.e, to = w3.o + w5.o;
			w4.e -= te + (te >> 1); w4.o -= to + (to >> 1);
		}
		if (FAST || e >= 1) { w3.e -= avg16(w2.e, w4.e); w3.o -= avg16(w2.o, w4.o); }
		if (!FAST && e == 2) {
			v2s me = mult08p(w3.e), mo = mult08p(w3.o);
			w2.e += me + me; w2.o += mo + mo;
		} else if (FAST || e >= 4) {
			w2.e += mult08x(w1.e, w3.e); w2.o += mult08x(w1.o, w3.o);
		}
		if (FAST || e >= 4) {
			v2s te = w0.e + w2.e, to = w0.o + w2.o;
			w1.e += (te >> 1) - (te >> 5); w1.o += (to >> 1) - (to >> 5);
		}
		if (FAST) { if (i >= 8) emit_pair(w0, w1); }
		else { emit(e - 4, w0); emit(e - 3, w1); }
		w0 = w2; w1 = w3; w2 = w4; w3 = w5;
	}
	}
	if (!FAST && y0 + S + 4 >= H) {
		if (!(H & 1)) {                              // src/lib/wavelet2d.cpp:476-491
			w3.e -= w2.e >> 3; w3.o -= w2.o >> 3;
			w2.e += mult08x(w1.e, w3.e); w2.o += mult08x(w1.o, w3.o);
			v2s te = w0.e + w2.e, to = w0.o + w2.o;
			w1.e += (te >> 1) - (te >> 5); w1.o += (to >> 1) - (to >> 5);
			w3.e += w2.e - (w2.e >> 4); w3.o += w2.o - (w2.o >> 4);
			emit(H - 4, w0); emit(H - 3, w1); emit(H - 2, w2); emit(H - 1, w3);
		} else {                                     // src/lib/wavelet2d.cpp:456-475
			v2s me = mult08p(w1.e), mo = mult08p(w1.o);
			w2.e += me + me; w2.o += mo + mo;
			v2s te = w0.e + w2.e, to = w0.o + w2.o;
			w1.e += (te >> 1) - (te >> 5); w1.o += (to >> 1) - (to >> 5);
			emit(H - 3, w0); emit(H - 2, w1); emit(H - 1, w2);
		}
	}
}

template <int TRANS, typename TI, typename TO, int S>
__global__ void __launch_bounds__(256) k_fwd(FwdArgs<TI, TO> a)
{
	const int lane = threadIdx.x & 63;
	const int seg = blockIdx.y * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: row math stays scalar
	if (seg >= a.nseg) return;                       // whole wave exits together
	const int X0 = blockIdx.x * kStripValid - kCols;
	const int x = X0 + lane * kCols;
	const int y0 = seg * S;
	// column W-1 inside the wave (halo lanes included) needs the boundary formulas
	const bool edge = X0 < 0 || X0 + kLanes * kCols >= a.W;
	const bool fast = !edge && a.vec && !a.nofast && y0 >= 16 && y0 + S + 4 < a.H;
	if constexpr (TRANS == CDF97 && sizeof(TI) == 2 && sizeof(TO) == 2) {
		if (fast) fwd97p_seg<S, true>(a, x, lane, y0);
		else fwd97p_seg<S, false>(a, x, lane, y0);
	} else {
		if (fast) fwd_seg<TRANS, TI, TO, S, true>(a, x, lane, y0);
		else fwd_seg<TRANS, TI, TO, S, false>(a, x, lane, y0);
	}
}

// ------------------------------------------- fused forward level + quantiser
// k_fwdq: one 9/7 short->short forward level fused with the band's whole
// device-side CodeBand work, so the unquantised bands never go back to HBM:
//   * CWavelet2D::Transform97 of the level (src/lib/wavelet2d.cpp:407-492);
//   * CBandCodec::buildTree's tsuqBlock + pRD + INSIGNIF marker on every 4x4
//     block of D, H, V (src/lib/bandcodec.cpp:159-319; the children's pRD are
//     the finer level's, already final because levels run finest first);
//   * the block-local zerotree record of every block, and the parent info of
//     the FINER level's blocks, whose parent this level is (symbols.h).
// The LL band (next level's input) is written unquantised.
//
// Geometry: one wave owns a 512-column strip (8 columns per lane, 16-byte
// row loads; lanes 0 and 63 are halo, so 496 output columns = 62 blocks of
// every band, one block column per lane) and a segment of S input rows
// (S/8 block rows).  Interior waves ("fast") keep everything in registers:
// the packed 16-bit lifting of fwd97p_seg on 8 columns (4 packed words per
// row), a 4-band-row buffer per band, and the quantiser on the buffer once a
// block row is complete.  Waves touching an image border ("edge") run the
// checked 4-column lifting (fwd97p_seg<S, false>) over their two 248-column
// halves, then quantise their own blocks from the just-written bands (the
// blocks of one lane were written by lanes of the same wave: a workgroup-scope
// fence orders it).
constexpr int kFqStrip = (kLanes - 2) * 8;   // 496 output columns per wave


// format tables staged in LDS once per workgroup
struct FqTables {
	SymTables T;
	EnumSplit E;
};

struct FqArgs {
	const int16_t* src; long sp;
	int W, H, nseg, vec8, vec16, nofast, high;
	int16_t* d[4]; long p[4];          // D, H, V, L
	int dx[3], dy[3], bw[3], bh[3];
	uint32_t* rd[3];                   // this level's pRD (raster, stride bw)
	const uint32_t* crd[3]; int cbw[3];   // the finer level's pRD, or null
	uint64_t* rec[3];                  // this level's block-local records
	uint8_t* cpin[3]; int cpw[3], cph[3];  // the finer level's parent info, or null
	int Q[3], iQ[3];
	int thres[3][16];
	uint64_t* wgt;                     // diagnostics: per-workgroup timestamps (dbg 128), or null
	int pk;                            // k_fwdq_gen: short bands whose thresholds pass pk_ok
	int level;
	int* err;                          // device error word (ring hand-off timeout), or null
	int fault;                         // fault injection (ric_diag_fault): force a ring timeout
	int in8;                           // the level's input is 8-bit pixels (|x| <= 2048): plain 16-bit mult08 sums
};

struct PRow8 { v2s q[4]; };            // (c0,c2) (c4,c6) | (c1,c3) (c5,c7)

__device__ __forceinline__ PRow8 prow8_from(const uint4& u)
{
	PRow8 r;
	r.q[0] = as_v2(__builtin_amdgcn_perm(u.y, u.x, 0x05040100u));
	r.q[2] = as_v2(__builtin_amdgcn_perm(u.y, u.x, 0x07060302u));
	r.q[1] = as_v2(__builtin_amdgcn_perm(u.w, u.z, 0x05040100u));
	r.q[3] = as_v2(__builtin_amdgcn_perm(u.w, u.z, 0x07060302u));
	return r;
}
// The same row from 8 u8 pixels (a gray frame's level 0, k_fwdq_pc_z<.., U8>):
// the ric level shift of k_gray_in8 applied on the way, (p - 128) << sh
// (src/ric/ric.cpp:144-148: sh 4 lossy, 0 lossless), so the coding plane is
// never written or read.  u.x = pixels c3 c2 c1 c0 (c0 the low byte).
__device__ __forceinline__ PRow8 prow8_from_u8(const uint2& u, int sh)
{
	PRow8 r;
	const v2s b = {128, 128}, s = {(short)sh, (short)sh};
	r.q[0] = (as_v2(__builtin_amdgcn_perm(0u, u.x, 0x0c020c00u)) - b) << s;
	r.q[2] = (as_v2(__builtin_amdgcn_perm(0u, u.x, 0x0c030c01u)) - b) << s;
	r.q[1] = (as_v2(__builtin_amdgcn_perm(0u, u.y, 0x0c020c00u)) - b) << s;
	r.q[3] = (as_v2(__builtin_amdgcn_perm(0u, u.y, 0x0c030c01u)) - b) << s;
	return r;
}
// a gray batch's u8 pixels for level 0 (kernel argument: one pointer per frame)
constexpr int kPixZ = 32;
struct PixSrc {
	const uint8_t* p[kPixZ];
	long sp;                           // bytes per row
	int sh;                            // the level shift
};
// the odd left neighbours of the evens: (lm, c1), (c3, c5)
__device__ __forceinline__ void left_odd8(const PRow8& r, v2s& l0, v2s& l1)
{
	l0 = as_v2(__builtin_amdgcn_alignbit(as_u32(r.q[2]), (uint32_t)from_left((int)as_u32(r.q[3])), 16));
	l1 = as_v2(__builtin_amdgcn_alignbit(as_u32(r.q[3]), as_u32(r.q[2]), 16));
}
// the even right neighbours of the odds: (c2, c4), (c6, rn)
__device__ __forceinline__ void right_even8(const PRow8& r, v2s& r0, v2s& r1)
{
	r0 = as_v2(__builtin_amdgcn_alignbit(as_u32(r.q[1]), as_u32(r.q[0]), 16));
	r1 = as_v2(__builtin_amdgcn_alignbit((uint32_t)from_right((int)as_u32(r.q[0])), as_u32(r.q[1]), 16));
}

// TransLine97 (src/lib/wavelet2d.cpp:320-359) on two interior rows at once
template <bool X>
__device__ __forceinline__ void row_fwd97p8x2(PRow8& r, PRow8& s)
{
	v2s a0, a1, b0, b1, t;
	left_odd8(r, a0, a1); left_odd8(s, b0, b1);                   // P1 (even)
	t = a0 + r.q[2]; r.q[0] -= t + (t >> 1);
	t = b0 + s.q[2]; s.q[0] -= t + (t >> 1);
	t = a1 + r.q[3]; r.q[1] -= t + (t >> 1);
	t = b1 + s.q[3]; s.q[1] -= t + (t >> 1);
	right_even8(r, a0, a1); right_even8(s, b0, b1);               // U1 (odd)
	r.q[2] -= avg16(r.q[0], a0); s.q[2] -= avg16(s.q[0], b0);
	r.q[3] -= avg16(r.q[1], a1); s.q[3] -= avg16(s.q[1], b1);
	left_odd8(r, a0, a1); left_odd8(s, b0, b1);                   // P2 (even)
	r.q[0] += m08s<X>(a0, r.q[2]); s.q[0] += m08s<X>(b0, s.q[2]);
	r.q[1] += m08s<X>(a1, r.q[3]); s.q[1] += m08s<X>(b1, s.q[3]);
	right_even8(r, a0, a1); right_even8(s, b0, b1);               // U2 (odd)
	t = r.q[0] + a0; r.q[2] += (t >> 1) - (t >> 5);
	t = s.q[0] + b0; s.q[2] += (t >> 1) - (t >> 5);
	t = r.q[1] + a1; r.q[3] += (t >> 1) - (t >> 5);
	t = s.q[1] + b1; s.q[3] += (t >> 1) - (t >> 5);
}

// Children of block (kx, ky) at the finer level: their parent info from this
// block's final values (symbols.h parent_info, computed on the parent side).
__device__ __forceinline__ void fq_child_pin(const FqArgs& a, int b, const int (&v)[16], bool full, int kx, int ky)
{
	uint8_t* cp = a.cpin[b];
	if (!cp) return;
	const uint32_t prop = (full && v[0] == kInsignif) ? 0x80u : 0u;
#pragma unroll
	for (int q = 0; q < 4; q++) {
		const int qx = q & 1, qy = q >> 1;
		const int cx = 2 * kx + qx, cy = 2 * ky + qy;
		const int o = 8 * qy + 2 * qx;
		if (cx < a.cpw[b] && cy < a.cph[b])
			cp[(long)cy * a.cpw[b] + cx] = (uint8_t)(pin_ctx_of<true>(v[o], v[o + 1], v[o + 4], v[o + 5]) | prop);
	}
}

// children pRD sum exactly as k_quant_level (u32 sum, then widened)
__device__ __forceinline__ uint32_t fq_dist(const FqArgs& a, int b, int cnt, int kx, int ky)
{
	uint64_t d = (uint64_t)cnt;
	if (a.crd[b]) {
		const uint32_t* c0 = a.crd[b] + (long)(2 * ky) * a.cbw[b] + 2 * kx;
		const uint32_t* c1 = c0 + a.cbw[b];
		d += (uint32_t)(c0[0] + c0[1] + c1[0] + c1[1]);
	}
	return d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
}

// parent info of the 4 children of a full block held as packed words
__device__ __forceinline__ void fq_child_pin_pk(const FqArgs& a, int b, const uint32_t (&w)[8], bool insig, int kx, int ky)
{
	uint8_t* cp = a.cpin[b];
	if (!cp) return;
	const uint32_t prop = insig ? 0x80u : 0u;
#pragma unroll
	for (int q = 0; q < 4; q++) {
		const int qx = q & 1, qy = q >> 1;
		const int cx = 2 * kx + qx, cy = 2 * ky + qy;
		// maxLen<2> over the quadrant, max from 0 (markers are negative)
		const v2s m2 = __builtin_elementwise_max(__builtin_elementwise_max(as_v2(w[4 * qy + qx]), as_v2(w[4 * qy + 2 + qx])),
		                                         (v2s){0, 0});
		const int mx = m2.x > m2.y ? m2.x : m2.y;
		if (cx < a.cpw[b] && cy < a.cph[b])
			cp[(long)cy * a.cpw[b] + cx] = (uint8_t)(((uint32_t)bitlen((uint32_t)mx >> 1) & 31) | prop);
	}
}

// The children pRD of block (kx, ky), loaded ahead of the block (consumer
// waves prefetch the next block row's): unconditional loads at clamped
// addresses -- a level without children reads its own pRD array's first word
// -- masked by `on` when summed (u32 sum, then widened, as fq_dist).
struct FqCrd { uint32_t c[4]; bool on; };
__device__ __forceinline__ FqCrd fq_crd_load(const FqArgs& a, int b, int kx, int ky)
{
	FqCrd r;
	r.on = a.crd[b] != nullptr;
	const uint32_t* crd = r.on ? a.crd[b] : a.rd[b];
	const int cw = r.on ? a.cbw[b] : 1, ch = r.on ? a.cph[b] : 1;
	const int cy0 = min(max(2 * ky, 0), ch - 1), cy1 = min(max(2 * ky + 1, 0), ch - 1);
	const int cx0 = min(max(2 * kx, 0), cw - 1), cx1 = min(max(2 * kx + 1, 0), cw - 1);
	r.c[0] = crd[(long)cy0 * cw + cx0]; r.c[1] = crd[(long)cy0 * cw + cx1];
	r.c[2] = crd[(long)cy1 * cw + cx0]; r.c[3] = crd[(long)cy1 * cw + cx1];
	return r;
}
__device__ __forceinline__ uint32_t fq_dist_pre(int cnt, const FqCrd& cr)
{
	const uint64_t d = (uint64_t)cnt + (cr.on ? (uint32_t)(cr.c[0] + cr.c[1] + cr.c[2] + cr.c[3]) : 0u);
	return d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
}

// one full block from the register buffer (4 band rows of 4 shorts = 8
// packed words, row r = words 2r, 2r + 1); cr = its children's pRD
// (fq_crd_load), or null to load them here
__device__ __forceinline__ void fq_block_regs(const FqArgs& a, const int* thr, const uint32_t* tpk, const FqTables& F,
                                              int b, const uint2 (&buf)[4], int kx, int ky, bool out_lane,
                                              const FqCrd* cr = nullptr)
{
	uint32_t w[8];
#pragma unroll
	for (int r = 0; r < 4; r++) { w[2 * r] = buf[r].x; w[2 * r + 1] = buf[r].y; }
	const int cnt = tsuq_full_pk(w, a.Q[b], a.iQ[b], thr[0], tpk);   // levels are fused only when pk_ok
	const uint32_t dist = cr ? fq_dist_pre(cnt, *cr) : fq_dist(a, b, cnt, kx, ky);
	if (dist == 0) w[0] = (w[0] & 0xFFFF0000u) | 0x8000u;   // INSIGNIF_BLOCK
	if (!out_lane) return;
	const long pb = a.p[b];
	int16_t* base = a.d[b] + (long)(4 * ky) * pb + 4 * kx;
#pragma unroll
	for (int r = 0; r < 4; r++) *reinterpret_cast<uint2*>(base + r * pb) = make_uint2(w[2 * r], w[2 * r + 1]);
	const long bi = (long)ky * a.bw[b] + kx;
	a.rd[b][bi] = dist;
	// significance mask: bit i = coefficient i != 0
	uint32_t acc = 0;
#pragma unroll
	for (int j = 0; j < 8; j++) acc |= as_w(__builtin_elementwise_min(as_v2u(w[j]), (v2u){1, 1})) << (2 * j);
	const uint32_t mask = (acc & 0x5555u) | ((acc >> 15) & 0xAAAAu);
	const bool insig = (w[0] & 0xFFFFu) == 0x8000u;
	a.rec[b][bi] = block_local_mask<true>(F.T, &F.E, mask, insig, a.high != 0);
	fq_child_pin_pk(a, b, w, insig, kx, ky);
}

// Image-border flags of one wave (fq_seg<S, true>).  Needs W % 8 == 0 and
// H % 8 == 0: column W-1 is then the last odd column of some lane, and every
// block the wave quantises is full.
struct FqBorder {
	uint32_t eL0;      // 0x0000FFFF on the lane whose word q0 low half is column 0
	uint32_t oR3;      // 0xFFFF0000 on the lane whose word q3 high half is column W-1
	bool top;          // y0 == 0: rows above the image, boundary formulas at e == 0, 2
	bool bottom;       // y0 + S >= H: the segment ends at H, tail formulas after the loop
	bool ld;           // this lane's 8 columns lie inside the image (loads allowed)
};

// TransLine97 with the left/right boundary formulas (src/lib/wavelet2d.cpp:
// 326-358: x0 -= 3 x1 at column 0, 2 mult08 at column 0 for P2, the odd last
// column from its left neighbour only), two rows at once
template <bool X>
__device__ __forceinline__ void row_fwd97p8x2_edge(PRow8& r, PRow8& s, const FqBorder& m)
{
	v2s a0, a1, b0, b1, t, u;
	left_odd8(r, a0, a1); left_odd8(s, b0, b1);                   // P1 (even)
	t = a0 + r.q[2]; t = t + (t >> 1); r.q[0] -= sel(m.eL0, mul3(r.q[2]), t);
	u = b0 + s.q[2]; u = u + (u >> 1); s.q[0] -= sel(m.eL0, mul3(s.q[2]), u);
	t = a1 + r.q[3]; r.q[1] -= t + (t >> 1);
	u = b1 + s.q[3]; s.q[1] -= u + (u >> 1);
	right_even8(r, a0, a1); right_even8(s, b0, b1);               // U1 (odd)
	r.q[2] -= avg16(r.q[0], a0); s.q[2] -= avg16(s.q[0], b0);
	r.q[3] -= sel(m.oR3, r.q[1] >> 3, avg16(r.q[1], a1));
	s.q[3] -= sel(m.oR3, s.q[1] >> 3, avg16(s.q[1], b1));
	left_odd8(r, a0, a1); left_odd8(s, b0, b1);                   // P2 (even)
	t = mult08p(r.q[2]); r.q[0] += sel(m.eL0, t + t, m08s<X>(a0, r.q[2]));
	u = mult08p(s.q[2]); s.q[0] += sel(m.eL0, u + u, m08s<X>(b0, s.q[2]));
	r.q[1] += m08s<X>(a1, r.q[3]); s.q[1] += m08s<X>(b1, s.q[3]);
	right_even8(r, a0, a1); right_even8(s, b0, b1);               // U2 (odd)
	t = r.q[0] + a0; r.q[2] += (t >> 1) - (t >> 5);
	u = s.q[0] + b0; s.q[2] += (u >> 1) - (u >> 5);
	t = r.q[1] + a1; r.q[3] += sel(m.oR3, r.q[1] - (r.q[1] >> 4), (t >> 1) - (t >> 5));
	u = s.q[1] + b1; s.q[3] += sel(m.oR3, s.q[1] - (s.q[1] >> 4), (u >> 1) - (u >> 5));
}

// The per-iteration hand-off barrier of k_fwdq_pc.  Only LDS is shared
// between the producer and the consumers, so the barrier waits for the
// wave's LDS operations alone (lgkmcnt) -- __syncthreads() would also drain
// every outstanding global load and store (vmcnt(0) of its workgroup-scope
// fence), i.e. wait out the producer's row prefetch and everyone's band /
// record stores once per iteration.  gfx950's s_barrier does not wait for
// memory by itself; the "memory" clobber keeps the compiler from moving LDS
// accesses across it.  dbg 1024: the full __syncthreads() (comparison).
constexpr int kWgIt = 20;                 // diagnostics: traced barrier iterations per wave
constexpr int kWgRec = 8 + 4 * 2 * kWgIt; // u64 per workgroup record
// tr (diagnostics, dbg 128): arrival and departure realtime stamps
__device__ __forceinline__ void pc_barrier(int dbg, uint64_t* tr = nullptr)
{
	if (tr && threadIdx.x % 64 == 0) tr[0] = __builtin_amdgcn_s_memrealtime();
	if (dbg & 1024) __syncthreads();
	else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
	if (tr && threadIdx.x % 64 == 0) tr[1] = __builtin_amdgcn_s_memrealtime();
}

// Decoupled hand-off (k_fwdq_pc<true>): a ring of kRing block-row slots in
// LDS with counters instead of one workgroup barrier per block row, so the
// producer may run up to kRing block rows ahead of the slowest consumer and
// neither side waits for the other's slowest iteration.  ring[0] = block rows
// published by the producer, ring[1 + b] = block rows consumer b has taken.
// A publish first waits for the wave's own LDS writes (lgkmcnt(0)), so a
// consumer that reads the new count and then the slot sees the slot's data.
constexpr int kRing = 4;
__device__ __forceinline__ int ring_get(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void ring_put(int* p, int v)
{
	asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Bounded spin (~30 ms): a protocol error must never hang the GPU.  A wait
// that gives up raises the launch's device error word (FqArgs::err, the
// arena's status word), which the host reads at its next sync point and turns
// into RIC_E_HIP: the slot it would have taken is not trusted.  limit: polls
// (the fault-injection knob, ric_diag_fault, shortens it).
constexpr int kRingPolls = 1 << 20;
__device__ __forceinline__ void ring_wait_ge(int* p, int need, int* err, int limit = kRingPolls)
{
	int n = 0;
	for (; ring_get(p) < need && n < limit; n++) __builtin_amdgcn_s_sleep(1);
	if (n >= limit && err) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	asm volatile("" ::: "memory");
}

// One wave's segment: the forward 9/7 of rows [y0, y0 + S) of a 496-column
// strip and the quantiser, records and parent info of the block rows they
// make, all in registers.  EDGE: the wave touches an image border (m).
// PC (producer-consumer mode, k_fwdq_pc): this wave only lifts; each
// completed block row goes to the LDS double buffer `pcbuf` and every loop
// iteration ends in a workgroup barrier that the consumer waves match.
struct NoStage {
	__device__ void operator()() const {}
};

// stage(): called once the prologue row loads are in flight (k_fwdq_pc
// stages the format tables there, so their latency overlaps the loads')
// U8: the input rows are u8 pixels at src8 (sp8 bytes per row), level-shifted
// on load (prow8_from_u8)
template <bool EDGE, bool PC = false, bool X = true, typename Stage = NoStage, bool U8 = false>
__device__ __forceinline__ void fq_seg(const FqArgs& a, const int (*thr)[16], const uint32_t (*tpk)[17 * 8],
                                       const FqTables& F, int x, int lane, int y0, int kx, const FqBorder& m, int S,
                                       uint2 (*pcbuf)[3][4][kLanes] = nullptr, int dbg = 0, uint64_t* tr = nullptr,
                                       const Stage& stage = Stage(), int* hring = nullptr,
                                       const uint8_t* src8 = nullptr, long sp8 = 0, int sh8 = 0)
{
	const bool out_lane = lane >= 1 && lane <= kLanes - 2 && (!EDGE || x < a.W);
	int16_t* pL = a.d[BL] + (long)(y0 >> 1) * a.p[BL] + (x >> 1);
	// input rows y0-4 .. y0+S+3 through a ring of PF row pairs (fwd97p_seg);
	// PF = 4 pairs = one block row of output, so the buffer slot of an emitted
	// pair is the unrolled index k
	constexpr int PF = 4;
	// S (a multiple of 8) rows: S / 8 + 1 iterations of PF row pairs; bottom
	// segment: pairs e = y0-4 .. H-2 only, then the tail formulas
	const int nit = (EDGE && m.bottom) ? (a.H - y0) / 8 + 1 : S / 8 + 1;   // loop iterations
	const int kend = (EDGE && m.bottom) ? 2 : PF;                          // pairs of the last one
	// prefetch depth in loop iterations (8 rows each): the producer of the
	// PC form has the registers for two
	constexpr int DEPTH = PC ? 2 : 1;
	using RowRaw = typename std::conditional<U8, uint2, uint4>::type;
	RowRaw ring[DEPTH][2 * PF];
	int yl = y0 - 4;
	// Every row load is unconditional, from a wave-uniform clamped row (the
	// refills past the segment re-read its last row, an L2 hit): a load under
	// a branch, or a select on its value, makes the compiler wait for it at
	// once, and the prefetch ring would degrade to one memory round trip per
	// row.  Border waves clamp the column too and zero the lanes outside the
	// image when the row is consumed.
	const int ylast = min(y0 + S + 3, a.H - 1);
	const int xcl = EDGE ? min(max(x, 0), a.W - 8) : x;
	auto load_next = [&](RowRaw& dst) {
		const int yc = min(max(yl, 0), ylast);
		if constexpr (U8) dst = *reinterpret_cast<const uint2*>(src8 + (long)yc * sp8 + xcl);
		else dst = *reinterpret_cast<const uint4*>(a.src + (long)yc * a.sp + xcl);
		yl++;
	};
#pragma unroll
	for (int d = 0; d < DEPTH; d++) {
#pragma unroll
		for (int j = 0; j < 2 * PF; j++) load_next(ring[d][j]);
	}
	stage();
	const v2s z = {0, 0};
	PRow8 w0, w1, w2, w3, w4, w5;
#pragma unroll
	for (int q = 0; q < 4; q++) { w0.q[q] = z; w1.q[q] = z; w2.q[q] = z; w3.q[q] = z; }
	uint2 bD[4], bH[4], bV[4];
	int cur = 0;                                // PC: the LDS buffer being filled
	auto emit = [&](int k) {                    // rows e-4 (D, H) and e-3 (V, L) are final
		const uint2 vd = make_uint2(as_u32(w0.q[0]), as_u32(w0.q[1]));
		const uint2 vh = make_uint2(as_u32(w0.q[2]), as_u32(w0.q[3]));
		const uint2 vv = make_uint2(as_u32(w1.q[0]), as_u32(w1.q[1]));
		if constexpr (PC) {
			if (!(dbg & 16)) { pcbuf[cur][BD][k][lane] = vd; pcbuf[cur][BH][k][lane] = vh; pcbuf[cur][BV][k][lane] = vv; }
			else if (vd.x == 0x7FFF1234u) pcbuf[cur][BD][k][lane] = vh;   // (keep the values live)
		} else {
			bD[k] = vd; bH[k] = vh; bV[k] = vv;
		}
		if (out_lane && !(dbg & 16)) *reinterpret_cast<uint2*>(pL) = make_uint2(as_u32(w1.q[2]), as_u32(w1.q[3]));
		pL += a.p[BL];
	};
	auto quant_row = [&](int ky) {
		// one block at a time: the scheduler would otherwise interleave the
		// three independent quantisers and spill
		__builtin_amdgcn_sched_barrier(0);
		fq_block_regs(a, thr[BD], tpk[BD], F, BD, bD, kx, ky, out_lane);
		__builtin_amdgcn_sched_barrier(0);
		fq_block_regs(a, thr[BH], tpk[BH], F, BH, bH, kx, ky, out_lane);
		__builtin_amdgcn_sched_barrier(0);
		fq_block_regs(a, thr[BV], tpk[BV], F, BV, bV, kx, ky, out_lane);
		__builtin_amdgcn_sched_barrier(0);
	};
	auto iteration = [&](int it, RowRaw (&rg)[2 * PF]) {
		const bool last = it + 1 == nit;
		if (PC && hring) {
			// block row it - 1 goes to slot (it - 1) % kRing, free once every
			// consumer has taken block row it - 1 - kRing
			cur = (it - 1) & (kRing - 1);
			const int need = it - kRing;
			if (need > 0) {
				ring_wait_ge(hring + 1, need, a.err);
				ring_wait_ge(hring + 2, need, a.err);
				ring_wait_ge(hring + 3, need, a.err);
			}
		} else {
			cur = it & 1;
		}
#pragma unroll
		for (int k = 0; k < PF; k++) {
			if (EDGE && last && k >= kend) break;
			const int e = y0 - 4 + 2 * (it * PF + k);   // the pair's even row
			if constexpr (U8) {
				w4 = prow8_from_u8(rg[2 * k], sh8);
				w5 = prow8_from_u8(rg[2 * k + 1], sh8);
				if (EDGE && !m.ld) {
#pragma unroll
					for (int q = 0; q < 4; q++) { w4.q[q] = z; w5.q[q] = z; }
				}
			} else {
				uint4 u0 = rg[2 * k], u1 = rg[2 * k + 1];
				if (EDGE && !m.ld) { u0 = make_uint4(0, 0, 0, 0); u1 = u0; }
				w4 = prow8_from(u0);
				w5 = prow8_from(u1);
			}
			load_next(rg[2 * k]);
			load_next(rg[2 * k + 1]);
			if (EDGE && e < 0) continue;                 // above the image (top segment)
			if (EDGE) row_fwd97p8x2_edge<X>(w4, w5, m);
			else row_fwd97p8x2<X>(w4, w5);
			// P1 at e, U1 at e-1, P2 at e-2, U2 at e-3 (src/lib/wavelet2d.cpp:425-454)
			if (EDGE && e == 0) {
#pragma unroll
				for (int q = 0; q < 4; q++) w4.q[q] -= mul3(w5.q[q]);
			} else {
#pragma unroll
				for (int q = 0; q < 4; q++) { v2s t = w3.q[q] + w5.q[q]; w4.q[q] -= t + (t >> 1); }
			}
			if (!EDGE || e >= 1) {
#pragma unroll
				for (int q = 0; q < 4; q++) w3.q[q] -= avg16(w2.q[q], w4.q[q]);
			}
			if (EDGE && e == 2) {
#pragma unroll
				for (int q = 0; q < 4; q++) { v2s t = mult08p(w3.q[q]); w2.q[q] += t + t; }
			} else if (!EDGE || e >= 4) {
#pragma unroll
				for (int q = 0; q < 4; q++) w2.q[q] += m08s<X>(w1.q[q], w3.q[q]);
			}
			if (!EDGE || e >= 4) {
#pragma unroll
				for (int q = 0; q < 4; q++) { v2s t = w0.q[q] + w2.q[q]; w1.q[q] += (t >> 1) - (t >> 5); }
			}
			if (it >= 1) emit(k);
			w0 = w2; w1 = w3; w2 = w4; w3 = w5;
		}
		if (EDGE && last && m.bottom) {
			// even H: the window holds rows H-4 .. H-1 (src/lib/wavelet2d.cpp:476-491)
#pragma unroll
			for (int q = 0; q < 4; q++) {
				w3.q[q] -= w2.q[q] >> 3;
				w2.q[q] += m08s<X>(w1.q[q], w3.q[q]);
				const v2s t = w0.q[q] + w2.q[q];
				w1.q[q] += (t >> 1) - (t >> 5);
				w3.q[q] += w2.q[q] - (w2.q[q] >> 4);
			}
			emit(2);
			w0 = w2; w1 = w3;
			emit(3);
		}
		if constexpr (PC) {
			if (hring) { if (it >= 1) ring_put(hring, it); }   // block row it - 1 published
			else pc_barrier(dbg, tr ? tr + 2 * min(it, kWgIt - 1) : nullptr);   // the consumers take the block row
		} else if (it >= 1) {
			quant_row((y0 >> 3) + it - 1);   // a block row is complete
		}
	};
	if constexpr (DEPTH == 1) {
#pragma unroll 1
		for (int it = 0; it < nit; it++) iteration(it, ring[0]);
	} else {
		// pairs of iterations, then the odd one out: a conditional second
		// iteration would put its refills under a branch (see load_next)
		int it = 0;
#pragma unroll 1
		for (; it + 1 < nit; it += 2) {
			iteration(it, ring[0]);
			iteration(it + 1, ring[1]);
		}
		if (it < nit) iteration(it, ring[0]);
	}
}

// A packed level covers whole 496 x S tiles: one wave per (strip, segment),
// the waves on the image border (fq_seg<S, true>) included.
// One __constant__ image of the format tables, copied as 16-byte words.
__constant__ FqTables kFqDev __attribute__((aligned(16))) = {RIC_SYM_TABLES_INIT, make_enum_split()};

// Stages the thresholds and format tables in LDS.  NT = the block size: the
// copy is unrolled so that every thread issues all of its global loads before
// its first LDS store -- one memory round trip for the whole staging (a
// strided loop of load-store pairs pays one per iteration).
template <int NT>
__device__ __forceinline__ void fq_stage_tables(const FqArgs& a, int (*s_thres)[16], FqTables& s_F, uint32_t (*s_tpk)[17 * 8],
                                                int t = -1)
{
	const int tid = t >= 0 ? t : (int)threadIdx.x;
	static_assert(sizeof(FqTables) % 16 == 0, "table words");
	constexpr int NW = (int)(sizeof(FqTables) / 16);
	constexpr int PER = (NW + NT - 1) / NT;
	constexpr int NTP = 3 * 17 * 8;
	constexpr int PT = (NTP + NT - 1) / NT;
	const uint4* src = reinterpret_cast<const uint4*>(&kFqDev);
	uint4 v[PER];
#pragma unroll
	for (int k = 0; k < PER; k++) {
		const int i = tid + k * NT;
		v[k] = src[i < NW ? i : NW - 1];
	}
	int th = tid < 48 ? a.thres[tid / 16][tid % 16] : 0;
	uint32_t lo[PT], hi[PT];
#pragma unroll
	for (int k = 0; k < PT; k++) {
		const int i = tid + k * NT;
		const int b = min(i / (17 * 8), 2), c = (i >> 3) % 17, q = i & 7;
		lo[k] = c + q < 16 ? (uint32_t)a.thres[b][min(c + q, 15)] & 0xFFFFu : 0xFFFFu;
		hi[k] = c + q + 8 < 16 ? (uint32_t)a.thres[b][min(c + q + 8, 15)] & 0xFFFFu : 0xFFFFu;
	}
	uint4* dst = reinterpret_cast<uint4*>(&s_F);
#pragma unroll
	for (int k = 0; k < PER; k++) {
		const int i = tid + k * NT;
		if (i < NW) dst[i] = v[k];
	}
	if (tid < 48) s_thres[tid / 16][tid % 16] = th;
#pragma unroll
	for (int k = 0; k < PT; k++) {
		const int i = tid + k * NT;
		if (i < NTP) s_tpk[i / (17 * 8)][i % (17 * 8)] = lo[k] | (hi[k] << 16);
	}
}

// A consumer wave of the ring hand-off (k_fwdq_pc<true>, k_fwdq_pc2<true>):
// stage this wave's share t of the format tables (the 3 consumer waves stage
// them together: flags ring[st + 0..2]), then quantise block rows ky0 ..
// ky0 + nrows - 1 of band b as the producers publish them (ring[0 .. npub-1]
// count the block rows published, ring[took] those this wave has taken).
// The children's pRD of the next block row load while this one is quantised:
// two rows per pass, so the loop-carried registers need no copy (a copy
// waits for its load).
__device__ __forceinline__ void fq_consume(const FqArgs& a, int (*s_thres)[16], FqTables& s_F, uint32_t (*s_tpk)[17 * 8],
                                           uint2 (*buf)[3][4][kLanes], int* ring, int took, int st, int npub, int b,
                                           int kx, int ky0, int nrows, int lane, bool out_lane, int t, int dbg,
                                           uint64_t* lt)
{
	FqCrd c0 = fq_crd_load(a, b, kx, ky0);
	fq_stage_tables<192>(a, s_thres, s_F, s_tpk, t);
	ring_put(ring + st + b, 1);
	ring_wait_ge(ring + st, 1, a.err); ring_wait_ge(ring + st + 1, 1, a.err); ring_wait_ge(ring + st + 2, 1, a.err);
	if (lt && lane == 0) lt[3 + b] = __builtin_amdgcn_s_memrealtime();
	auto row = [&](int j, const FqCrd& cr) {
		// fault injection (a.fault): the first block row waits for a count
		// that never comes, with a short limit
		const bool inject = a.fault && j == 0;
		ring_wait_ge(ring, inject ? (1 << 30) : j + 1, a.err, inject ? 64 : kRingPolls);
		if (npub > 1) ring_wait_ge(ring + 1, j + 1, a.err);
		uint2 v[4];
#pragma unroll
		for (int r = 0; r < 4; r++) v[r] = buf[j & (kRing - 1)][b][r][lane];
		ring_put(ring + took, j + 1);            // (after the slot reads completed)
		if (lt && lane == 0 && j < 20) lt[16 + 20 * b + j] = __builtin_amdgcn_s_memrealtime();
		if ((dbg & 3) == 2) return;
		fq_block_regs(a, s_thres[b], s_tpk[b], s_F, b, v, kx, ky0 + j, out_lane, &cr);
		if (lt && lane == 0 && j < 20) lt[96 + 20 * b + j] = __builtin_amdgcn_s_memrealtime();
	};
	int j = 0;
#pragma unroll 1
	for (; j + 1 < nrows; j += 2) {
		const FqCrd c1 = fq_crd_load(a, b, kx, ky0 + j + 1);
		row(j, c0);
		c0 = fq_crd_load(a, b, kx, ky0 + j + 2);
		row(j + 1, c1);
	}
	if (j < nrows) row(j, c0);
	if (lt && lane == 0) lt[6 + b] = __builtin_amdgcn_s_memrealtime();
}

// grid (ceil(W / 496), ceil(nseg / 4)), one wave per segment
template <int S>
__global__ void __launch_bounds__(256, 3) k_fwdq_fast(FqArgs a)
{
	__shared__ int s_thres[3][16];
	__shared__ FqTables s_F __attribute__((aligned(16)));
	__shared__ uint32_t s_tpk[3][17 * 8];
	fq_stage_tables<256>(a, s_thres, s_F, s_tpk);
	__syncthreads();
	const int lane = threadIdx.x & 63;
	const int seg = blockIdx.y * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	if (seg >= a.nseg) return;
	const int strip = blockIdx.x;
	const int X0 = strip * kFqStrip - 8, x = X0 + lane * 8, y0 = seg * S;
	const int kx = strip * (kFqStrip / 8) + lane - 1;
	FqBorder m;
	m.top = y0 == 0;
	m.bottom = y0 + S >= a.H;
	if (X0 < 0 || X0 + kLanes * 8 >= a.W || m.top || m.bottom) {
		m.eL0 = x == 0 ? 0x0000FFFFu : 0u;
		m.oR3 = x + 7 == a.W - 1 ? 0xFFFF0000u : 0u;
		m.ld = x >= 0 && x < a.W;
		fq_seg<true>(a, s_thres, s_tpk, s_F, x, lane, y0, kx, m, S);
	} else {
		fq_seg<false>(a, s_thres, s_tpk, s_F, x, lane, y0, kx, m, S);
	}
}

// Producer-consumer form: one workgroup per segment, wave 0 lifts (fq_seg in
// PC mode), waves 1-3 quantise the D, H and V blocks of the block row the
// producer finished one iteration earlier (LDS double buffer, one barrier per
// iteration).  The lifting chain and the three quantisers of a segment run on
// four SIMDs at once, and each wave needs fewer registers.
// S is a runtime multiple of 8, chosen so that the level is about one round
// of resident workgroups.  The producer role rotates over the four waves with
// the workgroup index, so the lifting chains of the workgroups on a CU spread
// over its four SIMDs.
constexpr uint32_t kHwRegHwId = (31u << 11) | 4u;    // hwreg(HW_REG_HW_ID, 0, 32)
constexpr uint32_t kHwRegXcc = (3u << 11) | 20u;     // hwreg(HW_REG_XCC_ID, 0, 4)
constexpr int kWgTraceMax = 8192;

// Roles are static (wave (index + block x + block y) & 3 lifts): placing the
// producers on distinct SIMDs by HW_ID made no measurable difference, and a
// role known before the first barrier lets the producer issue its prologue
// row loads before the workgroup stages the format tables.
template <bool ASYNC, bool X = true, bool U8 = false>
__device__ __forceinline__ void fwdq_pc_body(const FqArgs& a, int S, int dbg, const uint8_t* src8 = nullptr, long sp8 = 0,
                                             int sh8 = 0)
{
	__shared__ int s_thres[3][16];
	__shared__ FqTables s_F __attribute__((aligned(16)));
	__shared__ uint32_t s_tpk[3][17 * 8];
	__shared__ uint2 s_buf[ASYNC ? kRing : 2][3][4][kLanes];
	// ASYNC: [0] block rows published, [1 + b] taken by consumer b, [4 + b]
	// consumer b staged its share of the tables
	__shared__ int s_ring[7];
	if (ASYNC && threadIdx.x < 7) s_ring[threadIdx.x] = 0;
	// ASYNC: this is the only barrier; the consumers stage the tables among
	// themselves while the producer lifts (it does not read them)
	if constexpr (ASYNC) __syncthreads();
	// dbg 128 (diagnostics, level 0 only): per-workgroup record of kWgRec u64 --
	// start realtime (100 MHz), start shader clock, the end realtime of waves
	// 0-3, producer hw id << 32 | end shader clock of wave 0, workgroup index,
	// then the barrier stamps of each role
	const int wgi = blockIdx.y * gridDim.x + blockIdx.x;
	uint64_t* wgt = ((dbg & 128) && a.wgt && wgi < kWgTraceMax) ? a.wgt + kWgRec * wgi : nullptr;
	if (wgt && threadIdx.x == 0) {
		wgt[0] = __builtin_amdgcn_s_memrealtime();
		wgt[1] = __builtin_amdgcn_s_memtime();
	}
	const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int wave = __builtin_amdgcn_readfirstlane((w + blockIdx.x + blockIdx.y) & 3);   // 0 = producer, 1..3 = D, H, V
	const int lane = threadIdx.x & 63;
	// dbg 4: one workgroup (strip 1, or strip 0 with dbg 64), timing only
	const int strip = (dbg & 4) ? ((dbg & 64) ? 0 : 1) : blockIdx.x, seg = (dbg & 4) ? 2 : blockIdx.y;
	const int X0 = strip * kFqStrip - 8, x = X0 + lane * 8, y0 = seg * S;
	const int kx = strip * (kFqStrip / 8) + lane - 1;
	FqBorder m;
	m.top = y0 == 0;
	m.bottom = y0 + S >= a.H;
	const bool edge = X0 < 0 || X0 + kLanes * 8 >= a.W || m.top || m.bottom;
	if ((dbg & 32) && edge) return;   // timing experiment: interior workgroups only (results invalid)
	const int nit = m.bottom ? (a.H - y0) / 8 + 1 : S / 8 + 1;
	auto stage = [&]() {
		if constexpr (!ASYNC) {
			fq_stage_tables<256>(a, s_thres, s_F, s_tpk);
			__syncthreads();
		}
	};
	if (wave == 0) {
		// the lifting chain is the segment's critical path: it issues ahead
		// of the consumer waves of other workgroups on its SIMD (dbg 2048: off)
		if (!(dbg & 2048)) __builtin_amdgcn_s_setprio(2);
		if (edge) {
			m.eL0 = x == 0 ? 0x0000FFFFu : 0u;
			m.oR3 = x + 7 == a.W - 1 ? 0xFFFF0000u : 0u;
			m.ld = x >= 0 && x < a.W;
			fq_seg<true, true, X, decltype(stage), U8>(a, s_thres, s_tpk, s_F, x, lane, y0, kx, m, S, s_buf, dbg,
			                                           wgt ? wgt + 8 : nullptr, stage, ASYNC ? s_ring : nullptr, src8, sp8, sh8);
		} else {
			fq_seg<false, true, X, decltype(stage), U8>(a, s_thres, s_tpk, s_F, x, lane, y0, kx, m, S, s_buf, dbg,
			                                            wgt ? wgt + 8 : nullptr, stage, ASYNC ? s_ring : nullptr, src8, sp8, sh8);
		}
	} else {
		const int b = wave - 1;
		const bool out_lane = lane >= 1 && lane <= kLanes - 2 && x < a.W;
		if constexpr (ASYNC) {
			// block row j = the producer's iteration j + 1
			fq_consume(a, s_thres, s_F, s_tpk, s_buf, s_ring, 1 + b, 4, 1, b, kx, y0 >> 3, nit - 1, lane, out_lane,
			           (wave - 1) * 64 + lane, dbg, nullptr);
		} else {
			stage();
#pragma unroll 1
			for (int it = 0; it < nit; it++) {
				pc_barrier(dbg, wgt ? wgt + 8 + wave * 2 * kWgIt + 2 * min(it, kWgIt - 1) : nullptr);   // matches the producer's iteration `it`
				if (it == 0 || (dbg & 3) == 2) continue;     // dbg 2: timing of the lifting alone
				uint2 buf[4];
#pragma unroll
				for (int r = 0; r < 4; r++) buf[r] = s_buf[it & 1][b][r][lane];
				fq_block_regs(a, s_thres[b], s_tpk[b], s_F, b, buf, kx, (y0 >> 3) + it - 1, out_lane);
			}
		}
	}
	if (wgt && lane == 0) {
		wgt[2 + w] = __builtin_amdgcn_s_memrealtime();
		if (wave == 0) wgt[6] = ((uint64_t)__builtin_amdgcn_s_getreg(kHwRegHwId) << 32) |
		                        (uint32_t)__builtin_amdgcn_s_memtime();
		if (w == 0) wgt[7] = (uint64_t)wgi | ((uint64_t)__builtin_amdgcn_s_getreg(kHwRegXcc) << 32);
	}
}

// One frame (arguments by value), or a batch of frames: blockIdx.z = frame,
// per-frame arguments from a device array (their pointers differ), so the
// levels of many frames run as one grid.
// X: exact mult08 sums (m08s); !X only for 8-bit-pixel input (FqArgs::in8)
template <bool ASYNC, bool X>
__global__ void __launch_bounds__(256, 4) k_fwdq_pc(FqArgs a, int S, int dbg) { fwdq_pc_body<ASYNC, X>(a, S, dbg); }
template <bool ASYNC, bool X>
__global__ void __launch_bounds__(256, 4) k_fwdq_pc_z(const FqArgs* __restrict__ az, int S, int dbg)
{
	fwdq_pc_body<ASYNC, X>(az[blockIdx.z], S, dbg);
}
// the same over a gray batch's u8 pixels (the level shift fused, no coding plane)
template <bool ASYNC>
__global__ void __launch_bounds__(256, 4) k_fwdq_pc_z8(const FqArgs* __restrict__ az, int S, int dbg, PixSrc px)
{
	fwdq_pc_body<ASYNC, false, true>(az[blockIdx.z], S, dbg, px.p[blockIdx.z], px.sp, px.sh);
}

// ------------------------------------ two-producer fused level (k_fwdq_pc2)
// The producer of k_fwdq_pc is the segment's critical path: one wave lifts
// 8 columns per lane, and a wave alone on its SIMD issues one VALU op per
// 4 cycles, so an 8-row iteration costs it ~2.5 us even on an idle chip.
// Here two producer waves split the 496-column strip into 248-column halves
// (4 columns per lane, the packed lifting of fwd97p_seg, one halo lane per
// side) and run on two SIMDs at once; the three consumer waves are those of
// k_fwdq_pc.  Producer half h, lane l (1..62) holds band columns
// h*124 + 2(l-1) + {0, 1} of the strip: word (l-1) & 1 of consumer block
// h*31 + (l-1)/2 + 1 in the LDS hand-off buffer.
template <bool EDGE, typename Stage>
__device__ __forceinline__ void fq2_producer(const FqArgs& a, int x, int lane, int h, int y0, const FqBorder& mb,
                                             int S, uint2 (*pcbuf)[3][4][kLanes], int dbg, uint64_t* tr,
                                             const Stage& stage, int* hring)
{
	const bool out_lane = lane >= 1 && lane <= kLanes - 2 && (!EDGE || x < a.W);
	const EdgeMasks em = edge_masks(x, a.W);
	const bool ld = !EDGE || (x >= 0 && x < a.W);
	int16_t* pL = a.d[BL] + (long)(y0 >> 1) * a.p[BL] + (x >> 1);
	const int L = h * (kLanes / 2 - 1) + ((lane - 1) >> 1) + 1, word = (lane - 1) & 1;
	constexpr int PF = 4, DEPTH = 2;
	const int nit = (EDGE && mb.bottom) ? (a.H - y0) / 8 + 1 : S / 8 + 1;
	const int kend = (EDGE && mb.bottom) ? 2 : PF;
	uint2 ring[DEPTH][2 * PF];
	int yl = y0 - 4;
	// unconditional loads from a wave-uniform clamped row (see fq_seg)
	const int ylast = min(y0 + S + 3, a.H - 1);
	const int xcl = EDGE ? min(max(x, 0), a.W - 4) : x;
	auto load_next = [&](uint2& dst) {
		const int yc = min(max(yl, 0), ylast);
		dst = *reinterpret_cast<const uint2*>(a.src + (long)yc * a.sp + xcl);
		yl++;
	};
#pragma unroll
	for (int d = 0; d < DEPTH; d++) {
#pragma unroll
		for (int j = 0; j < 2 * PF; j++) load_next(ring[d][j]);
	}
	stage();
	const v2s z = {0, 0};
	PRow w0 = {z, z}, w1 = {z, z}, w2 = {z, z}, w3 = {z, z}, w4, w5;
	int cur = 0;
	auto emit = [&](int k) {                    // rows e-4 (D, H) and e-3 (V, L) are final
		if (out_lane && !(dbg & 16)) {
			reinterpret_cast<uint32_t*>(&pcbuf[cur][BD][k][L])[word] = as_u32(w0.e);
			reinterpret_cast<uint32_t*>(&pcbuf[cur][BH][k][L])[word] = as_u32(w0.o);
			reinterpret_cast<uint32_t*>(&pcbuf[cur][BV][k][L])[word] = as_u32(w1.e);
			*reinterpret_cast<uint32_t*>(pL) = as_u32(w1.o);
		}
		pL += a.p[BL];
	};
	auto iteration = [&](int it, uint2 (&rg)[2 * PF]) {
		const bool last = it + 1 == nit;
		if (hring) {
			// ring hand-off (see ring_put): hring[h] = block rows published by
			// this half, hring[2 + b] = block rows consumer b has taken
			cur = (it - 1) & (kRing - 1);
			const int need = it - kRing;
			if (need > 0) {
				ring_wait_ge(hring + 2, need, a.err);
				ring_wait_ge(hring + 3, need, a.err);
				ring_wait_ge(hring + 4, need, a.err);
			}
		} else {
			cur = it & 1;
		}
#pragma unroll
		for (int k = 0; k < PF; k++) {
			if (EDGE && last && k >= kend) break;
			const int e = y0 - 4 + 2 * (it * PF + k);   // the pair's even row
			uint2 u0 = rg[2 * k], u1 = rg[2 * k + 1];
			if (EDGE && !ld) { u0 = make_uint2(0, 0); u1 = u0; }
			w4 = prow_from_u2(u0);
			w5 = prow_from_u2(u1);
			load_next(rg[2 * k]);
			load_next(rg[2 * k + 1]);
			if (EDGE && e < 0) continue;                 // above the image (top segment)
			row_fwd97p2<EDGE>(w4, w5, em);
			// P1 at e, U1 at e-1, P2 at e-2, U2 at e-3 (src/lib/wavelet2d.cpp:425-454)
			if (EDGE && e == 0) {
				w4.e -= mul3(w5.e); w4.o -= mul3(w5.o);
			} else {
				v2s te = w3.e + w5.e, to = w3.o + w5.o;
				w4.e -= te + (te >> 1); w4.o -= to + (to >> 1);
			}
			if (!EDGE || e >= 1) { w3.e -= avg16(w2.e, w4.e); w3.o -= avg16(w2.o, w4.o); }
			if (EDGE && e == 2) {
				v2s me = mult08p(w3.e), mo = mult08p(w3.o);
				w2.e += me + me; w2.o += mo + mo;
			} else if (!EDGE || e >= 4) {
				w2.e += mult08x(w1.e, w3.e); w2.o += mult08x(w1.o, w3.o);
			}
			if (!EDGE || e >= 4) {
				v2s te = w0.e + w2.e, to = w0.o + w2.o;
				w1.e += (te >> 1) - (te >> 5); w1.o += (to >> 1) - (to >> 5);
			}
			if (it >= 1) emit(k);
			w0 = w2; w1 = w3; w2 = w4; w3 = w5;
		}
		if (EDGE && last && mb.bottom) {
			// even H: the window holds rows H-4 .. H-1 (src/lib/wavelet2d.cpp:476-491)
			w3.e -= w2.e >> 3; w3.o -= w2.o >> 3;
			w2.e += mult08x(w1.e, w3.e); w2.o += mult08x(w1.o, w3.o);
			v2s te = w0.e + w2.e, to = w0.o + w2.o;
			w1.e += (te >> 1) - (te >> 5); w1.o += (to >> 1) - (to >> 5);
			w3.e += w2.e - (w2.e >> 4); w3.o += w2.o - (w2.o >> 4);
			emit(2);
			w0 = w2; w1 = w3;
			emit(3);
		}
		if (hring) { if (it >= 1) ring_put(hring + h, it); }
		else pc_barrier(dbg, tr ? tr + 2 * min(it, kWgIt - 1) : nullptr);   // the consumers take the block row
	};
	int it = 0;
#pragma unroll 1
	for (; it + 1 < nit; it += 2) {
		iteration(it, ring[0]);
		iteration(it + 1, ring[1]);
	}
	if (it < nit) iteration(it, ring[0]);
}

// grid (strips, segments), 5 waves: 0, 1 = producers of the two halves,
// 2..4 = the D, H, V consumers
template <bool ASYNC>
__device__ __forceinline__ void fwdq_pc2_body(const FqArgs& a, int S, int dbg)
{
	__shared__ int s_thres[3][16];
	__shared__ FqTables s_F __attribute__((aligned(16)));
	__shared__ uint32_t s_tpk[3][17 * 8];
	__shared__ uint2 s_buf[ASYNC ? kRing : 2][3][4][kLanes];
	// ASYNC: [h] block rows published by producer h, [2 + b] taken by consumer
	// b, [5 + b] consumer b staged its share of the tables
	__shared__ int s_ring[8];
	if (ASYNC && threadIdx.x < 8) s_ring[threadIdx.x] = 0;
	if constexpr (ASYNC) __syncthreads();   // the only barrier (see k_fwdq_pc)
	const int wgi = blockIdx.y * gridDim.x + blockIdx.x;
	uint64_t* wgt = ((dbg & 128) && a.wgt && wgi < kWgTraceMax) ? a.wgt + kWgRec * wgi : nullptr;
	if (wgt && threadIdx.x == 0) {
		wgt[0] = __builtin_amdgcn_s_memrealtime();
		wgt[1] = __builtin_amdgcn_s_memtime();
	}
	// diagnostics (RIC_LVL_TRACE=level, async form): [0] start, [1 + h]
	// producer h done, [3 + b] consumer b staged, [6 + b] consumer b done,
	// [16 + 20 b + j] consumer b took block row j, [96 + 20 b + j] finished it
	uint64_t* lt = (ASYNC && !(dbg & 128) && a.wgt && wgi < kWgTraceMax) ? a.wgt + kWgRec * wgi : nullptr;
	if (lt && threadIdx.x == 0) lt[0] = __builtin_amdgcn_s_memrealtime();
	const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	const int strip = (dbg & 4) ? ((dbg & 64) ? 0 : 1) : blockIdx.x, seg = (dbg & 4) ? 2 : blockIdx.y;
	const int y0 = seg * S;
	const int SX = strip * kFqStrip;                            // first output column of the strip
	FqBorder mb;
	mb.top = y0 == 0;
	mb.bottom = y0 + S >= a.H;
	const bool edge = SX == 0 || SX - 8 + kLanes * 8 >= a.W || mb.top || mb.bottom;
	const int nit = mb.bottom ? (a.H - y0) / 8 + 1 : S / 8 + 1;
	auto stage = [&]() {
		if constexpr (!ASYNC) {
			fq_stage_tables<320>(a, s_thres, s_F, s_tpk);
			__syncthreads();
		}
	};
	if (w < 2) {
		if (!(dbg & 2048)) __builtin_amdgcn_s_setprio(2);
		const int x = SX + w * (kStripValid) - kCols + lane * kCols;   // 4 columns per lane
		uint64_t* tr = (wgt && w == 0) ? wgt + 8 : nullptr;        // trace roles: producer 0, D, H, V
		int* hr = ASYNC ? s_ring : nullptr;
		if (edge) fq2_producer<true>(a, x, lane, w, y0, mb, S, s_buf, dbg, tr, stage, hr);
		else fq2_producer<false>(a, x, lane, w, y0, mb, S, s_buf, dbg, tr, stage, hr);
		if (lt && lane == 0) lt[1 + w] = __builtin_amdgcn_s_memrealtime();
	} else {
		const int b = w - 2;
		const int xc = SX - 8 + lane * 8;                        // the block's 8 image columns
		const int kx = strip * (kFqStrip / 8) + lane - 1;
		const bool out_lane = lane >= 1 && lane <= kLanes - 2 && xc < a.W;
		if constexpr (ASYNC) {
			// block row j: both halves published
			fq_consume(a, s_thres, s_F, s_tpk, s_buf, s_ring, 2 + b, 5, 2, b, kx, y0 >> 3, nit - 1, lane, out_lane,
			           b * 64 + lane, dbg, lt);
		} else {
			stage();
#pragma unroll 1
			for (int it = 0; it < nit; it++) {
				pc_barrier(dbg, wgt ? wgt + 8 + (w - 1) * 2 * kWgIt + 2 * min(it, kWgIt - 1) : nullptr);
				if (it == 0 || (dbg & 3) == 2) continue;     // dbg 2: timing of the lifting alone
				uint2 buf[4];
#pragma unroll
				for (int r = 0; r < 4; r++) buf[r] = s_buf[it & 1][b][r][lane];
				fq_block_regs(a, s_thres[b], s_tpk[b], s_F, b, buf, kx, (y0 >> 3) + it - 1, out_lane);
			}
		}
	}
	if (wgt && lane == 0) {
		wgt[2 + (w < 4 ? w : 3)] = __builtin_amdgcn_s_memrealtime();
		if (w == 0) wgt[6] = ((uint64_t)__builtin_amdgcn_s_getreg(kHwRegHwId) << 32) |
		                     (uint32_t)__builtin_amdgcn_s_memtime();
		if (w == 0) wgt[7] = (uint64_t)wgi | ((uint64_t)__builtin_amdgcn_s_getreg(kHwRegXcc) << 32);
	}
}

template <bool ASYNC>
__global__ void __launch_bounds__(320) k_fwdq_pc2(FqArgs a, int S, int dbg) { fwdq_pc2_body<ASYNC>(a, S, dbg); }
template <bool ASYNC>
__global__ void __launch_bounds__(320) k_fwdq_pc2_z(const FqArgs* __restrict__ az, int S, int dbg)
{
	fwdq_pc2_body<ASYNC>(az[blockIdx.z], S, dbg);
}

int fq_seg_rows(int H)
{
	static const int forced = [] { const char* e = getenv("RIC_FQ_S"); return e ? atoi(e) : 0; }();
	if (forced == 8 || forced == 16 || forced == 32) return forced;
	return H >= 4096 ? 32 : 16;
}

int fq_pc()
{
	static const int v = [] { const char* e = getenv("RIC_FQ_PC"); return e ? atoi(e) : 1; }();
	return v;
}

template <int S>
void fq_launch_s(FqArgs& a, hipStream_t st)
{
	a.nseg = (a.H + S - 1) / S;
	const int nstrip = (a.W + kFqStrip - 1) / kFqStrip;
	dim3 grid(nstrip, (a.nseg + kWavesPerBlock - 1) / kWavesPerBlock);
	hipLaunchKernelGGL(k_fwdq_fast<S>, grid, dim3(256), 0, st, a);
}

// segment height of the producer-consumer form: about one round of resident
// workgroups (kPcResident per CU) over the level, at least 8 rows
constexpr int kPcResident = 4 * 256;
int pc_seg_rows(int W, int H)
{
	static const int forced = [] { const char* e = getenv("RIC_FQ_S"); return e ? atoi(e) : 0; }();
	if (forced >= 8 && forced % 8 == 0) return forced;
	const int nstrip = (W + kFqStrip - 1) / kFqStrip;
	const int want = (kPcResident + nstrip - 1) / nstrip;            // segments per strip
	const int s = ((H + want - 1) / want + 7) / 8 * 8;
	return s < 8 ? 8 : s;
}

// diagnostics: per-device workgroup trace buffer of k_fwdq_pc (dbg 128)
uint64_t* g_wgtrace[64] = {};
std::mutex g_wgtrace_mu;
uint64_t* fq_wgtrace()
{
	int dev = 0;
	if (hipGetDevice(&dev) != hipSuccess) return nullptr;
	std::lock_guard<std::mutex> g(g_wgtrace_mu);
	uint64_t*& b = g_wgtrace[dev & 63];
	if (!b && hipMalloc(&b, (size_t)kWgTraceMax * kWgRec * sizeof(uint64_t)) != hipSuccess) b = nullptr;
	if (b) (void)hipMemset(b, 0, (size_t)kWgTraceMax * kWgRec * sizeof(uint64_t));
	return b;
}

void fq_launch_pc(FqArgs& a, hipStream_t st)
{
	// tuning knobs RIC_FQ_SL0..2: segment rows of level 0..2 (multiples of 8)
	static const int sl[3] = {[] { const char* e = getenv("RIC_FQ_SL0"); return e ? atoi(e) : 0; }(),
	                          [] { const char* e = getenv("RIC_FQ_SL1"); return e ? atoi(e) : 0; }(),
	                          [] { const char* e = getenv("RIC_FQ_SL2"); return e ? atoi(e) : 0; }()};
	int S = pc_seg_rows(a.W, a.H);
	if (a.level < 3 && sl[a.level] >= 8 && sl[a.level] % 8 == 0) S = sl[a.level];
	a.nseg = (a.H + S - 1) / S;
	const int nstrip = (a.W + kFqStrip - 1) / kFqStrip;
	static const int onewg = [] { const char* e = getenv("RIC_FQ_ONEWG"); return e ? atoi(e) : 0; }();
	// RIC_FQ_ONEWG=1: one interior workgroup only (latency of one segment; results invalid)
	int dbg = fq_pc();
	static const int ltrace = [] { const char* e = getenv("RIC_LVL_TRACE"); return e ? atoi(e) : -1; }();
	a.wgt = ltrace == a.level ? fq_wgtrace() : nullptr;
	if ((dbg & 128) && a.high && !a.wgt && !(a.wgt = fq_wgtrace())) dbg &= ~128;
	// the two-producer form on the coarser levels (their segments are short
	// and latency-bound); level 0 is VALU-throughput-bound, where the
	// one-producer form's 8-column rows cost fewer instructions.
	// RIC_FQ_PC2=0/1 forces either form.
	static const int force2 = [] { const char* e = getenv("RIC_FQ_PC2"); return e ? atoi(e) : -1; }();
	const bool two = force2 >= 0 ? force2 != 0 : !a.high;
	if (two) {
		static const int async2 = [] { const char* e = getenv("RIC_FQ_ASYNC"); return e ? atoi(e) : 1; }();
		const dim3 grid2 = onewg ? dim3(1, 1) : dim3(nstrip, a.nseg);
		const int dbg2 = onewg ? dbg | 4 : dbg;
		if (async2) hipLaunchKernelGGL(k_fwdq_pc2<true>, grid2, dim3(320), 0, st, a, S, dbg2 & ~128);
		else hipLaunchKernelGGL(k_fwdq_pc2<false>, grid2, dim3(320), 0, st, a, S, dbg2);
	} else {
		// the ring hand-off (the single-frame calls run alone on the chip:
		// measured round 5 at C3, 63.0 against 65.0 us per frame for the
		// double buffer, despite the ring form's 20-28 bytes of scratch per lane)
		static const int async = [] { const char* e = getenv("RIC_FQ_ASYNC"); return e ? atoi(e) : 1; }();
		const dim3 grid = onewg ? dim3(1, 1) : dim3(nstrip, a.nseg);
		if (onewg) dbg |= 4;
		if (async && a.in8) hipLaunchKernelGGL((k_fwdq_pc<true, false>), grid, dim3(256), 0, st, a, S, dbg & ~128);
		else if (async) hipLaunchKernelGGL((k_fwdq_pc<true, true>), grid, dim3(256), 0, st, a, S, dbg & ~128);
		else if (a.in8) hipLaunchKernelGGL((k_fwdq_pc<false, false>), grid, dim3(256), 0, st, a, S, dbg);
		else hipLaunchKernelGGL((k_fwdq_pc<false, true>), grid, dim3(256), 0, st, a, S, dbg);
	}
}

// ------------------------------ generic fused forward level + quantiser
// k_fwdq_gen: the same fusion as k_fwdq_fast for the 9/7 levels the packed
// kernel does not take (int bands -- the coarsest level under ric's
// level_chg --, image sizes that are not multiples of 8, rd thresholds
// outside the packed range).  Geometry of k_fwd (4 columns per lane, 248
// output columns per wave) with 8-row segments, so even a small level has
// hundreds of waves: the wave lifts its segment with fwd_seg (checked path),
// then quantises the 31 x 3 blocks it produced, read back from HBM (they were
// written by lanes of this same wave: a workgroup-scope fence orders it), two
// blocks per lane.  On the coarsest level it also runs the LL TSUQ
// (src/lib/band.h:65-92) on the LL samples it wrote.
constexpr int kGenRows = 8;
constexpr int kGenBlocks = kStripValid / 8;   // 31 block columns per wave

struct GenLL {
	int on, iQ, T0;
};

template <typename TO>
__device__ __forceinline__ void gen_block(const FqArgs& a, const int* thr, const uint32_t* tpk, const FqTables& F,
                                          const TO* const* d, int b, int kx, int ky)
{
	constexpr bool SH = sizeof(TO) == 2;
	const int x0 = 4 * kx, y0 = 4 * ky, dx = a.dx[b], dy = a.dy[b];
	const int wdt = min(4, dx - x0), hgt = min(4, dy - y0);
	const bool full = wdt == 4 && hgt == 4;
	const long pb = a.p[b];
	TO* base = const_cast<TO*>(d[b]) + (long)y0 * pb + x0;
	// clamped addresses; the block's 16 values and the children's pRD are all
	// loaded before one pin of the whole batch: one memory round trip per
	// block (a pin per load waits for each load in turn)
	int v[16];
#pragma unroll
	for (int i = 0; i < 16; i++) {
		const int r = min(i >> 2, hgt - 1), c = min(i & 3, wdt - 1);
		v[i] = (int)base[r * pb + c];
	}
	uint32_t cr[4] = {0u, 0u, 0u, 0u};
	const uint32_t* crd = a.crd[b];
	if (crd) {
		const int cw = a.cbw[b], ch = a.cph[b];
		const int cy0 = min(2 * ky, ch - 1), cy1 = min(2 * ky + 1, ch - 1);
		const int cx0 = min(2 * kx, cw - 1), cx1 = min(2 * kx + 1, cw - 1);
		cr[0] = crd[(long)cy0 * cw + cx0]; cr[1] = crd[(long)cy0 * cw + cx1];
		cr[2] = crd[(long)cy1 * cw + cx0]; cr[3] = crd[(long)cy1 * cw + cx1];
	}
	asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
	                  "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15]));
	asm volatile("" : "+v"(cr[0]), "+v"(cr[1]), "+v"(cr[2]), "+v"(cr[3]));
#pragma unroll
	for (int i = 0; i < 16; i++) v[i] = ((i >> 2) < hgt && (i & 3) < wdt) ? v[i] : 0;
	// children pRD: u32 sum, as k_quant_level (full blocks only)
	const uint32_t csum = (full && crd) ? cr[0] + cr[1] + cr[2] + cr[3] : 0u;
	uint32_t dist;
	if (full) {
		int cnt;
		if (SH && a.pk) {
			// the packed quantiser (same result when the thresholds pass pk_ok)
			uint32_t w[8];
#pragma unroll
			for (int r = 0; r < 4; r++) {
				w[2 * r] = (uint32_t)(uint16_t)v[4 * r] | ((uint32_t)(uint16_t)v[4 * r + 1] << 16);
				w[2 * r + 1] = (uint32_t)(uint16_t)v[4 * r + 2] | ((uint32_t)(uint16_t)v[4 * r + 3] << 16);
			}
			cnt = tsuq_full_pk(w, a.Q[b], a.iQ[b], thr[0], tpk);
#pragma unroll
			for (int r = 0; r < 4; r++) {
				v[4 * r] = (int16_t)(w[2 * r] & 0xFFFFu); v[4 * r + 1] = (int16_t)(w[2 * r] >> 16);
				v[4 * r + 2] = (int16_t)(w[2 * r + 1] & 0xFFFFu); v[4 * r + 3] = (int16_t)(w[2 * r + 1] >> 16);
			}
		} else {
			cnt = tsuq_full<SH>(v, a.Q[b], a.iQ[b], thr);
		}
		const uint64_t dd = (uint64_t)cnt + csum;
		dist = dd > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)dd;
	} else {
		dist = (uint32_t)tsuq_edge<SH>(v, wdt, hgt, a.Q[b], a.iQ[b]);   // children ignored
	}
	if (dist == 0) v[0] = kInsignif;
#pragma unroll
	for (int i = 0; i < 16; i++)
		if ((i >> 2) < hgt && (i & 3) < wdt) base[(i >> 2) * pb + (i & 3)] = (TO)v[i];
	const long bi = (long)ky * a.bw[b] + kx;
	a.rd[b][bi] = dist;
	a.rec[b][bi] = full ? block_local_full(F.T, F.E, v, a.high != 0) : block_local_edge(F.T, v, wdt, hgt, a.high != 0);
	uint8_t* cp = a.cpin[b];
	if (cp) {
		const uint32_t prop = (full && v[0] == kInsignif) ? 0x80u : 0u;
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const int qx = q & 1, qy = q >> 1, cx = 2 * kx + qx, cy = 2 * ky + qy, o = 8 * qy + 2 * qx;
			if (cx < a.cpw[b] && cy < a.cph[b])
				cp[(long)cy * a.cpw[b] + cx] = (uint8_t)(pin_ctx_of<SH>(v[o], v[o + 1], v[o + 4], v[o + 5]) | prop);
		}
	}
}

// One workgroup per 8-row segment of a 248-column strip: each wave lifts two
// of its rows, then the workgroup stages the tables, and all 256 threads
// quantise the segment's 3 x 31 blocks (one round) and run the coarsest
// level's LL TSUQ.  The levels
// that take this kernel are small and latency-bound: the wide block phase
// replaces the two dependent rounds of a wave-per-segment form.
// GR: rows per workgroup (a multiple of 8; each wave lifts GR / 4 rows)
template <typename TI, typename TO, int GR>
__device__ __forceinline__ void fwdq_gen_body(const FqArgs& a, const GenLL& ll, int nseg)
{
	static_assert(GR % 8 == 0, "whole block rows per workgroup");
	constexpr int WR = GR / 4;   // rows lifted per wave
	__shared__ int s_thres[3][16];
	__shared__ FqTables s_F __attribute__((aligned(16)));
	__shared__ uint32_t s_tpk[3][17 * 8];
	const int lane = threadIdx.x & 63;
	const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int seg = blockIdx.y;
	const int strip = blockIdx.x;
	const int y0 = seg * GR;
	FwdArgs<TI, TO> f;
	f.src = reinterpret_cast<const TI*>(a.src); f.sp = a.sp; f.W = a.W; f.H = a.H;
#pragma unroll
	for (int b = 0; b < 4; b++) { f.d[b] = reinterpret_cast<TO*>(a.d[b]); f.p[b] = a.p[b]; }
	f.nseg = nseg; f.vec = a.vec8; f.nofast = 1;
	// diagnostics (RIC_LVL_TRACE=level): phase stamps of every workgroup
	const int wgi = blockIdx.y * gridDim.x + blockIdx.x;
	uint64_t* wgt = (a.wgt && wgi < kWgTraceMax) ? a.wgt + kWgRec * wgi : nullptr;
	if (wgt && threadIdx.x == 0) wgt[0] = __builtin_amdgcn_s_memrealtime();
	// the four waves lift two rows each (own halo rows): a lifting wave is
	// instruction-latency-bound, and 5 row pairs per wave instead of 8
	// shorten the chain that the whole segment waits for
	if (y0 + WR * w < a.H) {
		const int X0 = strip * kStripValid - kCols;
		if constexpr (sizeof(TI) == 2 && sizeof(TO) == 2)
			fwd97p_seg<WR, false>(f, X0 + lane * kCols, lane, y0 + WR * w);     // packed 16-bit lifting
		else
			fwd_seg<CDF97, TI, TO, WR, false>(f, X0 + lane * kCols, lane, y0 + WR * w);
	}
	if (wgt && lane == 0 && w == 0) wgt[1] = __builtin_amdgcn_s_memrealtime();
	fq_stage_tables<256>(a, s_thres, s_F, s_tpk);
	if (wgt && threadIdx.x == 64) wgt[2] = __builtin_amdgcn_s_memrealtime();
	// the bands wave 0 wrote are read by the whole workgroup
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
	__syncthreads();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
	if (wgt && threadIdx.x == 0) wgt[3] = __builtin_amdgcn_s_memrealtime();
	const TO* d[3] = {f.d[0], f.d[1], f.d[2]};
	constexpr int NB = 3 * kGenBlocks * (GR / 8);     // the segment's blocks: band, block row, column
	for (int i = threadIdx.x; i < NB; i += 256) {
		const int b = i / (kGenBlocks * (GR / 8)), rem = i - b * kGenBlocks * (GR / 8);
		const int ky = (y0 >> 3) + rem / kGenBlocks, kx = strip * kGenBlocks + rem % kGenBlocks;
		if (kx < a.bw[b] && ky < a.bh[b]) gen_block<TO>(a, s_thres[b], s_tpk[b], s_F, d, b, kx, ky);
	}
	if (wgt && lane == 0) wgt[4 + w] = __builtin_amdgcn_s_memrealtime();
	if (ll.on) {
		// CBand::TSUQ with Thres 0.5 on this segment's LL samples: all loads first
		constexpr bool SH = sizeof(TO) == 2;
		constexpr int NLL = (GR / 2) * (kStripValid / 2);
		constexpr int PER = (NLL + 255) / 256;
		const int ldx = a.W >> 1, ldy = a.H >> 1, c0 = strip * (kStripValid / 2), r0 = y0 >> 1;
		int val[PER];
		TO* q[PER];
		bool in[PER];
#pragma unroll
		for (int k = 0; k < PER; k++) {
			const int i = threadIdx.x + k * 256;
			const int r = r0 + i / (kStripValid / 2), c = c0 + i % (kStripValid / 2);
			in[k] = i < NLL && r < ldy && c < ldx;
			q[k] = f.d[BL] + (long)min(r, ldy - 1) * f.p[BL] + min(c, ldx - 1);
			val[k] = *q[k];
		}
#pragma unroll
		for (int k = 0; k < PER; k++) {
			const int v = val[k];
			if (in[k])
				*q[k] = (uint32_t)(v + ll.T0) <= (uint32_t)(2 * ll.T0) ? (TO)0
				        : (TO)tr<SH>((int)((uint32_t)v * (uint32_t)ll.iQ + 32768u) >> 16);
		}
		if (wgt && threadIdx.x == 0) wgt[8] = __builtin_amdgcn_s_memrealtime();
	}
}

template <typename TI, typename TO>
__global__ void __launch_bounds__(256) k_fwdq_gen(FqArgs a, GenLL ll, int nseg) { fwdq_gen_body<TI, TO, kGenRows>(a, ll, nseg); }
template <typename TI, typename TO, int GR>
__global__ void __launch_bounds__(256) k_fwdq_gen_z(const FqArgs* __restrict__ az, GenLL ll, int nseg)
{
	fwdq_gen_body<TI, TO, GR>(az[blockIdx.z], ll, nseg);
}

// ---------------------------------------------------------- inverse level
template <typename TB, typename TL, typename TO>
struct InvArgs {
	const TB* d[3]; long p[3];  // D, H, V bands (level type)
	const TL* ll; long pl;      // LL (level type)
	TO* out; long po;           // reconstructed plane (finer level type / image)
	int W, H, nseg, ovec, nofast;
	int quirk_dalign, quirk_halign;   // reference DimXAlign of D and H (5/3 only)
	int q[4];                   // fused TSUQi multipliers of D, H, V, LL (1 = none)
	// pixel output fused into a gray frame's level 0 (k_inv_z PIX): instead of
	// the int16 plane, the u8 pixels (W bytes per row) with ric's unshift +
	// clip (src/ric/ric.cpp:237-240; q: the frame's quantiser, 0 = lossless),
	// and the pixels' digest (launch_digest's formula) added into one of the
	// frame's 16 partial words dig[0..15] (folded by launch_digest_fold)
	uint8_t* pix; unsigned long long* dig; int pq;
};

// CBand::TSUQi (src/lib/band.h:94-107) on a loaded band value: v *= (C)q
template <bool SH>
__device__ __forceinline__ int deq(int v, int q) { return tr<SH>((int)((uint32_t)v * (uint32_t)q)); }
// the same on two packed shorts (the low 16 bits of the product)
__device__ __forceinline__ uint32_t deq2(uint32_t w, int q)
{
	return as_w(as_v2u(w) * splat2((uint32_t)q));
}

template <int TRANS, typename TB, typename TL, typename TO, int S, bool FAST>
__device__ __forceinline__ void inv_seg(const InvArgs<TB, TL, TO>& a, int x, int lane, int y0)
{
	constexpr bool SH = sizeof(TB) == 2;
	constexpr bool EDGE = !FAST;
	const int W = a.W, H = a.H;
	const int dxD = (W + 1) >> 1, dxH = W >> 1;
	const bool out_lane = lane >= 1 && lane <= kLanes - 2 && (FAST || x < W);
	const int bx = x >> 1;
	using R2 = typename Raw2<TB>::type;
	// even rows: D (cols 0,2) + H (cols 1,3); odd rows: V + LL
	auto load_pair = [&](int y, R2& lo, R2& hi) {
		const int by = y >> 1;
		if (!(y & 1)) {
			lo = load_band2<TB, EDGE>(a.d[BD] + (long)by * a.p[BD], bx, dxD);
			if (!FAST && TRANS == CDF53 && y == 2) {
				// Transform53I reads this H row with the D stride
				// (src/lib/wavelet2d.cpp:715): replay it on the reference layout.
				int v[2];
#pragma unroll
				for (int k = 0; k < 2; k++) {
					int b = bx + k;
					v[k] = 0;
					if (b >= 0 && b < dxH) {
						long f = (long)a.quirk_dalign + b;
						long rr = f / a.quirk_halign, cc = f % a.quirk_halign;
						if (cc < dxH && rr < ((H + 1) >> 1)) v[k] = a.d[BH][rr * a.p[BH] + cc];
					}
				}
				if constexpr (sizeof(TB) == 2) hi = (uint32_t)(uint16_t)v[0] | ((uint32_t)v[1] << 16);
				else hi = make_int2(v[0], v[1]);
			} else {
				hi = load_band2<TB, EDGE>(a.d[BH] + (long)by * a.p[BH], bx, dxH);
			}
		} else {
			lo = load_band2<TB, EDGE>(a.d[BV] + (long)by * a.p[BV], bx, dxD);
			hi = load_band2<TL, EDGE>(a.ll + (long)by * a.pl, bx, dxH);
		}
	};
	// odd: the row's bands are V + LL, else D + H (fused TSUQi multipliers)
	auto unpack_row = [&](const R2& lo, const R2& hi, int (&r)[4], bool odd) {
		unpack2<TB>(lo, r[0], r[2]);
		unpack2<TB>(hi, r[1], r[3]);
		const int ql = odd ? a.q[BV] : a.q[BD], qh = odd ? a.q[BL] : a.q[BH];
		r[0] = deq<SH>(r[0], ql); r[2] = deq<SH>(r[2], ql);
		r[1] = deq<SH>(r[1], qh); r[3] = deq<SH>(r[3], qh);
	};
	auto emit = [&](int y, const int (&rw)[4]) {
		if (!FAST && (y < y0 || y >= y0 + S || y >= H)) return;
		int r[4];
		FOR4 r[j] = rw[j];
		row_inv<TRANS, SH, EDGE>(r, x, W);
		if (!out_lane) return;
		TO* row = a.out + (long)y * a.po;
		if (FAST || (a.ovec && x + 3 < W)) {
			if constexpr (sizeof(TO) == 2) {
				*reinterpret_cast<uint2*>(row + x) =
					make_uint2((uint32_t)(uint16_t)r[0] | ((uint32_t)r[1] << 16),
					           (uint32_t)(uint16_t)r[2] | ((uint32_t)r[3] << 16));
			} else {
				*reinterpret_cast<int4*>(row + x) = make_int4(r[0], r[1], r[2], r[3]);
			}
		} else {
			FOR4 if (x + j < W) row[x + j] = (TO)r[j];
		}
	};

	if constexpr (TRANS == HAAR) {
		// TransformHaarI, src/lib/wavelet2d.cpp:821-855
		for (int e = y0; e < y0 + S && e + 1 < H; e += 2) {
			R2 l0, h0, l1, h1;
			int r0[4], r1[4];
			load_pair(e, l0, h0); load_pair(e + 1, l1, h1);
			unpack_row(l0, h0, r0, false); unpack_row(l1, h1, r1, true);
			FOR4 { r1[j] = tr<SH>(r1[j] - (r0[j] >> 1)); r0[j] = tr<SH>(r0[j] + r1[j]); }
			emit(e, r0); emit(e + 1, r1);
		}
	} else {
		constexpr int R = S + 8;                 // band rows of image rows y0-4 .. y0+S+3
		R2 rlo[R], rhi[R];
		if constexpr (!FAST && TRANS == CDF97) {
			// border waves: every raw element (clamped row of the same parity,
			// clamped columns) is loaded first and the batch pinned at once, then
			// the out-of-band rows / columns are zeroed -- one memory round trip
			// for the segment (a pin per load waits for each load in turn)
			int ra[R][4];
			const int hiD = max(dxD - 1, 0), hiH = max(dxH - 1, 0);
			const int cD0 = min(max(bx, 0), hiD), cD1 = min(max(bx + 1, 0), hiD);
			const int cH0 = min(max(bx, 0), hiH), cH1 = min(max(bx + 1, 0), hiH);
#pragma unroll
			for (int i = 0; i < R; i++) {
				const int y = y0 - 4 + i;
				const int yc = y < 0 ? (y & 1) : y >= H ? H - 1 - ((H - 1 - y) & 1) : y;
				const long by = yc >> 1;
				const TB* lo = (i & 1) ? a.d[BV] + by * a.p[BV] : a.d[BD] + by * a.p[BD];
				if (i & 1) {
					const TL* hl = a.ll + by * a.pl;
					ra[i][2] = (int)hl[cH0]; ra[i][3] = (int)hl[cH1];
				} else {
					const TB* hh = a.d[BH] + by * a.p[BH];
					ra[i][2] = (int)hh[cH0]; ra[i][3] = (int)hh[cH1];
				}
				ra[i][0] = (int)lo[cD0]; ra[i][1] = (int)lo[cD1];
			}
#pragma unroll
			for (int i = 0; i + 4 <= R; i += 4)
				asm volatile("" : "+v"(ra[i][0]), "+v"(ra[i][1]), "+v"(ra[i][2]), "+v"(ra[i][3]),
				                  "+v"(ra[i + 1][0]), "+v"(ra[i + 1][1]), "+v"(ra[i + 1][2]), "+v"(ra[i + 1][3]),
				                  "+v"(ra[i + 2][0]), "+v"(ra[i + 2][1]), "+v"(ra[i + 2][2]), "+v"(ra[i + 2][3]),
				                  "+v"(ra[i + 3][0]), "+v"(ra[i + 3][1]), "+v"(ra[i + 3][2]), "+v"(ra[i + 3][3]));
			if constexpr (R % 4 == 2)        // (S = 2: rows R-2, R-1)
				asm volatile("" : "+v"(ra[R - 2][0]), "+v"(ra[R - 2][1]), "+v"(ra[R - 2][2]), "+v"(ra[R - 2][3]),
				                  "+v"(ra[R - 1][0]), "+v"(ra[R - 1][1]), "+v"(ra[R - 1][2]), "+v"(ra[R - 1][3]));
			const bool iD0 = bx >= 0 && bx < dxD, iD1 = bx + 1 >= 0 && bx + 1 < dxD;
			const bool iH0 = bx >= 0 && bx < dxH, iH1 = bx + 1 >= 0 && bx + 1 < dxH;
#pragma unroll
			for (int i = 0; i < R; i++) {
				const int y = y0 - 4 + i;
				const bool in = y >= 0 && y < H;
				const int l0 = in && iD0 ? ra[i][0] : 0, l1 = in && iD1 ? ra[i][1] : 0;
				const int h0 = in && iH0 ? ra[i][2] : 0, h1 = in && iH1 ? ra[i][3] : 0;
				if constexpr (sizeof(TB) == 2) {
					rlo[i] = (uint32_t)(uint16_t)l0 | ((uint32_t)l1 << 16);
					rhi[i] = (uint32_t)(uint16_t)h0 | ((uint32_t)h1 << 16);
				} else {
					rlo[i] = make_int2(l0, l1);
					rhi[i] = make_int2(h0, h1);
				}
			}
		} else {
#pragma unroll
			for (int i = 0; i < R; i++) {
				const int y = y0 - 4 + i;
				if (FAST) {
					load_pair(y, rlo[i], rhi[i]);
				} else {
					// rows outside the image read as 0: the nearest row of the same
					// parity (same bands), then a select -- no divergent branch
					const int yc = y < 0 ? (y & 1) : y >= H ? H - 1 - ((H - 1 - y) & 1) : y;
					R2 lo, hi;
					load_pair(yc, lo, hi);
					const bool in = y >= 0 && y < H;
					rlo[i] = in ? lo : R2{}; rhi[i] = in ? hi : R2{};
				}
			}
		}
		int w0[4] = {0, 0, 0, 0}, w1[4] = {0, 0, 0, 0}, w2[4] = {0, 0, 0, 0}, w3[4] = {0, 0, 0, 0};
		int w4[4] = {0, 0, 0, 0}, w5[4], w6[4] = {0, 0, 0, 0};
		// window: w0..w6 = rows e-5 .. e+1
#pragma unroll
		for (int i = 0; i < R; i += 2) {
			const int e = y0 - 4 + i;
			if (!FAST && (e < 0 || e >= H)) continue;
			unpack_row(rlo[i], rhi[i], w5, false);
			if (FAST || e + 1 < H) unpack_row(rlo[i + 1], rhi[i + 1], w6, true);
			if constexpr (TRANS == CDF97) {
				// U2^-1 at e-1, P2^-1 at e-2, U1^-1 at e-3, P1^-1 at e-4
				// (src/lib/wavelet2d.cpp:512-561)
				if (FAST || e >= 2) { FOR4 { int t = tr<SH>(w3[j] + w5[j]); w4[j] = tr<SH>(w4[j] - ((t >> 1) - (t >> 5))); } }
				if (!FAST && e == 2) { FOR4 w3[j] = tr<SH>(w3[j] - 2 * mult08<SH>(w4[j])); }
				else if (FAST || e >= 4) { FOR4 w3[j] = tr<SH>(w3[j] - mult08<false>(w2[j] + w4[j])); }
				if (FAST || e >= 4) { FOR4 w2[j] = tr<SH>(w2[j] + ((w1[j] + w3[j]) >> 4)); }
				if (!FAST && e == 4) { FOR4 w1[j] = tr<SH>(w1[j] + w2[j] * 3); }
				else if (FAST || e >= 6) { FOR4 { int t = tr<SH>(w0[j] + w2[j]); w1[j] = tr<SH>(w1[j] + (t + (t >> 1))); } }
			} else {
				// U^-1 at e-1, P^-1 at e-2 (src/lib/wavelet2d.cpp:712-747)
				if (FAST || e >= 2) { FOR4 w4[j] = tr<SH>(w4[j] - ((w3[j] + w5[j]) >> 2)); }
				if (!FAST && e == 2) { FOR4 w3[j] = tr<SH>(w3[j] + w4[j]); }
				else if (FAST || e >= 4) { FOR4 w3[j] = tr<SH>(w3[j] + ((w2[j] + w4[j]) >> 1)); }
			}
			if (!FAST || i >= 8) { emit(e - 4, w1); emit(e - 3, w2); }
			FOR4 { w0[j] = w2[j]; w1[j] = w3[j]; w2[j] = w4[j]; w3[j] = w5[j]; w4[j] = w6[j]; }
		}
		if (!FAST && y0 + S + 4 >= H) {
			// window now holds rows e-3 .. e+1 of the last pair e in w0..w4
			if (!(H & 1)) {                      // rows H-5 .. H-1
				if constexpr (TRANS == CDF97) {  // src/lib/wavelet2d.cpp:572-587
					FOR4 w4[j] = tr<SH>(w4[j] - (w3[j] - (w3[j] >> 4)));
					FOR4 w3[j] = tr<SH>(w3[j] - mult08<false>(w2[j] + w4[j]));
					FOR4 w2[j] = tr<SH>(w2[j] + ((w1[j] + w3[j]) >> 4));
					FOR4 w4[j] = tr<SH>(w4[j] + (w3[j] >> 3));
					if (H == 4) { FOR4 w1[j] = tr<SH>(w1[j] + w2[j] * 3); }
					else { FOR4 { int t = tr<SH>(w0[j] + w2[j]); w1[j] = tr<SH>(w1[j] + (t + (t >> 1))); } }
					FOR4 { int t = tr<SH>(w2[j] + w4[j]); w3[j] = tr<SH>(w3[j] + (t + (t >> 1))); }
				} else {                          // src/lib/wavelet2d.cpp:752-759
					FOR4 w4[j] = tr<SH>(w4[j] - (w3[j] >> 1));
					FOR4 w3[j] = tr<SH>(w3[j] + ((w2[j] + w4[j]) >> 1));
				}
				emit(H - 4, w1); emit(H - 3, w2); emit(H - 2, w3); emit(H - 1, w4);
			} else {                             // rows H-4 .. H-1 in w0..w3
				if constexpr (TRANS == CDF97) {  // src/lib/wavelet2d.cpp:563-571
					FOR4 w3[j] = tr<SH>(w3[j] - 2 * mult08<SH>(w2[j]));
					FOR4 w2[j] = tr<SH>(w2[j] + ((w1[j] + w3[j]) >> 4));
					FOR4 { int t = tr<SH>(w0[j] + w2[j]); w1[j] = tr<SH>(w1[j] + (t + (t >> 1))); }
					FOR4 w3[j] = tr<SH>(w3[j] + w2[j] * 3);
				} else {                          // src/lib/wavelet2d.cpp:749-751
					FOR4 w3[j] = tr<SH>(w3[j] + w2[j]);
				}
				emit(H - 3, w1); emit(H - 2, w2); emit(H - 1, w3);
			}
		}
	}
}

// The fused pixel epilogue (InvArgs::pix): row y's 4 values at columns x..x+3
// -> u8 pixels (k_gray_out8's conversion), and their digest terms
struct PixAcc { unsigned long long s2; uint32_t s1; };
__device__ __forceinline__ void pix_put(const InvArgs<int16_t, int16_t, int16_t>& a, int y, int x, uint2 u, PixAcc& acc)
{
	const int W = a.W;
	const int v[4] = {(int16_t)(u.x & 0xffff), (int)u.x >> 16, (int16_t)(u.y & 0xffff), (int)u.y >> 16};
	uint32_t pk = 0, s = 0, t = 0;
	FOR4 {
		int c = a.pq ? (int16_t)(128 + ((v[j] + 8) >> 4)) : (int16_t)(v[j] + 128);
		c = c < 0 ? 0 : c > 255 ? 255 : c;
		if (x + j >= W) c = 0;
		pk |= (uint32_t)c << (8 * j);
		s += (uint32_t)c;
		t += (uint32_t)c * (uint32_t)j;
	}
	uint8_t* row = a.pix + (long)y * W;
	if (x + 3 < W) *reinterpret_cast<uint32_t*>(row + x) = pk;
	else FOR4 if (x + j < W) row[x + j] = (uint8_t)(pk >> (8 * j));
	acc.s2 += (unsigned long long)((long)y * W + x) * s + t;
	acc.s1 += s;
}

// Inverse 9/7 level, short bands -> short plane, packed (same schedule as inv_seg).
// PIX: a gray frame's level 0 with the pixel output fused (InvArgs::pix)
template <int S, bool FAST, bool PIX = false>
__device__ __forceinline__ void inv97p_seg(const InvArgs<int16_t, int16_t, int16_t>& a, int x, int lane, int y0,
                                           PixAcc* acc = nullptr)
{
	constexpr bool EDGE = !FAST;
	const int W = a.W, H = a.H;
	const EdgeMasks m = edge_masks(x, W);
	const int dxD = (W + 1) >> 1, dxH = W >> 1;
	const bool out_lane = lane >= 1 && lane <= kLanes - 2 && (FAST || x < W);
	const int bx = x >> 1;
	auto emit = [&](int y, const PRow& rw) {
		if (!FAST && (y < y0 || y >= y0 + S || y >= H)) return;
		PRow r = rw;
		row_inv97p<EDGE>(r, m);
		if (!out_lane) return;
		if constexpr (PIX) {
			pix_put(a, y, x, prow_to_u2(r), *acc);
			return;
		}
		int16_t* row = a.out + (long)y * a.po;
		const uint2 u = prow_to_u2(r);
		if (FAST || (a.ovec && x + 3 < W)) {
			*reinterpret_cast<uint2*>(row + x) = u;
		} else {
			const int c[4] = {(int16_t)(u.x & 0xffff), (int)u.x >> 16, (int16_t)(u.y & 0xffff), (int)u.y >> 16};
			FOR4 if (x + j < W) row[x + j] = (int16_t)c[j];
		}
	};
	// FAST: rows y, y+1 inverse-lifted together, written through a running pointer
	int16_t* po = a.out + (long)y0 * a.po + x;
	int ypo = y0;                                        // (PIX: the row po points at)
	auto emit_pair = [&](const PRow& rw0, const PRow& rw1) {
		PRow r0 = rw0, r1 = rw1;
		row_inv97p2<EDGE>(r0, r1, m);
		if constexpr (PIX) {
			if (out_lane) {
				pix_put(a, ypo, x, prow_to_u2(r0), *acc);
				pix_put(a, ypo + 1, x, prow_to_u2(r1), *acc);
			}
			ypo += 2;
			return;
		}
		if (out_lane) {
			*reinterpret_cast<uint2*>(po) = prow_to_u2(r0);
			*reinterpret_cast<uint2*>(po + a.po) = prow_to_u2(r1);
		}
		po += 2 * a.po;
	};
	// band rows of image rows y0-4 .. y0+S+3 (D/H feed even image rows, V/LL
	// odd ones) stream through a ring of PF row pairs, as in fwd97p_seg
	// (S = 2: the 5 pairs in one pass)
	constexpr int NP = (S + 8) / 2, PF = NP % 4 == 0 ? 4 : NP;
	// Ring slots: FAST, the (D, H, V, LL) words of one pair; border waves,
	// the raw elements at clamped band columns, masked when consumed.  Every
	// refill is unconditional, from a wave-uniform clamped band row (the
	// refills past the segment re-read valid rows): a load under a branch,
	// or a select right after it, is waited for at once -- one memory round
	// trip per row pair.  Rows outside the image are never consumed.
	struct ERaw { int d0, d1, h0, h1, v0, v1, l0, l1; };
	using Slot = typename std::conditional<FAST, uint4, ERaw>::type;
	// FAST: two rings, alternate iterations (prefetch depth two iterations);
	// a pass of the loop runs two iterations, so the ring registers are the
	// same at the back-edge and no copy waits for a load in flight
	constexpr int DEPTH = FAST && NP / PF > 1 ? 2 : 1;
	Slot ring[DEPTH][PF];
	int yl = y0 - 4;
	const int byl = FAST ? min((y0 + S + 3) >> 1, (H >> 1) - 1) : 0;
	const int hiD = max(dxD - 1, 0), hiH = max(dxH - 1, 0);
	const int beMax = max(((H + 1) >> 1) - 1, 0), boMax = max((H >> 1) - 1, 0);
	auto load_next = [&](Slot& dst) {
		if constexpr (FAST) {
			const long by = min(yl >> 1, byl);
			dst.x = load_band2<int16_t, false>(a.d[BD] + by * a.p[BD], bx, dxD);
			dst.y = load_band2<int16_t, false>(a.d[BH] + by * a.p[BH], bx, dxH);
			dst.z = load_band2<int16_t, false>(a.d[BV] + by * a.p[BV], bx, dxD);
			dst.w = load_band2<int16_t, false>(a.ll + by * a.pl, bx, dxH);
		} else {
			const int by = yl >> 1;
			const long be = min(max(by, 0), beMax), bo = min(max(by, 0), boMax);
			const int16_t* rD = a.d[BD] + be * a.p[BD];
			const int16_t* rH = a.d[BH] + be * a.p[BH];
			const int16_t* rV = a.d[BV] + bo * a.p[BV];
			const int16_t* rL = a.ll + bo * a.pl;
			const int cD0 = min(max(bx, 0), hiD), cD1 = min(max(bx + 1, 0), hiD);
			const int cH0 = min(max(bx, 0), hiH), cH1 = min(max(bx + 1, 0), hiH);
			dst.d0 = rD[cD0]; dst.d1 = rD[cD1];
			dst.h0 = rH[cH0]; dst.h1 = rH[cH1];
			dst.v0 = rV[cD0]; dst.v1 = rV[cD1];
			dst.l0 = rL[cH0]; dst.l1 = rL[cH1];
		}
		yl += 2;
	};
	// border waves: band columns outside the bands read as 0
	const bool inD0 = bx >= 0 && bx < dxD, inD1 = bx + 1 >= 0 && bx + 1 < dxD;
	const bool inH0 = bx >= 0 && bx < dxH, inH1 = bx + 1 >= 0 && bx + 1 < dxH;
	auto words = [&](const Slot& r) -> uint4 {
		if constexpr (FAST) {
			return make_uint4(deq2(r.x, a.q[BD]), deq2(r.y, a.q[BH]), deq2(r.z, a.q[BV]), deq2(r.w, a.q[BL]));
		} else {
			auto pk = [](bool i0, int a0, bool i1, int a1) {
				return (uint32_t)(uint16_t)(i0 ? a0 : 0) | ((uint32_t)(uint16_t)(i1 ? a1 : 0) << 16);
			};
			return make_uint4(deq2(pk(inD0, r.d0, inD1, r.d1), a.q[BD]), deq2(pk(inH0, r.h0, inH1, r.h1), a.q[BH]),
			                  deq2(pk(inD0, r.v0, inD1, r.v1), a.q[BV]), deq2(pk(inH0, r.l0, inH1, r.l1), a.q[BL]));
		}
	};
#pragma unroll
	for (int d = 0; d < DEPTH; d++) {
#pragma unroll
		for (int j = 0; j < PF; j++) load_next(ring[d][j]);
	}
	const v2s z = {0, 0};
	PRow w0 = {z, z}, w1 = {z, z}, w2 = {z, z}, w3 = {z, z}, w4 = {z, z}, w5 = {z, z}, w6 = {z, z};
	auto pair = [&](int it, int k, Slot& rs) {
		const int i = 2 * (it * PF + k);
		const int e = y0 - 4 + i;
		// take the slot into fresh registers first (FAST: an opaque copy), so
		// the refill can land in the slot's own registers and the loop-carried
		// ring needs no copy at the back-edge (a copy waits for its load)
		Slot slot;
		if constexpr (FAST) slot = opaque_copy(rs);
		else slot = rs;
		load_next(rs);
		if (!FAST && (e < 0 || e >= H)) return;
		const uint4 rr = words(slot);
		w5.e = as_v2(rr.x); w5.o = as_v2(rr.y);
		if (FAST || e + 1 < H) { w6.e = as_v2(rr.z); w6.o = as_v2(rr.w); }
		// U2^-1 at e-1, P2^-1 at e-2, U1^-1 at e-3, P1^-1 at e-4 (src/lib/wavelet2d.cpp:512-561)
		if (FAST || e >= 2) {
			v2s te = w3.e + w5.e, to = w3.o + w5.o;
			w4.e -= (te >> 1) - (te >> 5); w4.o -= (to >> 1) - (to >> 5);
		}
		if (!FAST && e == 2) {
			v2s me = mult08p(w4.e), mo = mult08p(w4.o);
			w3.e -= me + me; w3.o -= mo + mo;
		} else if (FAST || e >= 4) {
			w3.e -= mult08x(w2.e, w4.e); w3.o -= mult08x(w2.o, w4.o);
		}
		if (FAST || e >= 4) { w2.e += avg16(w1.e, w3.e); w2.o += avg16(w1.o, w3.o); }
		if (!FAST && e == 4) { w1.e += mul3(w2.e); w1.o += mul3(w2.o); }
		else if (FAST || e >= 6) {
			v2s te = w0.e + w2.e, to = w0.o + w2.o;
			w1.e += te + (te >> 1); w1.o += to + (to >> 1);
		}
		if (FAST) { if (i >= 8) emit_pair(w1, w2); }
		else { emit(e - 4, w1); emit(e - 3, w2); }
		w0 = w2; w1 = w3; w2 = w4; w3 = w5; w4 = w6;
	};
	auto iteration = [&](int it, Slot (&rg)[PF]) {
#pragma unroll
		for (int k = 0; k < PF; k++) pair(it, k, rg[k]);
	};
	constexpr int NIT = NP / PF;
	if constexpr (DEPTH == 2) {
		int it = 0;
#pragma unroll 1
		for (; it + 1 < NIT; it += 2) {
			iteration(it, ring[0]);
			iteration(it + 1, ring[1]);
		}
		if (it < NIT) iteration(it, ring[0]);
	} else {
#pragma unroll 1
		for (int it = 0; it < NIT; it++) iteration(it, ring[0]);
	}
	if (!FAST && y0 + S + 4 >= H) {
		if (!(H & 1)) {                              // src/lib/wavelet2d.cpp:572-587
			w4.e -= w3.e - (w3.e >> 4); w4.o -= w3.o - (w3.o >> 4);
			w3.e -= mult08x(w2.e, w4.e); w3.o -= mult08x(w2.o, w4.o);
			w2.e += avg16(w1.e, w3.e); w2.o += avg16(w1.o, w3.o);
			w4.e += w3.e >> 3; w4.o += w3.o >> 3;
			if (H == 4) { w1.e += mul3(w2.e); w1.o += mul3(w2.o); }
			else {
				v2s te = w0.e + w2.e, to = w0.o + w2.o;
				w1.e += te + (te >> 1); w1.o += to + (to >> 1);
			}
			v2s te = w2.e + w4.e, to = w2.o + w4.o;
			w3.e += te + (te >> 1); w3.o += to + (to >> 1);
			emit(H - 4, w1); emit(H - 3, w2); emit(H - 2, w3); emit(H - 1, w4);
		} else {                                     // src/lib/wavelet2d.cpp:563-571
			v2s me = mult08p(w2.e), mo = mult08p(w2.o);
			w3.e -= me + me; w3.o -= mo + mo;
			w2.e += avg16(w1.e, w3.e); w2.o += avg16(w1.o, w3.o);
			v2s te = w0.e + w2.e, to = w0.o + w2.o;
			w1.e += te + (te >> 1); w1.o += to + (to >> 1);
			w3.e += mul3(w2.e); w3.o += mul3(w2.o);
			emit(H - 3, w1); emit(H - 2, w2); emit(H - 1, w3);
		}
	}
}

template <int TRANS, typename TB, typename TL, typename TO, int S, bool PIX = false>
__device__ __forceinline__ void inv_body(const InvArgs<TB, TL, TO>& a)
{
	const int lane = threadIdx.x & 63;
	const int seg = blockIdx.y * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: row math stays scalar
	if (seg >= a.nseg) return;
	const int X0 = blockIdx.x * kStripValid - kCols;
	const int x = X0 + lane * kCols;
	const int y0 = seg * S;
	const bool edge = X0 < 0 || X0 + kLanes * kCols >= a.W;
	const bool fast = !edge && a.ovec && !a.nofast && y0 >= 16 && y0 + S + 4 < a.H;
	if constexpr (PIX) {
		static_assert(TRANS == CDF97 && sizeof(TB) == 2 && sizeof(TO) == 2, "the fused pixel output: 9/7 short levels");
		PixAcc acc = {0, 0};
		if (fast) inv97p_seg<S, true, true>(a, x, lane, y0, &acc);
		else inv97p_seg<S, false, true>(a, x, lane, y0, &acc);
		// the wave's digest terms: one atomic per wave into one of the frame's
		// 16 partial words (a single word per frame would take ~8000 atomics)
		unsigned long long d = acc.s2 * 0x9E3779B97F4A7C15ull + acc.s1;
#pragma unroll
		for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
		if (lane == 0 && a.dig) atomicAdd(a.dig + ((seg + blockIdx.x) & 15), d);
		return;
	}
	if constexpr (TRANS == CDF97 && sizeof(TB) == 2 && sizeof(TO) == 2) {
		if (fast) inv97p_seg<S, true>(a, x, lane, y0);
		else inv97p_seg<S, false>(a, x, lane, y0);
	} else {
		if (fast) inv_seg<TRANS, TB, TL, TO, S, true>(a, x, lane, y0);
		else inv_seg<TRANS, TB, TL, TO, S, false>(a, x, lane, y0);
	}
}

template <int TRANS, typename TB, typename TL, typename TO, int S>
__global__ void __launch_bounds__(256) k_inv(InvArgs<TB, TL, TO> a) { inv_body<TRANS, TB, TL, TO, S>(a); }
template <int TRANS, typename TB, typename TL, typename TO, int S, bool PIX = false>
__global__ void __launch_bounds__(256) k_inv_z(const InvArgs<TB, TL, TO>* __restrict__ az)
{
	inv_body<TRANS, TB, TL, TO, S, PIX>(az[blockIdx.z]);
}

// S rows per wave: enough waves to fill the chip on every level, short
// per-wave dependency chains on the small ones.
template <typename T>
int seg_rows(int H)
{
	static const int forced = [] { const char* e = getenv("RIC_DWT_S"); return e ? atoi(e) : 0; }();
	if (forced == 2 || forced == 8 || forced == 16 || ((forced == 32 || forced == 64) && sizeof(T) == 2)) return forced;
	// (16 rather than 32 rows on the 8K level: two rounds of waves balance
	// better, k_inv level 0 44 -> 39 us; 2 rows on the small levels, whose
	// waves are latency-bound: 5 row pairs per wave instead of 8)
	// (tuning knobs RIC_DWT_S16 / RIC_DWT_S2: the height thresholds)
	static const int t16 = [] { const char* e = getenv("RIC_DWT_S16"); return e ? atoi(e) : 2048; }();
	static const int t2 = [] { const char* e = getenv("RIC_DWT_S2"); return e ? atoi(e) : 600; }();
	return H >= t16 ? 16 : H >= t2 ? 8 : 2;
}
// tuning knob: RIC_DWT_NOFAST=1 runs every wave on the checked path
int dbg_nofast()
{
	static const int v = [] { const char* e = getenv("RIC_DWT_NOFAST"); return e ? atoi(e) : 0; }();
	return v;
}

template <int TRANS, typename TI, typename TO, int S>
void fwd_launch_s(const Level& L, const void* src, long sp, char* arena, int vec, hipStream_t st)
{
	FwdArgs<TI, TO> a;
	a.src = (const TI*)src; a.sp = sp; a.W = L.w; a.H = L.h;
	for (int b = 0; b < 4; b++) { a.d[b] = (TO*)(arena + L.b[b].off); a.p[b] = L.b[b].pitch; }
	a.nseg = (L.h + S - 1) / S;
	a.vec = vec;
	a.nofast = dbg_nofast();
	dim3 grid((L.w + kStripValid - 1) / kStripValid, (a.nseg + kWavesPerBlock - 1) / kWavesPerBlock);
	hipLaunchKernelGGL((k_fwd<TRANS, TI, TO, S>), grid, dim3(256), 0, st, a);
}

template <int TRANS, typename TI, typename TO>
void fwd_launch(const Level& L, const void* src, long sp, char* arena, int vec, hipStream_t st)
{
	const int S = seg_rows<TI>(L.h);
	if constexpr (sizeof(TI) == 2) {
		if (S == 64) { fwd_launch_s<TRANS, TI, TO, 64>(L, src, sp, arena, vec, st); return; }
		if (S == 32) { fwd_launch_s<TRANS, TI, TO, 32>(L, src, sp, arena, vec, st); return; }
	}
	if (S == 16) fwd_launch_s<TRANS, TI, TO, 16>(L, src, sp, arena, vec, st);
	else if (S == 2) fwd_launch_s<TRANS, TI, TO, 2>(L, src, sp, arena, vec, st);
	else fwd_launch_s<TRANS, TI, TO, 8>(L, src, sp, arena, vec, st);
}

template <typename TB, typename TO>
InvArgs<TB, TB, TO> inv_args(const Level& L, const Band& lls, char* arena, void* out, long po, const int* q, int S,
                             char* scratch = nullptr, size_t split = 0, size_t lo = 0)
{
	InvArgs<TB, TB, TO> a;
	memset(&a, 0, sizeof a);
	for (int b = 0; b < 4; b++) a.q[b] = q ? q[b] : 1;
	a.ovec = (po % 4 == 0) && ((uintptr_t)out % 16 == 0);
	a.nofast = dbg_nofast();
	// (a compacted pool's level-0 bands are expanded into the scratch arena)
	for (int b = 0; b < 3; b++) {
		a.d[b] = (const TB*)((scratch && L.b[b].off < lo ? scratch : arena) + L.b[b].off);
		a.p[b] = L.b[b].pitch;
	}
	// split arenas (ZFrames): the LL input from scratch when it lies in region C
	a.ll = (const TB*)((scratch && lls.off >= split ? scratch : arena) + lls.off); a.pl = lls.pitch;
	a.out = (TO*)out; a.po = po;
	a.W = L.w; a.H = L.h;
	a.nseg = (L.h + S - 1) / S;
	a.quirk_dalign = L.b[BD].ref_align; a.quirk_halign = L.b[BH].ref_align;
	return a;
}

template <int TRANS, typename TB, typename TO, int S>
void inv_launch_s(const Level& L, const Band& lls, char* arena, void* out, long po, const int* q, hipStream_t st)
{
	InvArgs<TB, TB, TO> a;
	for (int b = 0; b < 4; b++) a.q[b] = q ? q[b] : 1;
	a.ovec = (po % 4 == 0) && ((uintptr_t)out % 16 == 0);
	a.nofast = dbg_nofast();
	for (int b = 0; b < 3; b++) { a.d[b] = (const TB*)(arena + L.b[b].off); a.p[b] = L.b[b].pitch; }
	a.ll = (const TB*)(arena + lls.off); a.pl = lls.pitch;
	a.out = (TO*)out; a.po = po;
	a.W = L.w; a.H = L.h;
	a.nseg = (L.h + S - 1) / S;
	a.quirk_dalign = L.b[BD].ref_align; a.quirk_halign = L.b[BH].ref_align;
	dim3 grid((L.w + kStripValid - 1) / kStripValid, (a.nseg + kWavesPerBlock - 1) / kWavesPerBlock);
	hipLaunchKernelGGL((k_inv<TRANS, TB, TB, TO, S>), grid, dim3(256), 0, st, a);
}

template <int TRANS, typename TB, typename TO>
void inv_launch(const Level& L, const Band& lls, char* arena, void* out, long po, const int* q, hipStream_t st)
{
	const int S = seg_rows<TB>(L.h);
	if constexpr (sizeof(TB) == 2) {
		if (S == 64) { inv_launch_s<TRANS, TB, TO, 64>(L, lls, arena, out, po, q, st); return; }
		if (S == 32) { inv_launch_s<TRANS, TB, TO, 32>(L, lls, arena, out, po, q, st); return; }
	}
	if (S == 16) inv_launch_s<TRANS, TB, TO, 16>(L, lls, arena, out, po, q, st);
	else if (S == 2) inv_launch_s<TRANS, TB, TO, 2>(L, lls, arena, out, po, q, st);
	else inv_launch_s<TRANS, TB, TO, 8>(L, lls, arena, out, po, q, st);
}

template <int TRANS>
void fwd_dispatch(const Level& L, const void* src, long sp, char* arena, int vec, hipStream_t st)
{
	if (!L.in_is_int && !L.is_int) fwd_launch<TRANS, int16_t, int16_t>(L, src, sp, arena, vec, st);
	else if (!L.in_is_int && L.is_int) fwd_launch<TRANS, int16_t, int32_t>(L, src, sp, arena, vec, st);
	else fwd_launch<TRANS, int32_t, int32_t>(L, src, sp, arena, vec, st);
}

template <int TRANS>
void inv_dispatch(const Level& L, const Band& lls, char* arena, void* out, long po, int out_is_int, const int* q, hipStream_t st)
{
	if (!L.is_int) inv_launch<TRANS, int16_t, int16_t>(L, lls, arena, out, po, q, st);
	else if (out_is_int) inv_launch<TRANS, int32_t, int32_t>(L, lls, arena, out, po, q, st);
	else inv_launch<TRANS, int32_t, int16_t>(L, lls, arena, out, po, q, st);
}

}  // namespace

// fault injection (include/ric_gpu.h ric_diag_fault): the consumer waves of
// the next ring-form launches wait for a block row that never comes
std::atomic<int> g_ring_fault{0};
void diag_set_fault(int on) { g_ring_fault.store(on, std::memory_order_relaxed); }

void launch_fwd_level(const Level& L, const void* src, long sp, char* arena, int trans, int vec, hipStream_t st)
{
	if (trans == CDF97) fwd_dispatch<CDF97>(L, src, sp, arena, vec, st);
	else if (trans == CDF53) fwd_dispatch<CDF53>(L, src, sp, arena, vec, st);
	else fwd_dispatch<HAAR>(L, src, sp, arena, vec, st);
}

int fwdq_mode(const Level& L, int trans, const QuantParams& qp, int vec16)
{
	static const bool off = [] { const char* e = getenv("RIC_NOFUSE"); return e && atoi(e) != 0; }();
	// tuning knob: RIC_FQ_GEN_BELOW=h runs levels less than h rows high generically
	static const int gen_below = [] { const char* e = getenv("RIC_FQ_GEN_BELOW"); return e ? atoi(e) : 0; }();
	if (off || trans != CDF97) return FQ_NONE;
	const bool packed = L.h >= gen_below && !L.in_is_int && !L.is_int && vec16 && !dbg_nofast() && L.w % 8 == 0 && L.h % 8 == 0 &&
	                    pk_ok(qp.thres[0]) && pk_ok(qp.thres[1]) && pk_ok(qp.thres[2]);
	return packed ? FQ_PACKED : FQ_GENERIC;
}

namespace {
// The arguments of a fused level launch over one frame's arena.  gen: the
// generic kernel (k_fwdq_gen), else the packed ring forms.
// scratch (split arenas, ZFrames): offsets from P.b_end on (region C) there
FqArgs fq_args(const Pyramid& P, int l, const void* src, long sp, int vec8, int vec16, const QuantParams& qp,
               char* arena, bool gen, char* scratch = nullptr, size_t lo = 0)
{
	const Level& L = P.L[l];
	// (lo: a compacted pool's level-0 bands go to the scratch arena too)
	auto at = [&](size_t off) { return (scratch && (off >= P.b_end || off < lo) ? scratch : arena) + off; };
	FqArgs a;
	memset(&a, 0, sizeof a);   // (padding too: batched launches compare argument images)
	a.wgt = nullptr;
	a.src = (const int16_t*)src; a.sp = sp; a.W = L.w; a.H = L.h; a.nseg = 0;
	a.vec8 = vec8; a.high = l == 0; a.level = l;
	if (gen) {
		a.vec16 = 0; a.nofast = 1;
		a.pk = !L.is_int && pk_ok(qp.thres[0]) && pk_ok(qp.thres[1]) && pk_ok(qp.thres[2]);
	} else {
		a.vec16 = vec16; a.nofast = dbg_nofast(); a.pk = 1;
	}
	for (int b = 0; b < 4; b++) { a.d[b] = (int16_t*)at(L.b[b].off); a.p[b] = L.b[b].pitch; }
	for (int b = 0; b < 3; b++) {
		const Band& B = L.b[b];
		a.dx[b] = B.dx; a.dy[b] = B.dy; a.bw[b] = B.bw(); a.bh[b] = B.bh();
		a.rd[b] = (uint32_t*)at(B.rd_off);
		a.rec[b] = (uint64_t*)at(P.rec_off[l][b]);
		if (l > 0) {
			const Band& C = P.L[l - 1].b[b];
			a.crd[b] = (const uint32_t*)at(C.rd_off); a.cbw[b] = C.bw();
			a.cpin[b] = (uint8_t*)at(P.pin_off[l - 1][b]); a.cpw[b] = C.bw(); a.cph[b] = C.bh();
		} else {
			a.crd[b] = nullptr; a.cbw[b] = 0;
			a.cpin[b] = nullptr; a.cpw[b] = 0; a.cph[b] = 0;
		}
		a.Q[b] = qp.Q[b]; a.iQ[b] = qp.iQ[b];
		for (int i = 0; i < 16; i++) a.thres[b][i] = qp.thres[b][i];
	}
	a.err = (int*)at(P.status_off);
	a.fault = gen ? 0 : g_ring_fault.load(std::memory_order_relaxed);
	return a;
}
}  // namespace

void launch_fwdq_level(const Pyramid& P, int l, const void* src, long sp, int vec8, int vec16, const QuantParams& qp,
                       char* arena, hipStream_t st, int in8)
{
	const Level& L = P.L[l];
	FqArgs a = fq_args(P, l, src, sp, vec8, vec16, qp, arena, false);
	a.in8 = in8 && l == 0;
	if (fq_pc()) { fq_launch_pc(a, st); return; }
	const int S = fq_seg_rows(L.h);
	if (S == 32) fq_launch_s<32>(a, st);
	else if (S == 16) fq_launch_s<16>(a, st);
	else fq_launch_s<8>(a, st);
}

void launch_fwdq_gen_level(const Pyramid& P, int l, const void* src, long sp, int vec8, const QuantParams& qp,
                           int ll_on, int ll_iQ, int ll_T0, char* arena, hipStream_t st)
{
	const Level& L = P.L[l];
	FqArgs a = fq_args(P, l, src, sp, vec8, 0, qp, arena, true);
	static const int gtrace = [] { const char* e = getenv("RIC_LVL_TRACE"); return e ? atoi(e) : -1; }();
	a.wgt = gtrace == l ? fq_wgtrace() : nullptr;
	GenLL ll = {ll_on, ll_iQ, ll_T0};
	const int nseg = (L.h + kGenRows - 1) / kGenRows;
	a.nseg = nseg;
	dim3 grid((L.w + kStripValid - 1) / kStripValid, nseg);   // one workgroup per segment
	if (!L.in_is_int && !L.is_int) hipLaunchKernelGGL((k_fwdq_gen<int16_t, int16_t>), grid, dim3(256), 0, st, a, ll, nseg);
	else if (!L.in_is_int) hipLaunchKernelGGL((k_fwdq_gen<int16_t, int32_t>), grid, dim3(256), 0, st, a, ll, nseg);
	else hipLaunchKernelGGL((k_fwdq_gen<int32_t, int32_t>), grid, dim3(256), 0, st, a, ll, nseg);
}

void launch_inv_level(const Level& L, const Band& lls, char* arena, void* out, long po, int out_is_int,
                      int trans, hipStream_t st, const int* q)
{
	if (trans == CDF97) inv_dispatch<CDF97>(L, lls, arena, out, po, out_is_int, q, st);
	else if (trans == CDF53) inv_dispatch<CDF53>(L, lls, arena, out, po, out_is_int, q, st);
	else inv_dispatch<HAAR>(L, lls, arena, out, po, out_is_int, q, st);
}

// ------------------------------------------------- batched (blockIdx.z) forms
// The frames of a batch sit at fixed strides (arena, level input, output),
// so every launch below is one grid over nz frames, its per-frame arguments
// in a device array (ZArgs) that is only re-uploaded when it changes.
namespace {
uint64_t zargs_hash(const void* data, size_t bytes)
{
	// FNV-1a over 8-byte words (the images are arrays of pointers and ints)
	uint64_t h = 1469598103934665603ull ^ bytes;
	const unsigned char* p = (const unsigned char*)data;
	size_t i = 0;
	for (; i + 8 <= bytes; i += 8) {
		uint64_t w;
		memcpy(&w, p + i, 8);
		h = (h ^ w) * 1099511628211ull;
		h ^= h >> 29;
	}
	for (; i < bytes; i++) h = (h ^ p[i]) * 1099511628211ull;
	return h;
}

// the cache (see ZArgsImage): an image seen before, or a new one while there
// is room; -1 if neither
int zargs_cached(ZArgs& z, const void* data, size_t bytes, hipStream_t st)
{
	static const bool on = [] { const char* e = getenv("RIC_ZARGS_CACHE"); return !e || atoi(e) != 0; }();
	if (!on || bytes > ZArgs::kCacheBlock) return -1;
	const uint64_t h = zargs_hash(data, bytes);
	for (size_t i = 0; i < z.cache.size(); i++) {
		ZArgsImage& e = z.cache[i];
		if (e.hash == h && e.host.size() == bytes && memcmp(e.host.data(), data, bytes) == 0) {
			// (another stream: after the upload)
			if (e.st != st && hipStreamWaitEvent(st, e.ev, 0) != hipSuccess) return -2;
			return (int)i;
		}
	}
	const size_t need = (bytes + 255) & ~(size_t)255;
	if (z.ctotal + need > ZArgs::kCacheBytes) return -1;
	if (z.cdev.empty() || z.cused + need > ZArgs::kCacheBlock) {
		char* d = nullptr;
		char* hb = nullptr;
		if (hipMalloc(&d, ZArgs::kCacheBlock) != hipSuccess) return -2;
		if (hipHostMalloc(&hb, ZArgs::kCacheBlock, 0) != hipSuccess) { (void)dev_free(d); return -2; }
		z.cdev.push_back(d);
		z.chost.push_back(hb);
		z.cused = 0;
	}
	char* d = z.cdev.back() + z.cused;
	char* hb = z.chost.back() + z.cused;
	z.cused += need;
	z.ctotal += need;
	memcpy(hb, data, bytes);          // (the pinned source is never rewritten)
	ZArgsImage e;
	e.hash = h;
	e.dev = d;
	e.host.assign((const char*)data, (const char*)data + bytes);
	e.st = st;
	e.ev = nullptr;
	if (hipEventCreateWithFlags(&e.ev, hipEventDisableTiming) != hipSuccess) return -2;
	if (hipMemcpyAsync(d, hb, bytes, hipMemcpyHostToDevice, st) != hipSuccess) return -2;
	if (hipEventRecord(e.ev, st) != hipSuccess) return -2;
	z.cache.push_back(std::move(e));
	return (int)z.cache.size() - 1;
}
}  // namespace

int zargs_put(ZArgs& z, const void* data, size_t bytes, hipStream_t st)
{
	if (z.ccur >= 0) {
		const ZArgsImage& e = z.cache[z.ccur];
		if (e.host.size() == bytes && memcmp(e.host.data(), data, bytes) == 0) {
			if (e.st != st && hipStreamWaitEvent(st, e.ev, 0) != hipSuccess) return -1;
			return 0;
		}
	}
	if (z.ccur < 0 && z.cur >= 0 && z.img.size() == bytes && memcmp(z.img.data(), data, bytes) == 0) {
		if (z.st != st) {                            // (launches on another stream from here on: stream order)
			if (hipEventRecord(z.ev[z.cur], z.st) != hipSuccess || hipStreamWaitEvent(st, z.ev[z.cur], 0) != hipSuccess) return -1;
			z.st = st;
		}
		return 0;
	}
	{
		const int ci = zargs_cached(z, data, bytes, st);
		if (ci == -2) return -1;
		if (ci >= 0) {
			// leaving the ring's current slot: its launches are all queued, its
			// event follows them (z.cur stays the ring's position)
			if (z.ccur < 0 && z.cur >= 0) {
				if (hipEventRecord(z.ev[z.cur], z.st) != hipSuccess) return -1;
				z.evset[z.cur] = true;
			}
			z.ccur = ci;
			z.dev = z.cache[ci].dev;
			return 0;
		}
	}
	const bool from_cache = z.ccur >= 0;
	z.ccur = -1;
	if (z.cap < bytes) {
		// growth (rare: a larger group): every slot idle first
		if (z.st && hipStreamSynchronize(z.st) != hipSuccess) return -1;
		if (st && hipStreamSynchronize(st) != hipSuccess) return -1;
		if (z.dbase && dev_free(z.dbase) != hipSuccess) return -1;
		if (z.hbase && pinned_free(z.hbase) != hipSuccess) return -1;
		z.dbase = z.hbase = nullptr;
		z.cap = 0;
		z.cur = -1;
		const size_t c = (bytes + 255) & ~(size_t)255;
		if (hipMalloc(&z.dbase, c * ZArgs::kRing) != hipSuccess) return -1;
		if (hipHostMalloc(&z.hbase, c * ZArgs::kRing, 0) != hipSuccess) return -1;
		for (int k = 0; k < ZArgs::kRing; k++) {
			if (!z.ev[k] && hipEventCreateWithFlags(&z.ev[k], hipEventDisableTiming) != hipSuccess) return -1;
			z.evset[k] = false;
		}
		z.cap = c;
	}
	// the current slot's launches are all queued: its event follows them
	// (already recorded when the launches moved to a cached image)
	if (z.cur >= 0 && !from_cache) {
		if (hipEventRecord(z.ev[z.cur], z.st) != hipSuccess) return -1;
		z.evset[z.cur] = true;
	}
	const int k = (z.cur + 1) % ZArgs::kRing;
	if (z.evset[k] && hipEventSynchronize(z.ev[k]) != hipSuccess) return -1;
	z.evset[k] = false;
	char* h = z.hbase + (size_t)k * z.cap;
	char* d = z.dbase + (size_t)k * z.cap;
	memcpy(h, data, bytes);
	if (hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st) != hipSuccess) return -1;
	z.img.assign((const char*)data, (const char*)data + bytes);
	z.cur = k;
	z.st = st;
	z.dev = d;
	return 0;
}

void zargs_free(ZArgs& z)
{
	if (z.st) (void)hipStreamSynchronize(z.st);
	for (ZArgsImage& e : z.cache) {
		if (e.st) (void)hipStreamSynchronize(e.st);
		if (e.ev) (void)hipEventDestroy(e.ev);
	}
	for (char* d : z.cdev) (void)dev_free(d);
	for (char* h : z.chost) (void)pinned_free(h);
	if (z.dbase) (void)dev_free(z.dbase);
	if (z.hbase) (void)pinned_free(z.hbase);
	for (int k = 0; k < ZArgs::kRing; k++)
		if (z.ev[k]) (void)hipEventDestroy(z.ev[k]);
	z = ZArgs();
}

namespace {
// segment rows of the ring forms over nz frames: about one round of resident
// workgroups over the whole batch (tuning knobs RIC_FQZ_SL0..2)
int pc_seg_rows_z(int W, int H, int nz, int level, bool two_rounds = false)
{
	static const int sl[3] = {[] { const char* e = getenv("RIC_FQZ_SL0"); return e ? atoi(e) : 0; }(),
	                          [] { const char* e = getenv("RIC_FQZ_SL1"); return e ? atoi(e) : 0; }(),
	                          [] { const char* e = getenv("RIC_FQZ_SL2"); return e ? atoi(e) : 0; }()};
	if (level < 3 && sl[level] >= 8 && sl[level] % 8 == 0) return sl[level];
	// level 0 (VALU-bound): the single-frame segments (one round per frame,
	// many rounds per batch: the last round's imbalance is amortised; 8K:
	// 72 rows, 63.6 against 72.0 us per frame with 1080-row segments);
	// levels 1-2 (latency-bound chains): one round over the whole batch
	if (level == 0) return pc_seg_rows(W, H);
	const int nstrip = (W + kFqStrip - 1) / kFqStrip;
	// (two_rounds: level 1's one-producer form alone on the chip, measured
	// 19.0-19.3 against 19.4-20.0 us per C3 frame, profiles/r05_level12_sweep.log)
	const int want = std::max(1, kPcResident / (nstrip * nz)) * (two_rounds ? 2 : 1);   // segments per strip per frame
	const int s = ((H + want - 1) / want + 7) / 8 * 8;
	return s < 8 ? 8 : s;
}
}  // namespace

int launch_fwdq_level_z(const Pyramid& P, int l, const ZFrames& fr, int vec8, int vec16, const QuantParams& qp,
                        ZArgs& z, hipStream_t st, int in8)
{
	const Level& L = P.L[l];
	// the one-producer form on level 0 (VALU-bound), two producers above (see
	// fq_launch_pc); knob RIC_FQZ_PC1 = the last level on one producer
	static const int pc1_env = [] { const char* e = getenv("RIC_FQZ_PC1"); return e ? atoi(e) : -1; }();
	const int pc1 = pc1_env >= 0 ? pc1_env : fr.pc1;
	const int S = pc_seg_rows_z(L.w, L.h, fr.nz, l, l == 1 && l <= pc1);
	std::vector<FqArgs> v(fr.nz);
	for (int f = 0; f < fr.nz; f++) {
		v[f] = fq_args(P, l, (const char*)fr.src + f * fr.sstride, fr.sp, vec8, vec16, qp, fr.arena + f * fr.astride, false,
		               fr.scratch ? fr.c_base(f) : nullptr, fr.lo);
		v[f].nseg = (L.h + S - 1) / S;
	}
	if (zargs_put(z, v.data(), v.size() * sizeof(FqArgs), st)) return -1;
	const FqArgs* d = (const FqArgs*)z.dev;
	const dim3 grid((L.w + kFqStrip - 1) / kFqStrip, v[0].nseg, fr.nz);
	// the ring or the double-buffered hand-off (ZFrames::ring; knob
	// RIC_FQZ_ASYNC=0/1 overrides)
	static const int async_env = [] { const char* e = getenv("RIC_FQZ_ASYNC"); return e ? atoi(e) : -1; }();
	const int async = async_env >= 0 ? async_env : fr.ring;
	if (l == 0 && in8 && fr.pix8) {
		if (fr.nz > kPixZ) return -1;
		PixSrc px;
		for (int f = 0; f < kPixZ; f++) px.p[f] = f < fr.nz ? fr.pix8[f] : nullptr;
		px.sp = L.w;
		px.sh = fr.sh8;
		if (async) hipLaunchKernelGGL(k_fwdq_pc_z8<true>, grid, dim3(256), 0, st, d, S, 0, px);
		else hipLaunchKernelGGL(k_fwdq_pc_z8<false>, grid, dim3(256), 0, st, d, S, 0, px);
	}
	else if (l <= pc1 && l == 0 && in8 && !async) hipLaunchKernelGGL((k_fwdq_pc_z<false, false>), grid, dim3(256), 0, st, d, S, 0);
	else if (l <= pc1 && l == 0 && in8) hipLaunchKernelGGL((k_fwdq_pc_z<true, false>), grid, dim3(256), 0, st, d, S, 0);
	else if (l <= pc1) hipLaunchKernelGGL((k_fwdq_pc_z<true, true>), grid, dim3(256), 0, st, d, S, 0);
	else hipLaunchKernelGGL(k_fwdq_pc2_z<true>, grid, dim3(320), 0, st, d, S, 0);
	return 0;
}

int launch_fwdq_gen_level_z(const Pyramid& P, int l, const ZFrames& fr, int vec8, const QuantParams& qp, int ll_on,
                            int ll_iQ, int ll_T0, ZArgs& z, hipStream_t st)
{
	const Level& L = P.L[l];
	// rows per workgroup in a batch (knob RIC_GENZ_ROWS = 8 / 16 / 32): a
	// batch has workgroups to spare, so longer segments (less halo lifting
	// per row, fewer workgroups) than the single frame's 8
	static const int gr_env = [] { const char* e = getenv("RIC_GENZ_ROWS"); return e ? atoi(e) : 0; }();
	const int GR = (gr_env == 8 || gr_env == 16 || gr_env == 32) ? gr_env : 16;
	const int nseg = (L.h + GR - 1) / GR;
	std::vector<FqArgs> v(fr.nz);
	for (int f = 0; f < fr.nz; f++) {
		v[f] = fq_args(P, l, (const char*)fr.src + f * fr.sstride, fr.sp, vec8, 0, qp, fr.arena + f * fr.astride, true,
		               fr.scratch ? fr.c_base(f) : nullptr, fr.lo);
		v[f].nseg = nseg;
	}
	if (zargs_put(z, v.data(), v.size() * sizeof(FqArgs), st)) return -1;
	const FqArgs* d = (const FqArgs*)z.dev;
	const GenLL ll = {ll_on, ll_iQ, ll_T0};
	const dim3 grid((L.w + kStripValid - 1) / kStripValid, nseg, fr.nz);
	auto go = [&](auto gr) {
		constexpr int G = decltype(gr)::value;
		if (!L.in_is_int && !L.is_int) hipLaunchKernelGGL((k_fwdq_gen_z<int16_t, int16_t, G>), grid, dim3(256), 0, st, d, ll, nseg);
		else if (!L.in_is_int) hipLaunchKernelGGL((k_fwdq_gen_z<int16_t, int32_t, G>), grid, dim3(256), 0, st, d, ll, nseg);
		else hipLaunchKernelGGL((k_fwdq_gen_z<int32_t, int32_t, G>), grid, dim3(256), 0, st, d, ll, nseg);
	};
	if (GR == 8) go(std::integral_constant<int, 8>());
	else if (GR == 32) go(std::integral_constant<int, 32>());
	else go(std::integral_constant<int, 16>());
	return 0;
}

namespace {
// rows per inverse wave in a batch (tuning knob RIC_INVZ_S: forced value)
template <typename T>
int inv_seg_rows_z(int H, int nz)
{
	static const int forced = [] { const char* e = getenv("RIC_INVZ_S"); return e ? atoi(e) : 0; }();
	if (forced == 2 || forced == 8 || forced == 16 || ((forced == 32 || forced == 64) && sizeof(T) == 2)) return forced;
	(void)nz;
	// a batch has waves to spare: longer segments (less halo per row) on the
	// short levels below the 8K one (C3, 16 frames: levels 1-3 13.97 / 4.86 /
	// 2.15 -> 12.41 / 4.28 / 1.96 us per frame at 32 rows)
	if (sizeof(T) == 2 && H < 4096) return 32;
	return seg_rows<T>(H);
}

template <int TRANS, typename TB, typename TO, int S>
int inv_launch_z(const Level& L, const Band& lls, const ZFrames& fr, int nz, const int* q, ZArgs& z, hipStream_t st)
{
	std::vector<InvArgs<TB, TB, TO>> v(nz);
	for (int f = 0; f < nz; f++) {
		v[f] = inv_args<TB, TO>(L, lls, fr.arena + f * fr.astride, (char*)fr.out + f * fr.ostride, fr.po,
		                        q ? q + 4 * f : nullptr, S, fr.scratch ? fr.c_base(f) : nullptr, fr.split, fr.lo);
		if (fr.pix) {
			v[f].pix = fr.pix[f];
			v[f].dig = fr.dig_part ? fr.dig_part + 16 * (size_t)f : nullptr;
			v[f].pq = fr.pix_q[f];
		}
	}
	if (zargs_put(z, v.data(), v.size() * sizeof(v[0]), st)) return -1;
	const dim3 grid((L.w + kStripValid - 1) / kStripValid, (v[0].nseg + kWavesPerBlock - 1) / kWavesPerBlock, nz);
	if constexpr (TRANS == CDF97 && sizeof(TB) == 2 && sizeof(TO) == 2) {
		if (fr.pix) {
			hipLaunchKernelGGL((k_inv_z<TRANS, TB, TB, TO, S, true>), grid, dim3(256), 0, st, (const InvArgs<TB, TB, TO>*)z.dev);
			return 0;
		}
	}
	if (fr.pix) return -1;                               // (pix_fusable() refuses these)
	hipLaunchKernelGGL((k_inv_z<TRANS, TB, TB, TO, S>), grid, dim3(256), 0, st, (const InvArgs<TB, TB, TO>*)z.dev);
	return 0;
}

template <int TRANS, typename TB, typename TO>
int inv_launch_zs(const Level& L, const Band& lls, const ZFrames& fr, const int* q, ZArgs& z, hipStream_t st)
{
	const int S = inv_seg_rows_z<TB>(L.h, fr.nz);
	if constexpr (sizeof(TB) == 2) {
		if (S == 64) return inv_launch_z<TRANS, TB, TO, 64>(L, lls, fr, fr.nz, q, z, st);
		if (S == 32) return inv_launch_z<TRANS, TB, TO, 32>(L, lls, fr, fr.nz, q, z, st);
	}
	if (S == 16) return inv_launch_z<TRANS, TB, TO, 16>(L, lls, fr, fr.nz, q, z, st);
	if (S == 2) return inv_launch_z<TRANS, TB, TO, 2>(L, lls, fr, fr.nz, q, z, st);
	return inv_launch_z<TRANS, TB, TO, 8>(L, lls, fr, fr.nz, q, z, st);
}

template <int TRANS>
int inv_dispatch_z(const Level& L, const Band& lls, const ZFrames& fr, int out_is_int, const int* q, ZArgs& z,
                   hipStream_t st)
{
	if (!L.is_int) return inv_launch_zs<TRANS, int16_t, int16_t>(L, lls, fr, q, z, st);
	if (out_is_int) return inv_launch_zs<TRANS, int32_t, int32_t>(L, lls, fr, q, z, st);
	return inv_launch_zs<TRANS, int32_t, int16_t>(L, lls, fr, q, z, st);
}
}  // namespace

int launch_inv_level_z(const Level& L, const Band& lls, const ZFrames& fr, int out_is_int, int trans, const int* q,
                       ZArgs& z, hipStream_t st)
{
	if (trans == CDF97) return inv_dispatch_z<CDF97>(L, lls, fr, out_is_int, q, z, st);
	if (trans == CDF53) return inv_dispatch_z<CDF53>(L, lls, fr, out_is_int, q, z, st);
	return inv_dispatch_z<HAAR>(L, lls, fr, out_is_int, q, z, st);
}

}  // namespace ric

namespace ric {
// diagnostics (include/ric_gpu.h ric_diag_wgtrace): copy the level-0
// workgroup trace of the last k_fwdq_pc launch traced on `device`
int diag_wgtrace(int device, uint64_t* host, int n)
{
	if (hipSetDevice(device) != hipSuccess) return -1;
	uint64_t* b;
	{
		std::lock_guard<std::mutex> g(g_wgtrace_mu);
		b = g_wgtrace[device & 63];
	}
	if (!b) return 0;
	if (n > kWgTraceMax * kWgRec) n = kWgTraceMax * kWgRec;
	if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(host, b, (size_t)n * 8, hipMemcpyDeviceToHost) != hipSuccess)
		return -1;
	return n;
}
}  // namespace ric
