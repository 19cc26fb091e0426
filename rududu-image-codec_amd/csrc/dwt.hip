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
#include <cstdlib>
#include "ric_types.h"
#include "ric_kernels.h"

namespace ric {

namespace {

constexpr int kLanes = 64;
constexpr int kCols = 4;                          // columns per lane
constexpr int kStripValid = (kLanes - 2) * kCols; // 248 valid output columns per wave
constexpr int kWavesPerBlock = 4;

template <typename T>
__device__ __forceinline__ void load4(const T* __restrict__ row, int x, int W, bool vec, int (&c)[4])
{
	if (vec && x >= 0 && x + 3 < W) {
		if constexpr (sizeof(T) == 2) {
			uint2 u = *reinterpret_cast<const uint2*>(row + x);
			c[0] = (int16_t)(u.x & 0xffff); c[1] = (int16_t)(u.x >> 16);
			c[2] = (int16_t)(u.y & 0xffff); c[3] = (int16_t)(u.y >> 16);
		} else {
			int4 u = *reinterpret_cast<const int4*>(row + x);
			c[0] = u.x; c[1] = u.y; c[2] = u.z; c[3] = u.w;
		}
	} else {
#pragma unroll
		for (int j = 0; j < 4; j++) c[j] = (x + j >= 0 && x + j < W) ? (int)row[x + j] : 0;
	}
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
	if (bx < 0) { a = b = 0; return; }     // halo lane left of the image
	if (bx + 1 < dx) {
		if constexpr (sizeof(T) == 2) {
			uint32_t u = *reinterpret_cast<const uint32_t*>(row + bx);
			a = (int16_t)(u & 0xffff); b = (int16_t)(u >> 16);
		} else {
			int2 u = *reinterpret_cast<const int2*>(row + bx);
			a = u.x; b = u.y;
		}
	} else {
		a = bx < dx ? (int)row[bx] : 0;
		b = 0;
	}
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
typedef short v2s __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2s as_v2(uint32_t u) { return __builtin_bit_cast(v2s, u); }
__device__ __forceinline__ uint32_t as_u32(v2s v) { return __builtin_bit_cast(uint32_t, v); }
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
	v2s arg = OL + O;
	if (EDGE) arg = sel(m.eAny, sel(m.eL, O, OL), arg);
	v2s mm = mult08p(arg);
	if (EDGE) mm = sel(m.eAny, mm + mm, mm);
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
	v2s arg = OL + O;
	if (EDGE) arg = sel(m.eAny, sel(m.eL, O, OL), arg);
	v2s mm = mult08p(arg);
	if (EDGE) mm = sel(m.eAny, mm + mm, mm);
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
	v2s arg = OL + O, arg2 = PL + P;
	if (EDGE) { arg = sel(m.eAny, sel(m.eL, O, OL), arg); arg2 = sel(m.eAny, sel(m.eL, P, PL), arg2); }
	v2s mm = mult08p(arg), mm2 = mult08p(arg2);
	if (EDGE) { mm = sel(m.eAny, mm + mm, mm); mm2 = sel(m.eAny, mm2 + mm2, mm2); }
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
	v2s arg = OL + O, arg2 = PL + P;
	if (EDGE) { arg = sel(m.eAny, sel(m.eL, O, OL), arg); arg2 = sel(m.eAny, sel(m.eL, P, PL), arg2); }
	v2s mm = mult08p(arg), mm2 = mult08p(arg2);
	if (EDGE) { mm = sel(m.eAny, mm + mm, mm); mm2 = sel(m.eAny, mm2 + mm2, mm2); }
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
#pragma unroll
		for (int i = 0; i < R; i++) {
			const int y = y0 - 4 + i;
			if (FAST || (y >= 0 && y < H)) raw[i] = load_row4<TI, EDGE>(a.src + (long)y * a.sp, x, W, a.vec != 0);
			else raw[i] = RT{};
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
				else if (FAST || e >= 4) { FOR4 w2[j] = tr<SH>(w2[j] + mult08<SH>(w1[j] + w3[j])); }
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
					FOR4 w2[j] = tr<SH>(w2[j] + mult08<SH>(w1[j] + w3[j]));
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
	constexpr int NP = (S + 8) / 2, PF = 4;
	static_assert(NP % PF == 0, "segment rows");
	uint2 ring[2 * PF];
	const int16_t* rp = a.src + (long)(y0 - 4) * a.sp;   // wave-uniform row pointer
	int yl = y0 - 4;
	auto load_next = [&](uint2& dst) {
		if (FAST || (yl >= 0 && yl < H)) dst = load_row4<int16_t, EDGE>(rp, x, W, a.vec != 0);
		else dst = make_uint2(0, 0);
		rp += a.sp; yl++;
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
		const PRow n0 = prow_from_u2(ring[2 * k]), n1 = prow_from_u2(ring[2 * k + 1]);
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
			w2.e += mult08p(w1.e + w3.e); w2.o += mult08p(w1.o + w3.o);
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
			w2.e += mult08p(w1.e + w3.e); w2.o += mult08p(w1.o + w3.o);
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

// ---------------------------------------------------------- inverse level
template <typename TB, typename TL, typename TO>
struct InvArgs {
	const TB* d[3]; long p[3];  // D, H, V bands (level type)
	const TL* ll; long pl;      // LL (level type)
	TO* out; long po;           // reconstructed plane (finer level type / image)
	int W, H, nseg, ovec, nofast;
	int quirk_dalign, quirk_halign;   // reference DimXAlign of D and H (5/3 only)
};

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
	auto unpack_row = [&](const R2& lo, const R2& hi, int (&r)[4]) {
		unpack2<TB>(lo, r[0], r[2]);
		unpack2<TB>(hi, r[1], r[3]);
		FOR4 r[j] = tr<SH>(r[j]);
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
			unpack_row(l0, h0, r0); unpack_row(l1, h1, r1);
			FOR4 { r1[j] = tr<SH>(r1[j] - (r0[j] >> 1)); r0[j] = tr<SH>(r0[j] + r1[j]); }
			emit(e, r0); emit(e + 1, r1);
		}
	} else {
		constexpr int R = S + 8;                 // band rows of image rows y0-4 .. y0+S+3
		R2 rlo[R], rhi[R];
#pragma unroll
		for (int i = 0; i < R; i++) {
			const int y = y0 - 4 + i;
			if (FAST || (y >= 0 && y < H)) load_pair(y, rlo[i], rhi[i]);
			else { rlo[i] = R2{}; rhi[i] = R2{}; }
		}
		int w0[4] = {0, 0, 0, 0}, w1[4] = {0, 0, 0, 0}, w2[4] = {0, 0, 0, 0}, w3[4] = {0, 0, 0, 0};
		int w4[4] = {0, 0, 0, 0}, w5[4], w6[4] = {0, 0, 0, 0};
		// window: w0..w6 = rows e-5 .. e+1
#pragma unroll
		for (int i = 0; i < R; i += 2) {
			const int e = y0 - 4 + i;
			if (!FAST && (e < 0 || e >= H)) continue;
			unpack_row(rlo[i], rhi[i], w5);
			if (FAST || e + 1 < H) unpack_row(rlo[i + 1], rhi[i + 1], w6);
			if constexpr (TRANS == CDF97) {
				// U2^-1 at e-1, P2^-1 at e-2, U1^-1 at e-3, P1^-1 at e-4
				// (src/lib/wavelet2d.cpp:512-561)
				if (FAST || e >= 2) { FOR4 { int t = tr<SH>(w3[j] + w5[j]); w4[j] = tr<SH>(w4[j] - ((t >> 1) - (t >> 5))); } }
				if (!FAST && e == 2) { FOR4 w3[j] = tr<SH>(w3[j] - 2 * mult08<SH>(w4[j])); }
				else if (FAST || e >= 4) { FOR4 w3[j] = tr<SH>(w3[j] - mult08<SH>(w2[j] + w4[j])); }
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
					FOR4 w3[j] = tr<SH>(w3[j] - mult08<SH>(w2[j] + w4[j]));
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

// Inverse 9/7 level, short bands -> short plane, packed (same schedule as inv_seg).
template <int S, bool FAST>
__device__ __forceinline__ void inv97p_seg(const InvArgs<int16_t, int16_t, int16_t>& a, int x, int lane, int y0)
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
	auto emit_pair = [&](const PRow& rw0, const PRow& rw1) {
		PRow r0 = rw0, r1 = rw1;
		row_inv97p2<EDGE>(r0, r1, m);
		if (out_lane) {
			*reinterpret_cast<uint2*>(po) = prow_to_u2(r0);
			*reinterpret_cast<uint2*>(po + a.po) = prow_to_u2(r1);
		}
		po += 2 * a.po;
	};
	// band rows of image rows y0-4 .. y0+S+3 (D/H feed even image rows, V/LL
	// odd ones) stream through a ring of PF row pairs, as in fwd97p_seg
	constexpr int NP = (S + 8) / 2, PF = 4;
	static_assert(NP % PF == 0, "segment rows");
	uint4 ring[PF];                               // (D, H, V, LL) words of one pair
	const long by0 = (y0 - 4) >> 1;
	const int16_t* pD = a.d[BD] + by0 * a.p[BD];
	const int16_t* pH = a.d[BH] + by0 * a.p[BH];
	const int16_t* pV = a.d[BV] + by0 * a.p[BV];
	const int16_t* pL = a.ll + by0 * a.pl;
	int yl = y0 - 4;
	auto load_next = [&](uint4& dst) {
		if (FAST || (yl >= 0 && yl < H)) {
			dst.x = load_band2<int16_t, EDGE>(pD, bx, dxD);
			dst.y = load_band2<int16_t, EDGE>(pH, bx, dxH);
		} else {
			dst.x = 0; dst.y = 0;
		}
		if (FAST || (yl + 1 >= 0 && yl + 1 < H)) {
			dst.z = load_band2<int16_t, EDGE>(pV, bx, dxD);
			dst.w = load_band2<int16_t, EDGE>(pL, bx, dxH);
		} else {
			dst.z = 0; dst.w = 0;
		}
		pD += a.p[BD]; pH += a.p[BH]; pV += a.p[BV]; pL += a.pl; yl += 2;
	};
#pragma unroll
	for (int j = 0; j < PF; j++) load_next(ring[j]);
	const v2s z = {0, 0};
	PRow w0 = {z, z}, w1 = {z, z}, w2 = {z, z}, w3 = {z, z}, w4 = {z, z}, w5 = {z, z}, w6 = {z, z};
#pragma unroll 1
	for (int it = 0; it < NP / PF; it++) {
#pragma unroll
	for (int k = 0; k < PF; k++) {
		const int i = 2 * (it * PF + k);
		const int e = y0 - 4 + i;
		const uint4 rr = ring[k];
		if (!FAST && (e < 0 || e >= H)) { if (it + 1 < NP / PF) load_next(ring[k]); continue; }
		w5.e = as_v2(rr.x); w5.o = as_v2(rr.y);
		if (FAST || e + 1 < H) { w6.e = as_v2(rr.z); w6.o = as_v2(rr.w); }
		if (it + 1 < NP / PF) load_next(ring[k]);
		// U2^-1 at e-1, P2^-1 at e-2, U1^-1 at e-3, P1^-1 at e-4 (src/lib/wavelet2d.cpp:512-561)
		if (FAST || e >= 2) {
			v2s te = w3.e + w5.e, to = w3.o + w5.o;
			w4.e -= (te >> 1) - (te >> 5); w4.o -= (to >> 1) - (to >> 5);
		}
		if (!FAST && e == 2) {
			v2s me = mult08p(w4.e), mo = mult08p(w4.o);
			w3.e -= me + me; w3.o -= mo + mo;
		} else if (FAST || e >= 4) {
			w3.e -= mult08p(w2.e + w4.e); w3.o -= mult08p(w2.o + w4.o);
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
	}
	}
	if (!FAST && y0 + S + 4 >= H) {
		if (!(H & 1)) {                              // src/lib/wavelet2d.cpp:572-587
			w4.e -= w3.e - (w3.e >> 4); w4.o -= w3.o - (w3.o >> 4);
			w3.e -= mult08p(w2.e + w4.e); w3.o -= mult08p(w2.o + w4.o);
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

template <int TRANS, typename TB, typename TL, typename TO, int S>
__global__ void __launch_bounds__(256) k_inv(InvArgs<TB, TL, TO> a)
{
	const int lane = threadIdx.x & 63;
	const int seg = blockIdx.y * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: row math stays scalar
	if (seg >= a.nseg) return;
	const int X0 = blockIdx.x * kStripValid - kCols;
	const int x = X0 + lane * kCols;
	const int y0 = seg * S;
	const bool edge = X0 < 0 || X0 + kLanes * kCols >= a.W;
	const bool fast = !edge && a.ovec && !a.nofast && y0 >= 16 && y0 + S + 4 < a.H;
	if constexpr (TRANS == CDF97 && sizeof(TB) == 2 && sizeof(TO) == 2) {
		if (fast) inv97p_seg<S, true>(a, x, lane, y0);
		else inv97p_seg<S, false>(a, x, lane, y0);
	} else {
		if (fast) inv_seg<TRANS, TB, TL, TO, S, true>(a, x, lane, y0);
		else inv_seg<TRANS, TB, TL, TO, S, false>(a, x, lane, y0);
	}
}

// S rows per wave: enough waves to fill the chip on every level, short
// per-wave dependency chains on the small ones.
template <typename T>
int seg_rows(int H)
{
	static const int forced = [] { const char* e = getenv("RIC_DWT_S"); return e ? atoi(e) : 0; }();
	if (forced == 8 || forced == 16 || ((forced == 32 || forced == 64) && sizeof(T) == 2)) return forced;
	return (sizeof(T) == 2 && H >= 4096) ? 32 : H >= 1024 ? 16 : 8;
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
	else fwd_launch_s<TRANS, TI, TO, 8>(L, src, sp, arena, vec, st);
}

template <int TRANS, typename TB, typename TO, int S>
void inv_launch_s(const Level& L, const Band& lls, char* arena, void* out, long po, hipStream_t st)
{
	InvArgs<TB, TB, TO> a;
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
void inv_launch(const Level& L, const Band& lls, char* arena, void* out, long po, hipStream_t st)
{
	const int S = seg_rows<TB>(L.h);
	if constexpr (sizeof(TB) == 2) {
		if (S == 64) { inv_launch_s<TRANS, TB, TO, 64>(L, lls, arena, out, po, st); return; }
		if (S == 32) { inv_launch_s<TRANS, TB, TO, 32>(L, lls, arena, out, po, st); return; }
	}
	if (S == 16) inv_launch_s<TRANS, TB, TO, 16>(L, lls, arena, out, po, st);
	else inv_launch_s<TRANS, TB, TO, 8>(L, lls, arena, out, po, st);
}

template <int TRANS>
void fwd_dispatch(const Level& L, const void* src, long sp, char* arena, int vec, hipStream_t st)
{
	if (!L.in_is_int && !L.is_int) fwd_launch<TRANS, int16_t, int16_t>(L, src, sp, arena, vec, st);
	else if (!L.in_is_int && L.is_int) fwd_launch<TRANS, int16_t, int32_t>(L, src, sp, arena, vec, st);
	else fwd_launch<TRANS, int32_t, int32_t>(L, src, sp, arena, vec, st);
}

template <int TRANS>
void inv_dispatch(const Level& L, const Band& lls, char* arena, void* out, long po, int out_is_int, hipStream_t st)
{
	if (!L.is_int) inv_launch<TRANS, int16_t, int16_t>(L, lls, arena, out, po, st);
	else if (out_is_int) inv_launch<TRANS, int32_t, int32_t>(L, lls, arena, out, po, st);
	else inv_launch<TRANS, int32_t, int16_t>(L, lls, arena, out, po, st);
}

}  // namespace

void launch_fwd_level(const Level& L, const void* src, long sp, char* arena, int trans, int vec, hipStream_t st)
{
	if (trans == CDF97) fwd_dispatch<CDF97>(L, src, sp, arena, vec, st);
	else if (trans == CDF53) fwd_dispatch<CDF53>(L, src, sp, arena, vec, st);
	else fwd_dispatch<HAAR>(L, src, sp, arena, vec, st);
}

void launch_inv_level(const Level& L, const Band& lls, char* arena, void* out, long po, int out_is_int,
                      int trans, hipStream_t st)
{
	if (trans == CDF97) inv_dispatch<CDF97>(L, lls, arena, out, po, out_is_int, st);
	else if (trans == CDF53) inv_dispatch<CDF53>(L, lls, arena, out, po, out_is_int, st);
	else inv_dispatch<HAAR>(L, lls, arena, out, po, out_is_int, st);
}

}  // namespace ric
