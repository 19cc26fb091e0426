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

// ------------------------------------------------------------------ rows
// TransLine97, src/lib/wavelet2d.cpp:320-359, on 4 columns per lane.
// x = absolute column of c[0] (multiple of 4).
template <bool SH, bool EDGE>
__device__ __forceinline__ void row_fwd97(int (&c)[4], int x, int W)
{
	int t, lm, rn;
	lm = __shfl_up(c[3], 1);                                    // P1 (even)
	if (EDGE && x == 0) c[0] = tr<SH>(c[0] - c[1] * 3);
	else if (EDGE && x == W - 1) c[0] = tr<SH>(c[0] - lm * 3);
	else { t = tr<SH>(lm + c[1]); c[0] = tr<SH>(c[0] - (t + (t >> 1))); }
	if (EDGE && x + 2 == W - 1) c[2] = tr<SH>(c[2] - c[1] * 3);
	else { t = tr<SH>(c[1] + c[3]); c[2] = tr<SH>(c[2] - (t + (t >> 1))); }
	rn = __shfl_down(c[0], 1);                                  // U1 (odd)
	if (EDGE && x + 1 == W - 1) c[1] = tr<SH>(c[1] - (c[0] >> 3));
	else c[1] = tr<SH>(c[1] - ((c[0] + c[2]) >> 4));
	if (EDGE && x + 3 == W - 1) c[3] = tr<SH>(c[3] - (c[2] >> 3));
	else c[3] = tr<SH>(c[3] - ((c[2] + rn) >> 4));
	lm = __shfl_up(c[3], 1);                                    // P2 (even)
	if (EDGE && x == 0) c[0] = tr<SH>(c[0] + 2 * mult08<SH>(c[1]));
	else if (EDGE && x == W - 1) c[0] = tr<SH>(c[0] + 2 * mult08<SH>(lm));
	else c[0] = tr<SH>(c[0] + mult08<SH>(lm + c[1]));
	if (EDGE && x + 2 == W - 1) c[2] = tr<SH>(c[2] + 2 * mult08<SH>(c[1]));
	else c[2] = tr<SH>(c[2] + mult08<SH>(c[1] + c[3]));
	rn = __shfl_down(c[0], 1);                                  // U2 (odd)
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
	rn = __shfl_down(c[0], 1);                                  // U2^-1 (odd)
	if (EDGE && x + 1 == W - 1) c[1] = tr<SH>(c[1] - (c[0] - (c[0] >> 4)));
	else { t = tr<SH>(c[0] + c[2]); c[1] = tr<SH>(c[1] - ((t >> 1) - (t >> 5))); }
	if (EDGE && x + 3 == W - 1) c[3] = tr<SH>(c[3] - (c[2] - (c[2] >> 4)));
	else { t = tr<SH>(c[2] + rn); c[3] = tr<SH>(c[3] - ((t >> 1) - (t >> 5))); }
	lm = __shfl_up(c[3], 1);                                    // P2^-1 (even)
	if (EDGE && x == 0) c[0] = tr<SH>(c[0] - 2 * mult08<SH>(c[1]));
	else if (EDGE && x == W - 1) c[0] = tr<SH>(c[0] - 2 * mult08<SH>(lm));
	else c[0] = tr<SH>(c[0] - mult08<SH>(lm + c[1]));
	if (EDGE && x + 2 == W - 1) c[2] = tr<SH>(c[2] - 2 * mult08<SH>(c[1]));
	else c[2] = tr<SH>(c[2] - mult08<SH>(c[1] + c[3]));
	rn = __shfl_down(c[0], 1);                                  // U1^-1 (odd)
	if (EDGE && x + 1 == W - 1) c[1] = tr<SH>(c[1] + (c[0] >> 3));
	else c[1] = tr<SH>(c[1] + ((c[0] + c[2]) >> 4));
	if (EDGE && x + 3 == W - 1) c[3] = tr<SH>(c[3] + (c[2] >> 3));
	else c[3] = tr<SH>(c[3] + ((c[2] + rn) >> 4));
	lm = __shfl_up(c[3], 1);                                    // P1^-1 (even)
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
	int lm = __shfl_up(c[3], 1);                                // P (even)
	if (EDGE && x == 0) c[0] = tr<SH>(c[0] - c[1]);
	else if (EDGE && x == W - 1) c[0] = tr<SH>(c[0] - lm);
	else c[0] = tr<SH>(c[0] - ((lm + c[1]) >> 1));
	if (EDGE && x + 2 == W - 1) c[2] = tr<SH>(c[2] - c[1]);
	else c[2] = tr<SH>(c[2] - ((c[1] + c[3]) >> 1));
	int rn = __shfl_down(c[0], 1);                              // U (odd)
	if (EDGE && x + 1 == W - 1) c[1] = tr<SH>(c[1] + (c[0] >> 1));
	else c[1] = tr<SH>(c[1] + ((c[0] + c[2]) >> 2));
	if (EDGE && x + 3 == W - 1) c[3] = tr<SH>(c[3] + (c[2] >> 1));
	else c[3] = tr<SH>(c[3] + ((c[2] + rn) >> 2));
}

// TransLine53I, src/lib/wavelet2d.cpp:613-634
template <bool SH, bool EDGE>
__device__ __forceinline__ void row_inv53(int (&c)[4], int x, int W)
{
	int rn = __shfl_down(c[0], 1);                              // U^-1 (odd)
	if (EDGE && x + 1 == W - 1) c[1] = tr<SH>(c[1] - (c[0] >> 1));
	else c[1] = tr<SH>(c[1] - ((c[0] + c[2]) >> 2));
	if (EDGE && x + 3 == W - 1) c[3] = tr<SH>(c[3] - (c[2] >> 1));
	else c[3] = tr<SH>(c[3] - ((c[2] + rn) >> 2));
	int lm = __shfl_up(c[3], 1);                                // P^-1 (even)
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

// ---------------------------------------------------------- forward level
template <typename TI, typename TO>
struct FwdArgs {
	const TI* src; long sp;   // input plane + pitch (elements)
	int W, H;
	TO* d[4]; long p[4];      // D, H, V, L outputs + pitches
	int S, nseg, vec;
};

template <int TRANS, typename TI, typename TO, bool EDGE>
__device__ __forceinline__ void fwd_body(const FwdArgs<TI, TO>& a, int x, int lane, int y0)
{
	constexpr bool SH = sizeof(TO) == 2;
	const int W = a.W, H = a.H;
	const bool out_lane = lane >= 1 && lane <= kLanes - 2 && x < W;
	const int bx = x >> 1;
	auto emit = [&](int y, const int (&r)[4]) {
		if (!out_lane || y < y0 || y >= y0 + a.S || y >= H) return;
		int by = y >> 1;
		if (!(y & 1)) {
			store2(a.d[BD] + (long)by * a.p[BD], bx, (W + 1) >> 1, r[0], r[2]);
			store2(a.d[BH] + (long)by * a.p[BH], bx, W >> 1, r[1], r[3]);
		} else {
			store2(a.d[BV] + (long)by * a.p[BV], bx, (W + 1) >> 1, r[0], r[2]);
			store2(a.d[BL] + (long)by * a.p[BL], bx, W >> 1, r[1], r[3]);
		}
	};
	auto fetch = [&](int y, int (&r)[4]) {
		load4(a.src + (long)y * a.sp, x, W, a.vec != 0, r);
		FOR4 r[j] = tr<SH>(r[j]);
		row_fwd<TRANS, SH, EDGE>(r, x, W);
	};

	if constexpr (TRANS == HAAR) {
		// TransformHaar, src/lib/wavelet2d.cpp:788-819: complete row pairs only
		for (int e = y0; e < y0 + a.S && e + 1 < H; e += 2) {
			int r0[4], r1[4];
			fetch(e, r0); fetch(e + 1, r1);
			FOR4 { r0[j] = tr<SH>(r0[j] - r1[j]); r1[j] = tr<SH>(r1[j] + (r0[j] >> 1)); }
			emit(e, r0); emit(e + 1, r1);
		}
		return;
	} else {
		const int ra = y0 >= 4 ? y0 - 4 : 0;
		const int rb = min(y0 + a.S + 4, H);
		int w0[4] = {0, 0, 0, 0}, w1[4] = {0, 0, 0, 0}, w2[4] = {0, 0, 0, 0};
		int w3[4] = {0, 0, 0, 0}, w4[4], w5[4] = {0, 0, 0, 0};
		for (int e = ra; e < rb; e += 2) {
			fetch(e, w4);
			if (e + 1 < H) fetch(e + 1, w5);
			if constexpr (TRANS == CDF97) {
				// P1 at e, U1 at e-1, P2 at e-2, U2 at e-3 (src/lib/wavelet2d.cpp:425-454)
				if (e == 0) { FOR4 w4[j] = tr<SH>(w4[j] - w5[j] * 3); }
				else if (e == H - 1) { FOR4 w4[j] = tr<SH>(w4[j] - w3[j] * 3); }
				else { FOR4 { int t = tr<SH>(w3[j] + w5[j]); w4[j] = tr<SH>(w4[j] - (t + (t >> 1))); } }
				if (e >= 1) { FOR4 w3[j] = tr<SH>(w3[j] - ((w2[j] + w4[j]) >> 4)); }
				if (e == 2) { FOR4 w2[j] = tr<SH>(w2[j] + 2 * mult08<SH>(w3[j])); }
				else if (e >= 4) { FOR4 w2[j] = tr<SH>(w2[j] + mult08<SH>(w1[j] + w3[j])); }
				if (e >= 4) { FOR4 { int t = tr<SH>(w0[j] + w2[j]); w1[j] = tr<SH>(w1[j] + ((t >> 1) - (t >> 5))); } }
			} else {
				// P at e, U at e-1 (src/lib/wavelet2d.cpp:654-668)
				if (e == 0) { FOR4 w4[j] = tr<SH>(w4[j] - w5[j]); }
				else if (e == H - 1) { FOR4 w4[j] = tr<SH>(w4[j] - w3[j]); }
				else { FOR4 w4[j] = tr<SH>(w4[j] - ((w3[j] + w5[j]) >> 1)); }
				if (e >= 1) { FOR4 w3[j] = tr<SH>(w3[j] + ((w2[j] + w4[j]) >> 2)); }
			}
			emit(e - 4, w0); emit(e - 3, w1);
			FOR4 { w0[j] = w2[j]; w1[j] = w3[j]; w2[j] = w4[j]; w3[j] = w5[j]; }
		}
		if (rb == H) {
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

template <int TRANS, typename TI, typename TO>
__global__ void __launch_bounds__(256) k_fwd(FwdArgs<TI, TO> a)
{
	const int lane = threadIdx.x & 63;
	const int seg = blockIdx.y * kWavesPerBlock + (threadIdx.x >> 6);
	if (seg >= a.nseg) return;                       // whole wave exits together
	const int X0 = blockIdx.x * kStripValid - kCols;
	const int x = X0 + lane * kCols;
	const int y0 = seg * a.S;
	const bool edge = X0 < 0 || X0 + kLanes * kCols >= a.W;   // column W-1 inside the wave, halo lanes included
	if (edge) fwd_body<TRANS, TI, TO, true>(a, x, lane, y0);
	else fwd_body<TRANS, TI, TO, false>(a, x, lane, y0);
}

// ---------------------------------------------------------- inverse level
template <typename TB, typename TL, typename TO>
struct InvArgs {
	const TB* d[3]; long p[3];  // D, H, V bands (level type)
	const TL* ll; long pl;      // LL (level type)
	TO* out; long po;           // reconstructed plane (finer level type / image)
	int W, H, S, nseg, ovec;
	int quirk_dalign, quirk_halign;   // reference DimXAlign of D and H (5/3 only)
};

template <int TRANS, typename TB, typename TL, typename TO, bool EDGE>
__device__ __forceinline__ void inv_body(const InvArgs<TB, TL, TO>& a, int x, int lane, int y0)
{
	constexpr bool SH = sizeof(TB) == 2;
	const int W = a.W, H = a.H;
	const int dxD = (W + 1) >> 1, dxH = W >> 1;
	const bool out_lane = lane >= 1 && lane <= kLanes - 2 && x < W;
	const int bx = x >> 1;
	auto fetch = [&](int y, int (&r)[4]) {
		int by = y >> 1;
		if (!(y & 1)) {
			load2(a.d[BD] + (long)by * a.p[BD], bx, dxD, r[0], r[2]);
			if (TRANS == CDF53 && y == 2) {
				// Transform53I reads this H row with the D stride
				// (src/lib/wavelet2d.cpp:715): replay it on the reference layout.
#pragma unroll
				for (int k = 0; k < 2; k++) {
					int b = bx + k, v = 0;
					if (b >= 0 && b < dxH) {
						long f = (long)a.quirk_dalign + b;
						long rr = f / a.quirk_halign, cc = f % a.quirk_halign;
						if (cc < dxH && rr < ((H + 1) >> 1)) v = a.d[BH][rr * a.p[BH] + cc];
					}
					r[1 + 2 * k] = v;
				}
			} else {
				load2(a.d[BH] + (long)by * a.p[BH], bx, dxH, r[1], r[3]);
			}
		} else {
			load2(a.d[BV] + (long)by * a.p[BV], bx, dxD, r[0], r[2]);
			load2(a.ll + (long)by * a.pl, bx, dxH, r[1], r[3]);
		}
		FOR4 r[j] = tr<SH>(r[j]);
	};
	auto emit = [&](int y, const int (&rw)[4]) {
		if (y < y0 || y >= y0 + a.S || y >= H) return;
		int r[4];
		FOR4 r[j] = rw[j];
		row_inv<TRANS, SH, EDGE>(r, x, W);
		if (!out_lane) return;
		TO* row = a.out + (long)y * a.po;
		if (a.ovec && x + 3 < W) {
			if constexpr (sizeof(TO) == 2) {
				uint2 u;
				u.x = (uint32_t)(uint16_t)r[0] | ((uint32_t)(uint16_t)r[1] << 16);
				u.y = (uint32_t)(uint16_t)r[2] | ((uint32_t)(uint16_t)r[3] << 16);
				*reinterpret_cast<uint2*>(row + x) = u;
			} else {
				*reinterpret_cast<int4*>(row + x) = make_int4(r[0], r[1], r[2], r[3]);
			}
		} else {
			FOR4 if (x + j < W) row[x + j] = (TO)r[j];
		}
	};

	if constexpr (TRANS == HAAR) {
		// TransformHaarI, src/lib/wavelet2d.cpp:821-855
		for (int e = y0; e < y0 + a.S && e + 1 < H; e += 2) {
			int r0[4], r1[4];
			fetch(e, r0); fetch(e + 1, r1);
			FOR4 { r1[j] = tr<SH>(r1[j] - (r0[j] >> 1)); r0[j] = tr<SH>(r0[j] + r1[j]); }
			emit(e, r0); emit(e + 1, r1);
		}
		return;
	} else {
		const int ra = y0 >= 4 ? y0 - 4 : 0;
		const int rb = min(y0 + a.S + 4, H);
		int w0[4] = {0, 0, 0, 0}, w1[4] = {0, 0, 0, 0}, w2[4] = {0, 0, 0, 0}, w3[4] = {0, 0, 0, 0};
		int w4[4] = {0, 0, 0, 0}, w5[4], w6[4] = {0, 0, 0, 0};
		// window: w0..w6 = rows e-5 .. e+1
		for (int e = ra; e < rb; e += 2) {
			fetch(e, w5);
			if (e + 1 < H) fetch(e + 1, w6);
			if constexpr (TRANS == CDF97) {
				// U2^-1 at e-1, P2^-1 at e-2, U1^-1 at e-3, P1^-1 at e-4
				// (src/lib/wavelet2d.cpp:512-561)
				if (e >= 2) { FOR4 { int t = tr<SH>(w3[j] + w5[j]); w4[j] = tr<SH>(w4[j] - ((t >> 1) - (t >> 5))); } }
				if (e == 2) { FOR4 w3[j] = tr<SH>(w3[j] - 2 * mult08<SH>(w4[j])); }
				else if (e >= 4) { FOR4 w3[j] = tr<SH>(w3[j] - mult08<SH>(w2[j] + w4[j])); }
				if (e >= 4) { FOR4 w2[j] = tr<SH>(w2[j] + ((w1[j] + w3[j]) >> 4)); }
				if (e == 4) { FOR4 w1[j] = tr<SH>(w1[j] + w2[j] * 3); }
				else if (e >= 6) { FOR4 { int t = tr<SH>(w0[j] + w2[j]); w1[j] = tr<SH>(w1[j] + (t + (t >> 1))); } }
			} else {
				// U^-1 at e-1, P^-1 at e-2 (src/lib/wavelet2d.cpp:712-747)
				if (e >= 2) { FOR4 w4[j] = tr<SH>(w4[j] - ((w3[j] + w5[j]) >> 2)); }
				if (e == 2) { FOR4 w3[j] = tr<SH>(w3[j] + w4[j]); }
				else if (e >= 4) { FOR4 w3[j] = tr<SH>(w3[j] + ((w2[j] + w4[j]) >> 1)); }
			}
			emit(e - 4, w1); emit(e - 3, w2);
			FOR4 { w0[j] = w2[j]; w1[j] = w3[j]; w2[j] = w4[j]; w3[j] = w5[j]; w4[j] = w6[j]; }
		}
		if (rb == H) {
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

template <int TRANS, typename TB, typename TL, typename TO>
__global__ void __launch_bounds__(256) k_inv(InvArgs<TB, TL, TO> a)
{
	const int lane = threadIdx.x & 63;
	const int seg = blockIdx.y * kWavesPerBlock + (threadIdx.x >> 6);
	if (seg >= a.nseg) return;
	const int X0 = blockIdx.x * kStripValid - kCols;
	const int x = X0 + lane * kCols;
	const int y0 = seg * a.S;
	const bool edge = X0 < 0 || X0 + kLanes * kCols >= a.W;   // column W-1 inside the wave, halo lanes included
	if (edge) inv_body<TRANS, TB, TL, TO, true>(a, x, lane, y0);
	else inv_body<TRANS, TB, TL, TO, false>(a, x, lane, y0);
}

int seg_rows(int H) { return H >= 2048 ? 64 : 32; }

template <int TRANS, typename TI, typename TO>
void fwd_launch(const Level& L, const void* src, long sp, char* arena, int vec, hipStream_t st)
{
	FwdArgs<TI, TO> a;
	a.src = (const TI*)src; a.sp = sp; a.W = L.w; a.H = L.h;
	for (int b = 0; b < 4; b++) { a.d[b] = (TO*)(arena + L.b[b].off); a.p[b] = L.b[b].pitch; }
	a.S = seg_rows(L.h);
	a.nseg = (L.h + a.S - 1) / a.S;
	a.vec = vec;
	dim3 grid((L.w + kStripValid - 1) / kStripValid, (a.nseg + kWavesPerBlock - 1) / kWavesPerBlock);
	hipLaunchKernelGGL((k_fwd<TRANS, TI, TO>), grid, dim3(256), 0, st, a);
}

template <int TRANS, typename TB, typename TO>
void inv_launch(const Level& L, const Band& lls, char* arena, void* out, long po, hipStream_t st)
{
	InvArgs<TB, TB, TO> a;
	a.ovec = (po % 4 == 0) && ((uintptr_t)out % 16 == 0);
	for (int b = 0; b < 3; b++) { a.d[b] = (const TB*)(arena + L.b[b].off); a.p[b] = L.b[b].pitch; }
	a.ll = (const TB*)(arena + lls.off); a.pl = lls.pitch;
	a.out = (TO*)out; a.po = po;
	a.W = L.w; a.H = L.h;
	a.S = seg_rows(L.h);
	a.nseg = (L.h + a.S - 1) / a.S;
	a.quirk_dalign = L.b[BD].ref_align; a.quirk_halign = L.b[BH].ref_align;
	dim3 grid((L.w + kStripValid - 1) / kStripValid, (a.nseg + kWavesPerBlock - 1) / kWavesPerBlock);
	hipLaunchKernelGGL((k_inv<TRANS, TB, TB, TO>), grid, dim3(256), 0, st, a);
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
