// quant.hip -- per-band RD quantiser + zerotree significance (buildTree), the
// LL dead-zone quantiser and the dequantiser, hand-written for gfx950.
//
// k_quant_level restates CBandCodec::buildTree / tsuqBlock / makeThres
// (src/lib/bandcodec.cpp:149-319) for the D, H and V bands of one level: one
// lane per 4x4 block, the 16 coefficients held in registers (quant_block.h).
// Levels run finest -> coarsest because a parent's significance adds its four
// children's pRD (bandcodec.cpp:267-269).  It serves the levels the fused
// forward+quantiser (dwt.hip k_fwdq) does not cover.
#include <hip/hip_runtime.h>
#include "ric_types.h"
#include "ric_kernels.h"
#include "quant_block.h"

namespace ric {

namespace {

struct QArgs {
	void* band[3];
	int pitch[3], dx[3], dy[3], bw[3];
	int first[4];                 // block-index prefix over D, H, V
	uint32_t* rd[3];
	const uint32_t* crd[3];       // children pRD (nullptr at the finest level)
	int cbw[3];
	int Q[3], iQ[3];
	int thres[3][16];
};

template <typename T>
__global__ void __launch_bounds__(256) k_quant_level(QArgs a, int nblk)
{
	constexpr bool SH = sizeof(T) == 2;
	__shared__ int s_thres[3][16];
	if (threadIdx.x < 48) s_thres[threadIdx.x / 16][threadIdx.x % 16] = a.thres[threadIdx.x / 16][threadIdx.x % 16];
	__syncthreads();
	int gid = blockIdx.x * blockDim.x + threadIdx.x;
	if (gid >= nblk) return;
	int b = gid >= a.first[2] ? 2 : gid >= a.first[1] ? 1 : 0;
	int k = gid - a.first[b];
	int bwid = a.bw[b];
	int kx = k % bwid, ky = k / bwid;
	int x0 = kx * 4, y0 = ky * 4;
	int dx = a.dx[b], dy = a.dy[b], pitch = a.pitch[b];
	int Q = a.Q[b], iQ = a.iQ[b];
	T* base = (T*)a.band[b] + (long)y0 * pitch + x0;
	uint32_t dist;

	if (x0 + 4 <= dx && y0 + 4 <= dy) {
		// tsuqBlock (RD), src/lib/bandcodec.cpp:159-213
		int v[16];
#pragma unroll
		for (int r = 0; r < 4; r++) {
			if constexpr (SH) {
				uint2 u = *reinterpret_cast<const uint2*>(base + (long)r * pitch);
				v[4 * r + 0] = (int16_t)(u.x & 0xffff); v[4 * r + 1] = (int16_t)(u.x >> 16);
				v[4 * r + 2] = (int16_t)(u.y & 0xffff); v[4 * r + 3] = (int16_t)(u.y >> 16);
			} else {
				int4 u = *reinterpret_cast<const int4*>(base + (long)r * pitch);
				v[4 * r + 0] = u.x; v[4 * r + 1] = u.y; v[4 * r + 2] = u.z; v[4 * r + 3] = u.w;
			}
		}
		int cnt = tsuq_full<SH>(v, Q, iQ, s_thres[b]);
		uint64_t d = (uint64_t)cnt;
		if (a.crd[b]) {
			const uint32_t* c0 = a.crd[b] + (long)(2 * ky) * a.cbw[b];
			const uint32_t* c1 = c0 + a.cbw[b];
			d += (uint32_t)(c0[2 * kx] + c0[2 * kx + 1] + c1[2 * kx] + c1[2 * kx + 1]);
		}
		dist = d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
		if (dist == 0) v[0] = kInsignif;
#pragma unroll
		for (int r = 0; r < 4; r++) {
			if constexpr (SH) {
				uint2 u;
				u.x = (uint32_t)(uint16_t)v[4 * r] | ((uint32_t)(uint16_t)v[4 * r + 1] << 16);
				u.y = (uint32_t)(uint16_t)v[4 * r + 2] | ((uint32_t)(uint16_t)v[4 * r + 3] << 16);
				*reinterpret_cast<uint2*>(base + (long)r * pitch) = u;
			} else {
				*reinterpret_cast<int4*>(base + (long)r * pitch) = make_int4(v[4 * r], v[4 * r + 1], v[4 * r + 2], v[4 * r + 3]);
			}
		}
	} else {
		// edge tsuqBlock, src/lib/bandcodec.cpp:215-237 (children ignored)
		int wdt = min(4, dx - x0), hgt = min(4, dy - y0);
		int v[16];
#pragma unroll
		for (int i = 0; i < 16; i++) v[i] = ((i >> 2) < hgt && (i & 3) < wdt) ? (int)base[(long)(i >> 2) * pitch + (i & 3)] : 0;
		int cnt = tsuq_edge<SH>(v, wdt, hgt, Q, iQ);
		for (int r = 0; r < hgt; r++)
			for (int c = 0; c < wdt; c++) base[(long)r * pitch + c] = (T)v[4 * r + c];
		dist = (uint32_t)cnt;
		if (dist == 0) *base = (T)kInsignif;
	}
	a.rd[b][(long)ky * bwid + kx] = dist;
}

template <typename T>
__global__ void k_quant_ll(T* p, int pitch, int dx, int dy, int iQ, int T0)
{
	constexpr bool SH = sizeof(T) == 2;
	int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= dx * dy) return;
	T* q = p + (long)(i / dx) * pitch + i % dx;
	int v = *q;
	if ((uint32_t)(v + T0) <= (uint32_t)(2 * T0)) *q = 0;
	else *q = (T)tr<SH>((int)((uint32_t)v * (uint32_t)iQ + 32768u) >> 16);
}

// CBand::TSUQ (src/lib/band.h:65-92) on one band, with the Count accumulated
template <typename T>
__global__ void k_tsuq(T* p, int pitch, int dx, int dy, int iQ, int T0, unsigned int* count)
{
	constexpr bool SH = sizeof(T) == 2;
	int i = blockIdx.x * blockDim.x + threadIdx.x;
	unsigned nz = 0;
	if (i < dx * dy) {
		T* q = p + (long)(i / dx) * pitch + i % dx;
		int v = *q;
		if ((uint32_t)(v + T0) <= (uint32_t)(2 * T0)) *q = 0;
		else { *q = (T)tr<SH>((int)((uint32_t)v * (uint32_t)iQ + 32768u) >> 16); nz = 1; }
	}
	unsigned long long b = __ballot(nz);
	if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (unsigned)__popcll(b));
}

template <typename T>
__global__ void k_dequant(T* p, int pitch, int dx, int dy, int q)
{
	constexpr bool SH = sizeof(T) == 2;
	int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= dx * dy) return;
	T* e = p + (long)(i / dx) * pitch + i % dx;
	*e = (T)tr<SH>((int)((uint32_t)(int)*e * (uint32_t)q));
}

// CBand::TSUQ on one band with its statistics (band.h:65-92): stats[0] +=
// the non-zero count, stats[1] = max(stats[1], quantised value), stats[2] =
// min(...), over the values the reference compares (the stored C value).
template <typename T>
__global__ __launch_bounds__(256) void k_band_tsuq(T* p, int pitch, int dx, int dy, int iQ, int T0, int* stats)
{
	constexpr bool SH = sizeof(T) == 2;
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	unsigned nz = 0;
	int mx = 0, mn = 0;
	if (i < dx * dy) {
		T* q = p + (long)(i / dx) * pitch + i % dx;
		const int v = *q;
		if ((uint32_t)(v + T0) <= (uint32_t)(2 * T0)) *q = 0;
		else {
			const int r = tr<SH>((int)((uint32_t)v * (uint32_t)iQ + 32768u) >> 16);
			*q = (T)r;
			nz = 1; mx = r > 0 ? r : 0; mn = r < 0 ? r : 0;
		}
	}
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) {
		mx = max(mx, __shfl_xor(mx, o, 64));
		mn = min(mn, __shfl_xor(mn, o, 64));
	}
	const unsigned long long b = __ballot(nz);
	if ((threadIdx.x & 63) == 0) {
		if (b) atomicAdd(stats, (int)__popcll(b));
		if (mx) atomicMax(stats + 1, mx);
		if (mn) atomicMin(stats + 2, mn);
	}
}

// CBand::Mean's sums (band.h:116-132): Sum of the values (int64), SSum of
// their squares as the reference computes them (an int product, wrapping)
template <typename T>
__global__ __launch_bounds__(256) void k_band_sums(const T* p, int pitch, int dx, int dy, unsigned long long* out)
{
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	long long s = 0, ss = 0;
	if (i < dx * dy) {
		const int v = p[(long)(i / dx) * pitch + i % dx];
		s = v;
		ss = (int)((uint32_t)v * (uint32_t)v);
	}
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) {
		s += __shfl_xor(s, o, 64);
		ss += __shfl_xor(ss, o, 64);
	}
	if ((threadIdx.x & 63) == 0) {
		atomicAdd(out, (unsigned long long)s);
		atomicAdd(out + 1, (unsigned long long)ss);
	}
}

// CBand::Add (band.h:135-141): every sample of the band's rows, padding included
template <typename T>
__global__ __launch_bounds__(256) void k_band_add(T* p, long n, int val)
{
	constexpr bool SH = sizeof(T) == 2;
	const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) p[i] = (T)tr<SH>((int)((uint32_t)(int)p[i] + (uint32_t)val));
}

}  // namespace

void launch_band_tsuq(const Band& B, int iQ, int T0, char* arena, int* stats, hipStream_t st)
{
	const int n = B.dx * B.dy;
	if (n == 0) return;
	const dim3 grid((n + 255) / 256);
	if (B.is_int) hipLaunchKernelGGL(k_band_tsuq<int32_t>, grid, dim3(256), 0, st, (int32_t*)(arena + B.off), B.pitch, B.dx, B.dy, iQ, T0, stats);
	else hipLaunchKernelGGL(k_band_tsuq<int16_t>, grid, dim3(256), 0, st, (int16_t*)(arena + B.off), B.pitch, B.dx, B.dy, iQ, T0, stats);
}

void launch_band_sums(const Band& B, const char* arena, unsigned long long* out, hipStream_t st)
{
	const int n = B.dx * B.dy;
	if (n == 0) return;
	const dim3 grid((n + 255) / 256);
	if (B.is_int) hipLaunchKernelGGL(k_band_sums<int32_t>, grid, dim3(256), 0, st, (const int32_t*)(arena + B.off), B.pitch, B.dx, B.dy, out);
	else hipLaunchKernelGGL(k_band_sums<int16_t>, grid, dim3(256), 0, st, (const int16_t*)(arena + B.off), B.pitch, B.dx, B.dy, out);
}

void launch_band_add(const Band& B, int val, char* arena, hipStream_t st)
{
	const long n = (long)B.pitch * B.dy;
	if (n == 0) return;
	const dim3 grid((unsigned)((n + 255) / 256));
	if (B.is_int) hipLaunchKernelGGL(k_band_add<int32_t>, grid, dim3(256), 0, st, (int32_t*)(arena + B.off), n, val);
	else hipLaunchKernelGGL(k_band_add<int16_t>, grid, dim3(256), 0, st, (int16_t*)(arena + B.off), n, val);
}

void launch_quant_level(const Pyramid& P, int l, const QuantParams& qp, char* arena, hipStream_t st)
{
	const Level& L = P.L[l];
	QArgs a;
	int n = 0;
	for (int b = 0; b < 3; b++) {
		const Band& B = L.b[b];
		a.band[b] = arena + B.off;
		a.pitch[b] = B.pitch; a.dx[b] = B.dx; a.dy[b] = B.dy; a.bw[b] = B.bw();
		a.first[b] = n; n += B.bw() * B.bh();
		a.rd[b] = (uint32_t*)(arena + B.rd_off);
		if (l > 0) {
			const Band& C = P.L[l - 1].b[b];
			a.crd[b] = (const uint32_t*)(arena + C.rd_off);
			a.cbw[b] = C.bw();
		} else {
			a.crd[b] = nullptr; a.cbw[b] = 0;
		}
		a.Q[b] = qp.Q[b]; a.iQ[b] = qp.iQ[b];
		for (int i = 0; i < 16; i++) a.thres[b][i] = qp.thres[b][i];
	}
	a.first[3] = n;
	if (n == 0) return;
	dim3 grid((n + 255) / 256);
	if (L.is_int) hipLaunchKernelGGL(k_quant_level<int32_t>, grid, dim3(256), 0, st, a, n);
	else hipLaunchKernelGGL(k_quant_level<int16_t>, grid, dim3(256), 0, st, a, n);
}

void launch_quant_ll(const Pyramid& P, int Q, int iQ, int T0, char* arena, hipStream_t st)
{
	const Band& B = P.L[P.nlev - 1].b[BL];
	(void)Q;
	int n = B.dx * B.dy;
	if (n == 0) return;
	dim3 grid((n + 255) / 256);
	if (B.is_int) hipLaunchKernelGGL(k_quant_ll<int32_t>, grid, dim3(256), 0, st, (int32_t*)(arena + B.off), B.pitch, B.dx, B.dy, iQ, T0);
	else hipLaunchKernelGGL(k_quant_ll<int16_t>, grid, dim3(256), 0, st, (int16_t*)(arena + B.off), B.pitch, B.dx, B.dy, iQ, T0);
}

void launch_tsuq_band(const Band& B, int iQ, int T0, char* arena, unsigned int* count, hipStream_t st)
{
	int n = B.dx * B.dy;
	if (n == 0) return;
	dim3 grid((n + 255) / 256);
	if (B.is_int) hipLaunchKernelGGL(k_tsuq<int32_t>, grid, dim3(256), 0, st, (int32_t*)(arena + B.off), B.pitch, B.dx, B.dy, iQ, T0, count);
	else hipLaunchKernelGGL(k_tsuq<int16_t>, grid, dim3(256), 0, st, (int16_t*)(arena + B.off), B.pitch, B.dx, B.dy, iQ, T0, count);
}

void launch_dequant_band(const Band& B, int q, char* arena, hipStream_t st)
{
	int n = B.dx * B.dy;
	if (n == 0) return;
	dim3 grid((n + 255) / 256);
	if (B.is_int) hipLaunchKernelGGL(k_dequant<int32_t>, grid, dim3(256), 0, st, (int32_t*)(arena + B.off), B.pitch, B.dx, B.dy, q);
	else hipLaunchKernelGGL(k_dequant<int16_t>, grid, dim3(256), 0, st, (int16_t*)(arena + B.off), B.pitch, B.dx, B.dy, q);
}

}  // namespace ric
