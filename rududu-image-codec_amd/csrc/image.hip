// image.hip -- caller-side pixel conversions of the ric CLI on the GPU:
// level shift (src/ric/ric.cpp:144-148), RGBtoYCoCg (:76-91), and on decode
// the unshift/clip (:237-240) and YCoCgtoRGB (:93-112).  All arithmetic is the
// reference's `short` arithmetic.
#include <hip/hip_runtime.h>
#include <algorithm>
#include "ric_types.h"
#include "ric_image.h"

namespace ric {

namespace {

constexpr int kShift = 4;   // SHIFT, src/ric/ric.cpp:39

__device__ __forceinline__ int16_t clip255(int v) { return (int16_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

__global__ void k_gray_in(const uint8_t* __restrict__ pix, int16_t* __restrict__ out, int w, int h, long po, int q)
{
	int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
	if (x >= w) return;
	int p = pix[(long)y * w + x];
	out[(long)y * po + x] = q ? (int16_t)((p - 128) << kShift) : (int16_t)(p - 128);
}

// planes out: [0] = Y, [1] = Cg, [2] = Co (the coding order of src/ric/ric.cpp:162-168)
__global__ void k_rgb_in(const uint8_t* __restrict__ pix, int16_t* __restrict__ out, int w, int h, long po, int q)
{
	int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
	if (x >= w) return;
	long n = (long)w * h, i = (long)y * w + x;
	int16_t R = pix[i], G = pix[n + i], B = pix[2 * n + i];
	R = (int16_t)(R - B);
	B = (int16_t)(B + (R >> 1));
	G = (int16_t)(G - B);
	B = (int16_t)(B + ((G >> 1) - 128));
	if (q) { R = (int16_t)(R << (kShift - 1)); G = (int16_t)(G << (kShift - 1)); B = (int16_t)(B << kShift); }
	long o = (long)y * po + x, ps = po * h;
	out[o] = B; out[ps + o] = G; out[2 * ps + o] = R;
}

__global__ void k_gray_out(const int16_t* __restrict__ in, long pi, int w, int h, int q,
                           uint8_t* __restrict__ pix, int16_t* __restrict__ planes)
{
	int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
	if (x >= w) return;
	int16_t v = in[(long)y * pi + x];
	if (q == 0) v = (int16_t)(v + 128);
	else v = clip255((int16_t)(128 + ((v + (1 << (kShift - 1))) >> kShift)));
	long i = (long)y * w + x;
	if (planes) planes[i] = v;
	if (pix) pix[i] = (uint8_t)clip255(v);
}

__global__ void k_rgb_out(const int16_t* __restrict__ in, long pi, int w, int h, int q,
                          uint8_t* __restrict__ pix, int16_t* __restrict__ planes)
{
	int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
	if (x >= w) return;
	long o = (long)y * pi + x, ps = pi * h;
	int16_t B = in[o], G = in[ps + o], R = in[2 * ps + o];   // Y, Cg, Co
	if (q) {
		R = (int16_t)((R + (1 << (kShift - 2))) >> (kShift - 1));
		G = (int16_t)((G + (1 << (kShift - 2))) >> (kShift - 1));
		B = (int16_t)((B + (1 << (kShift - 1))) >> kShift);
	}
	B = (int16_t)(B - ((G >> 1) - 128));
	G = (int16_t)(G + B);
	B = (int16_t)(B - (R >> 1));
	R = (int16_t)(R + B);
	if (q) { R = clip255(R); G = clip255(G); B = clip255(B); }
	long n = (long)w * h, i = (long)y * w + x;
	if (planes) { planes[i] = R; planes[n + i] = G; planes[2 * n + i] = B; }
	if (pix) { pix[i] = (uint8_t)clip255(R); pix[n + i] = (uint8_t)clip255(G); pix[2 * n + i] = (uint8_t)clip255(B); }
}

// Vector forms: 8 pixels per thread (8-byte pixel loads / stores, 16-byte
// plane loads / stores), used when every row starts aligned (w % 8 == 0 and
// aligned buffers, checked on the host).  Same arithmetic as the scalar
// kernels above.
__device__ __forceinline__ void unpack8(uint2 u, int (&p)[8])
{
#pragma unroll
	for (int i = 0; i < 4; i++) { p[i] = (u.x >> (8 * i)) & 255; p[4 + i] = (u.y >> (8 * i)) & 255; }
}
__device__ __forceinline__ uint4 pack8s(const int16_t (&v)[8])
{
	return make_uint4((uint16_t)v[0] | ((uint32_t)(uint16_t)v[1] << 16), (uint16_t)v[2] | ((uint32_t)(uint16_t)v[3] << 16),
	                  (uint16_t)v[4] | ((uint32_t)(uint16_t)v[5] << 16), (uint16_t)v[6] | ((uint32_t)(uint16_t)v[7] << 16));
}
__device__ __forceinline__ void unpack8s(uint4 u, int16_t (&v)[8])
{
	const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
	for (int i = 0; i < 4; i++) { v[2 * i] = (int16_t)(w[i] & 0xFFFF); v[2 * i + 1] = (int16_t)(w[i] >> 16); }
}
__device__ __forceinline__ uint2 pack8b(const int16_t (&v)[8])
{
	uint2 r = {0, 0};
#pragma unroll
	for (int i = 0; i < 4; i++) {
		r.x |= (uint32_t)(uint8_t)clip255(v[i]) << (8 * i);
		r.y |= (uint32_t)(uint8_t)clip255(v[4 + i]) << (8 * i);
	}
	return r;
}

__global__ void k_gray_in8(const uint8_t* __restrict__ pix, int16_t* __restrict__ out, int w, long po, int q)
{
	const int x = (blockIdx.x * blockDim.x + threadIdx.x) * 8, y = blockIdx.y;
	if (x >= w) return;
	int p[8];
	unpack8(*reinterpret_cast<const uint2*>(pix + (long)y * w + x), p);
	int16_t v[8];
#pragma unroll
	for (int i = 0; i < 8; i++) v[i] = q ? (int16_t)((p[i] - 128) << kShift) : (int16_t)(p[i] - 128);
	*reinterpret_cast<uint4*>(out + (long)y * po + x) = pack8s(v);
}

__global__ void k_rgb_in8(const uint8_t* __restrict__ pix, int16_t* __restrict__ out, int w, int h, long po, int q)
{
	const int x = (blockIdx.x * blockDim.x + threadIdx.x) * 8, y = blockIdx.y;
	if (x >= w) return;
	const long n = (long)w * h, i0 = (long)y * w + x;
	int r[8], g[8], b[8];
	unpack8(*reinterpret_cast<const uint2*>(pix + i0), r);
	unpack8(*reinterpret_cast<const uint2*>(pix + n + i0), g);
	unpack8(*reinterpret_cast<const uint2*>(pix + 2 * n + i0), b);
	int16_t Y[8], Cg[8], Co[8];
#pragma unroll
	for (int i = 0; i < 8; i++) {
		int16_t R = (int16_t)r[i], G = (int16_t)g[i], B = (int16_t)b[i];
		R = (int16_t)(R - B);
		B = (int16_t)(B + (R >> 1));
		G = (int16_t)(G - B);
		B = (int16_t)(B + ((G >> 1) - 128));
		if (q) { R = (int16_t)(R << (kShift - 1)); G = (int16_t)(G << (kShift - 1)); B = (int16_t)(B << kShift); }
		Y[i] = B; Cg[i] = G; Co[i] = R;
	}
	const long o = (long)y * po + x, ps = po * h;
	*reinterpret_cast<uint4*>(out + o) = pack8s(Y);
	*reinterpret_cast<uint4*>(out + ps + o) = pack8s(Cg);
	*reinterpret_cast<uint4*>(out + 2 * ps + o) = pack8s(Co);
}

constexpr unsigned long long kDigestMul = 0x9E3779B97F4A7C15ull;

// DIG: `rows` rows per workgroup and the frame's output digest (the formula of
// k_digest below, ric_batch_set_digests) taken from the bytes as they are
// written -- no second pass over the frame; one atomic per workgroup
template <bool DIG>
__global__ void k_gray_out8(const int16_t* __restrict__ in, long pi, int w, int h, int q, uint8_t* __restrict__ pix,
                            int16_t* __restrict__ planes, int rows, unsigned long long* dig)
{
	const int x = (blockIdx.x * blockDim.x + threadIdx.x) * 8, y0 = blockIdx.y * rows;
	// the digest sum_k pix[k] (k M + 1) mod 2^64 as M sum_k pix[k] k + sum_k
	// pix[k]: per 8 pixels at k = i0 + i, sum_k pix[k] k = i0 (sum pix) + sum
	// pix[i] i -- one 64-bit product per 8 pixels instead of eight
	unsigned long long s = 0, s2 = 0;
	uint32_t s1 = 0;
	if (x < w) {
		for (int y = y0; y < y0 + rows && y < h; y++) {
			int16_t v[8];
			unpack8s(*reinterpret_cast<const uint4*>(in + (long)y * pi + x), v);
#pragma unroll
			for (int i = 0; i < 8; i++) {
				if (q == 0) v[i] = (int16_t)(v[i] + 128);
				else v[i] = clip255((int16_t)(128 + ((v[i] + (1 << (kShift - 1))) >> kShift)));
			}
			const long i0 = (long)y * w + x;
			if (planes) *reinterpret_cast<uint4*>(planes + i0) = pack8s(v);
			if (pix) *reinterpret_cast<uint2*>(pix + i0) = pack8b(v);
			if (DIG) {
				uint32_t a = 0, t = 0;
#pragma unroll
				for (int i = 0; i < 8; i++) {
					const uint32_t c = (uint8_t)clip255(v[i]);
					a += c;
					t += c * (uint32_t)i;
				}
				s2 += (unsigned long long)i0 * a + t;
				s1 += a;
			}
		}
		if (DIG) s = s2 * kDigestMul + s1;
	}
	if (DIG) {
#pragma unroll
		for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
		__shared__ unsigned long long part[4];
		if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
		__syncthreads();
		if (threadIdx.x == 0) atomicAdd(dig, part[0] + part[1] + part[2] + part[3]);
	}
}

__global__ void k_rgb_out8(const int16_t* __restrict__ in, long pi, int w, int h, int q, uint8_t* __restrict__ pix,
                           int16_t* __restrict__ planes)
{
	const int x = (blockIdx.x * blockDim.x + threadIdx.x) * 8, y = blockIdx.y;
	if (x >= w) return;
	const long o = (long)y * pi + x, ps = pi * h;
	int16_t Bv[8], Gv[8], Rv[8];
	unpack8s(*reinterpret_cast<const uint4*>(in + o), Bv);               // Y
	unpack8s(*reinterpret_cast<const uint4*>(in + ps + o), Gv);          // Cg
	unpack8s(*reinterpret_cast<const uint4*>(in + 2 * ps + o), Rv);      // Co
#pragma unroll
	for (int i = 0; i < 8; i++) {
		int16_t B = Bv[i], G = Gv[i], R = Rv[i];
		if (q) {
			R = (int16_t)((R + (1 << (kShift - 2))) >> (kShift - 1));
			G = (int16_t)((G + (1 << (kShift - 2))) >> (kShift - 1));
			B = (int16_t)((B + (1 << (kShift - 1))) >> kShift);
		}
		B = (int16_t)(B - ((G >> 1) - 128));
		G = (int16_t)(G + B);
		B = (int16_t)(B - (R >> 1));
		R = (int16_t)(R + B);
		if (q) { R = clip255(R); G = clip255(G); B = clip255(B); }
		Rv[i] = R; Gv[i] = G; Bv[i] = B;
	}
	const long n = (long)w * h, i0 = (long)y * w + x;
	if (planes) {
		*reinterpret_cast<uint4*>(planes + i0) = pack8s(Rv);
		*reinterpret_cast<uint4*>(planes + n + i0) = pack8s(Gv);
		*reinterpret_cast<uint4*>(planes + 2 * n + i0) = pack8s(Bv);
	}
	if (pix) {
		*reinterpret_cast<uint2*>(pix + i0) = pack8b(Rv);
		*reinterpret_cast<uint2*>(pix + n + i0) = pack8b(Gv);
		*reinterpret_cast<uint2*>(pix + 2 * n + i0) = pack8b(Bv);
	}
}

bool vec8_ok(const void* pix, const void* planes, const void* planes2, int w, long pitch)
{
	return w % 8 == 0 && pitch % 8 == 0 && ((uintptr_t)pix % 8) == 0 && ((uintptr_t)planes % 16) == 0 &&
	       ((uintptr_t)planes2 % 16) == 0;
}

}  // namespace

void launch_pix_in(const uint8_t* pix, int16_t* planes, int w, int h, long po, int channels, int q, hipStream_t st)
{
	if (vec8_ok(pix, planes, nullptr, w, po)) {
		dim3 grid8((w / 8 + 255) / 256, h);
		if (channels == 3) hipLaunchKernelGGL(k_rgb_in8, grid8, dim3(256), 0, st, pix, planes, w, h, po, q);
		else hipLaunchKernelGGL(k_gray_in8, grid8, dim3(256), 0, st, pix, planes, w, po, q);
		return;
	}
	dim3 grid((w + 255) / 256, h);
	if (channels == 3) hipLaunchKernelGGL(k_rgb_in, grid, dim3(256), 0, st, pix, planes, w, h, po, q);
	else hipLaunchKernelGGL(k_gray_in, grid, dim3(256), 0, st, pix, planes, w, h, po, q);
}

namespace {
// 16 bytes per thread (a 16-byte load where the run is aligned and whole),
// a block sum, one 64-bit atomic add per block
__global__ __launch_bounds__(256) void k_digest(const uint8_t* __restrict__ p, size_t n, unsigned long long* out)
{
	const size_t i0 = ((size_t)blockIdx.x * 256 + threadIdx.x) * 16;
	unsigned long long s = 0;
	if (i0 + 16 <= n && ((uintptr_t)(p + i0) & 15) == 0) {
		const uint4 v = *(const uint4*)(p + i0);
		const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
		for (int k = 0; k < 16; k++) s += (unsigned long long)((w[k >> 2] >> (8 * (k & 3))) & 255u) * ((i0 + k) * kDigestMul + 1);
	} else {
		for (size_t i = i0; i < i0 + 16 && i < n; i++) s += (unsigned long long)p[i] * (i * kDigestMul + 1);
	}
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
	__shared__ unsigned long long part[4];
	if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
	__syncthreads();
	if (threadIdx.x == 0) atomicAdd(out, part[0] + part[1] + part[2] + part[3]);
}
}  // namespace

namespace {
// ric_device_digests: one launch over a gather chunk's streams (blockIdx.y =
// run), each workgroup striding over its run 16 bytes per thread; the run's
// workgroups reduce through one 64-bit atomic each into a zeroed word
struct DigestRuns {
	const uint8_t* base;
	size_t off[kDigestRuns], len[kDigestRuns];
};
__global__ __launch_bounds__(256) void k_digests(DigestRuns r, unsigned long long* out)
{
	const int run = (int)blockIdx.y;
	const size_t n = r.len[run];
	const uint8_t* p = r.base + r.off[run];
	unsigned long long s = 0;
	for (size_t i0 = ((size_t)blockIdx.x * 256 + threadIdx.x) * 16; i0 < n; i0 += (size_t)gridDim.x * 256 * 16) {
		if (i0 + 16 <= n && ((uintptr_t)(p + i0) & 15) == 0) {
			const uint4 v = *(const uint4*)(p + i0);
			const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
			for (int k = 0; k < 16; k++) s += (unsigned long long)((w[k >> 2] >> (8 * (k & 3))) & 255u) * ((i0 + k) * kDigestMul + 1);
		} else {
			for (size_t i = i0; i < i0 + 16 && i < n; i++) s += (unsigned long long)p[i] * (i * kDigestMul + 1);
		}
	}
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
	__shared__ unsigned long long part[4];
	if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
	__syncthreads();
	if (threadIdx.x == 0 && (part[0] | part[1] | part[2] | part[3])) atomicAdd(out + run, part[0] + part[1] + part[2] + part[3]);
}
}  // namespace

void launch_digests(const uint8_t* base, const size_t* off, const size_t* len, int n, unsigned long long* out, hipStream_t st)
{
	if (n <= 0) return;
	DigestRuns r;
	r.base = base;
	size_t mx = 0;
	for (int i = 0; i < kDigestRuns; i++) {
		r.off[i] = i < n ? off[i] : 0;
		r.len[i] = i < n ? len[i] : 0;
		mx = std::max(mx, r.len[i]);
	}
	if (!mx) return;
	// at most 64 workgroups per run (a 64 MiB chunk of 64 streams: 4096)
	const size_t gx = std::min<size_t>(64, (mx + 16 * 256 - 1) / (16 * 256));
	hipLaunchKernelGGL(k_digests, dim3((unsigned)gx, (unsigned)n), dim3(256), 0, st, r, out);
}

__global__ void k_digest_fold(const unsigned long long* __restrict__ part, unsigned long long* __restrict__ out, int n)
{
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	unsigned long long s = 0;
#pragma unroll
	for (int k = 0; k < 16; k++) s += part[16 * (size_t)i + k];
	out[i] = s;
}

void launch_digest_fold(const unsigned long long* part, unsigned long long* out, int n, hipStream_t st)
{
	if (n <= 0) return;
	hipLaunchKernelGGL(k_digest_fold, dim3((n + 63) / 64), dim3(64), 0, st, part, out, n);
}

void launch_digest(const uint8_t* p, size_t n, unsigned long long* out, hipStream_t st)
{
	if (!n) return;
	const size_t blocks = (n + 16 * 256 - 1) / (16 * 256);
	hipLaunchKernelGGL(k_digest, dim3((unsigned)blocks), dim3(256), 0, st, p, n, out);
}

void launch_pix_out(const int16_t* planes_in, long pi, int w, int h, int channels, int q,
                    uint8_t* pix, int16_t* planes_out, hipStream_t st, unsigned long long* dig)
{
	if (vec8_ok(pix, planes_in, planes_out, w, pi)) {
		dim3 grid8((w / 8 + 255) / 256, h);
		if (channels == 3) {
			hipLaunchKernelGGL(k_rgb_out8, grid8, dim3(256), 0, st, planes_in, pi, w, h, q, pix, planes_out);
		} else if (dig && pix) {
			constexpr int kRows = 16;
			hipLaunchKernelGGL(k_gray_out8<true>, dim3(grid8.x, (h + kRows - 1) / kRows), dim3(256), 0, st, planes_in, pi, w, h,
			                   q, pix, planes_out, kRows, dig);
			return;
		} else {
			hipLaunchKernelGGL(k_gray_out8<false>, grid8, dim3(256), 0, st, planes_in, pi, w, h, q, pix, planes_out, 1,
			                   (unsigned long long*)nullptr);
		}
		if (dig && pix) launch_digest(pix, (size_t)w * h * channels, dig, st);
		return;
	}
	dim3 grid((w + 255) / 256, h);
	if (channels == 3) hipLaunchKernelGGL(k_rgb_out, grid, dim3(256), 0, st, planes_in, pi, w, h, q, pix, planes_out);
	else hipLaunchKernelGGL(k_gray_out, grid, dim3(256), 0, st, planes_in, pi, w, h, q, pix, planes_out);
	if (dig && pix) launch_digest(pix, (size_t)w * h * channels, dig, st);
}

}  // namespace ric
