// image.hip -- caller-side pixel conversions of the ric CLI on the GPU:
// level shift (src/ric/ric.cpp:144-148), RGBtoYCoCg (:76-91), and on decode
// the unshift/clip (:237-240) and YCoCgtoRGB (:93-112).  All arithmetic is the
// reference's `short` arithmetic.
#include <hip/hip_runtime.h>
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

}  // namespace

void launch_pix_in(const uint8_t* pix, int16_t* planes, int w, int h, long po, int channels, int q, hipStream_t st)
{
	dim3 grid((w + 255) / 256, h);
	if (channels == 3) hipLaunchKernelGGL(k_rgb_in, grid, dim3(256), 0, st, pix, planes, w, h, po, q);
	else hipLaunchKernelGGL(k_gray_in, grid, dim3(256), 0, st, pix, planes, w, h, po, q);
}

void launch_pix_out(const int16_t* planes_in, long pi, int w, int h, int channels, int q,
                    uint8_t* pix, int16_t* planes_out, hipStream_t st)
{
	dim3 grid((w + 255) / 256, h);
	if (channels == 3) hipLaunchKernelGGL(k_rgb_out, grid, dim3(256), 0, st, planes_in, pi, w, h, q, pix, planes_out);
	else hipLaunchKernelGGL(k_gray_out, grid, dim3(256), 0, st, planes_in, pi, w, h, q, pix, planes_out);
}

}  // namespace ric
