// membench.hip -- DIAGNOSTIC (not product): HBM bandwidth of the access
// pattern of the fused forward level (one wave per 512-column strip x S-row
// segment, 16-byte lane loads, a ring of D rows in flight, one 16-byte store
// per lane per row) against a linear copy.
//   hipcc --offload-arch=gfx950 -O3 scripts/membench.hip -o /tmp/membench && /tmp/membench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, long n)
{
	for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) out[i] = in[i];
}

// one wave per (strip, seg); 4 waves per block = 4 consecutive segments
template <int D>
__global__ void __launch_bounds__(256) k_strip(const uint16_t* __restrict__ in, uint16_t* __restrict__ out, int W, int H,
                                              int S, int nseg, int nstrip)
{
	const int lane = threadIdx.x & 63;
	const int seg = blockIdx.y * 4 + (threadIdx.x >> 6);
	const int strip = blockIdx.x;
	if (seg >= nseg) return;
	const int x = strip * 496 - 8 + lane * 8;
	const int xc = min(max(x, 0), W - 8);
	const int y0 = seg * S;
	const int r0 = max(y0 - 4, 0), r1 = min(y0 + S + 4, H);
	uint4 ring[D];
	const uint16_t* p = in + (long)r0 * W + xc;
#pragma unroll
	for (int j = 0; j < D; j++) ring[j] = *reinterpret_cast<const uint4*>(p + (long)min(r0 + j, H - 1) * 0 + (long)j * W);
	uint4 acc = make_uint4(0, 0, 0, 0);
	int r = r0;
	for (; r + D <= r1; r += D) {
#pragma unroll
		for (int j = 0; j < D; j++) {
			uint4 v = ring[j];
			const int nr = min(r + D + j, H - 1);
			ring[j] = *reinterpret_cast<const uint4*>(in + (long)nr * W + xc);
			acc.x += v.x; acc.y ^= v.y; acc.z += v.z; acc.w ^= v.w;
			if (lane >= 1 && lane <= 62 && r + j >= y0 && r + j < y0 + S)
				*reinterpret_cast<uint4*>(out + (long)(r + j) * W + xc) = acc;
		}
	}
	if (acc.x == 0x12345678u) out[0] = 1;
}

int main()
{
	const int W = 7680, H = 4320;
	const long n = (long)W * H;
	uint16_t *in, *out;
	CK(hipMalloc(&in, n * 2 + 4096));
	CK(hipMalloc(&out, n * 2 + 4096));
	CK(hipMemset(in, 1, n * 2));
	hipEvent_t a, b;
	CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
	auto timeit = [&](auto launch, const char* name, double bytes) {
		for (int i = 0; i < 3; i++) launch();
		hipEventRecord(a);
		const int it = 20;
		for (int i = 0; i < it; i++) launch();
		hipEventRecord(b);
		hipEventSynchronize(b);
		float ms = 0;
		hipEventElapsedTime(&ms, a, b);
		const double us = ms * 1e3 / it;
		printf("%-40s %8.2f us  %7.1f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
	};
	timeit([&] { hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, 0, (const uint4*)in, (uint4*)out, n / 8); },
	       "linear copy 4096x256", 2.0 * n * 2);
	const int nstrip = (W + 495) / 496;
	for (int S : {16, 32, 72}) {
		const int nseg = (H + S - 1) / S;
		char name[64];
		double bytes = 2.0 * n * 2;
		snprintf(name, sizeof name, "strip S=%d D=8 (%d waves)", S, nstrip * nseg);
		timeit([&] { hipLaunchKernelGGL(k_strip<8>, dim3(nstrip, (nseg + 3) / 4), dim3(256), 0, 0, in, out, W, H, S, nseg, nstrip); }, name, bytes);
		snprintf(name, sizeof name, "strip S=%d D=16 (%d waves)", S, nstrip * nseg);
		timeit([&] { hipLaunchKernelGGL(k_strip<16>, dim3(nstrip, (nseg + 3) / 4), dim3(256), 0, 0, in, out, W, H, S, nseg, nstrip); }, name, bytes);
		snprintf(name, sizeof name, "strip S=%d D=4 (%d waves)", S, nstrip * nseg);
		timeit([&] { hipLaunchKernelGGL(k_strip<4>, dim3(nstrip, (nseg + 3) / 4), dim3(256), 0, 0, in, out, W, H, S, nseg, nstrip); }, name, bytes);
	}
	return 0;
}
