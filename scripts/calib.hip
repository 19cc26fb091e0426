// calib.hip -- latency calibration for the DWT design (not part of the product).
//   hipcc --offload-arch=gfx950 -O3 scripts/calib.hip -o /tmp/calib && /tmp/calib
// Prints, for one wave alone on the chip: shader clock, cycles per dependent
// v_pk_add_u16 / v_add_u32 / DPP-mov chain step, and global-load latency
// (pointer chase, cold and warm) -- in cycles and ns.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef short v2s __attribute__((ext_vector_type(2)));

__global__ void k_dep_pk(uint32_t* out, long long* cyc, int n)
{
	v2s a = __builtin_bit_cast(v2s, (uint32_t)threadIdx.x), b = {1, 3};
	long long t0 = clock64();
	for (int i = 0; i < n; i++) {
#pragma unroll
		for (int j = 0; j < 16; j++) a = a + b;
	}
	long long t1 = clock64();
	out[threadIdx.x] = __builtin_bit_cast(uint32_t, a);
	if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_dep_u32(uint32_t* out, long long* cyc, int n)
{
	uint32_t a = threadIdx.x;
	long long t0 = clock64();
	for (int i = 0; i < n; i++) {
#pragma unroll
		for (int j = 0; j < 16; j++) a = (a + 0x9e37u) ^ (a >> 3);
	}
	long long t1 = clock64();
	out[threadIdx.x] = a;
	if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_dep_dpp(uint32_t* out, long long* cyc, int n)
{
	int a = threadIdx.x;
	long long t0 = clock64();
	for (int i = 0; i < n; i++) {
#pragma unroll
		for (int j = 0; j < 16; j++) a = __builtin_amdgcn_update_dpp(0, a, 0x138, 0xF, 0xF, true) + 1;
	}
	long long t1 = clock64();
	out[threadIdx.x] = a;
	if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_chase(const uint32_t* next, long long* cyc, int n, uint32_t* sink)
{
	uint32_t p = 0;
	long long t0 = clock64();
	for (int i = 0; i < n; i++) p = __builtin_nontemporal_load(next + p);
	long long t1 = clock64();
	sink[0] = p;
	cyc[0] = t1 - t0;
}

__global__ void k_spin(long long* cyc, long long ticks)
{
	long long t0 = clock64(), t;
	do { t = clock64(); } while (t - t0 < ticks);
	cyc[0] = t - t0;
}

int main()
{
	uint32_t* out; long long* cyc; uint32_t* next; uint32_t* sink;
	const int N = 1 << 24;   // 64 MB chase table
	hipMalloc(&out, 4096); hipMalloc(&cyc, 64); hipMalloc(&sink, 64); hipMalloc(&next, (size_t)N * 4);
	std::vector<uint32_t> h(N);
	// stride of 4099 elements (16 KB+): every hop a new cache line and page region
	for (int i = 0; i < N; i++) h[i] = (uint32_t)(((long)i + 4099L * 17) % N);
	hipMemcpy(next, h.data(), (size_t)N * 4, hipMemcpyHostToDevice);
	hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
	long long c = 0; float ms = 0;

	// clock: spin 10M ticks, wall time by events
	hipLaunchKernelGGL(k_spin, 1, 64, 0, 0, cyc, 1000000LL);
	hipDeviceSynchronize();
	hipEventRecord(e0); hipLaunchKernelGGL(k_spin, 1, 64, 0, 0, cyc, 20000000LL); hipEventRecord(e1);
	hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
	hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
	const double ghz = c / (ms * 1e6);
	printf("clock64: %lld ticks in %.3f ms -> %.3f GHz (clock64 rate)\n", c, ms, ghz);

	const int n = 4096;
	hipLaunchKernelGGL(k_dep_pk, 1, 64, 0, 0, out, cyc, n); hipDeviceSynchronize();
	hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
	printf("dependent v_pk_add_u16 : %.2f ticks/op\n", (double)c / (n * 16));
	hipLaunchKernelGGL(k_dep_u32, 1, 64, 0, 0, out, cyc, n); hipDeviceSynchronize();
	hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
	printf("dependent add+xor+shr u32: %.2f ticks/step (3 ops)\n", (double)c / (n * 16));
	hipLaunchKernelGGL(k_dep_dpp, 1, 64, 0, 0, out, cyc, n); hipDeviceSynchronize();
	hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
	printf("dependent dpp-mov + add: %.2f ticks/step\n", (double)c / (n * 16));

	const int hops = 2000;
	hipLaunchKernelGGL(k_chase, 1, 64, 0, 0, next, cyc, hops, sink); hipDeviceSynchronize();
	hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
	printf("global load chase (cold-ish, 64MB table): %.1f ticks/hop = %.0f ns\n", (double)c / hops,
	       (double)c / hops / ghz);
	hipLaunchKernelGGL(k_chase, 1, 64, 0, 0, next, cyc, hops, sink); hipDeviceSynchronize();
	hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
	printf("global load chase (second pass): %.1f ticks/hop = %.0f ns\n", (double)c / hops, (double)c / hops / ghz);
	return 0;
}
