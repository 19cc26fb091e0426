// tput.hip -- VALU issue-throughput calibration (development tool, not the
// product): per instruction kind, 8 independent chains per wave, 8 waves per
// SIMD on every CU; prints shader cycles per wave-instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 scripts/tput.hip -o scripts/tput.bin && scripts/tput.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define OP8(ins) \
	asm volatile(ins " %0, %0, %8\n\t" ins " %1, %1, %8\n\t" ins " %2, %2, %8\n\t" ins " %3, %3, %8\n\t" \
	             ins " %4, %4, %8\n\t" ins " %5, %5, %8\n\t" ins " %6, %6, %8\n\t" ins " %7, %7, %8" \
	             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b))

template <int K>
__global__ void __launch_bounds__(256) k_tput(uint32_t* out, long long* clk, int n)
{
	uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
	uint32_t b = blockIdx.x | 0x10001;
	long long t0 = __builtin_amdgcn_s_memtime();
	for (int i = 0; i < n; i++) {
		if constexpr (K == 0) OP8("v_add_u32");
		else if constexpr (K == 1) OP8("v_pk_add_u16");
		else if constexpr (K == 2) OP8("v_pk_min_u16");
		else if constexpr (K == 3) OP8("v_xor_b32");
		else if constexpr (K == 4) OP8("v_pk_ashrrev_i16");
		else if constexpr (K == 5) OP8("v_lshlrev_b32");
		else if constexpr (K == 6) OP8("v_pk_sub_u16");
		else if constexpr (K == 7) OP8("v_max_i32");
	}
	long long t1 = __builtin_amdgcn_s_memtime();
	out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
	if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}

template <int K>
void run(const char* name, uint32_t* out, long long* clk, int cus)
{
	const int n = 4096, blocks = cus * 8;             // 8 blocks of 4 waves per CU = 8 waves per SIMD
	hipEvent_t e0, e1;
	hipEventCreate(&e0); hipEventCreate(&e1);
	hipLaunchKernelGGL(k_tput<K>, dim3(blocks), dim3(256), 0, 0, out, clk, 64);
	hipEventRecord(e0);
	hipLaunchKernelGGL(k_tput<K>, dim3(blocks), dim3(256), 0, 0, out, clk, n);
	hipEventRecord(e1);
	hipEventSynchronize(e1);
	float ms;
	hipEventElapsedTime(&ms, e0, e1);
	long long c;
	hipMemcpy(&c, clk, 8, hipMemcpyDeviceToHost);
	// wave-instructions per SIMD: 8 waves x n x 8
	const double per_simd = 8.0 * n * 8;
	printf("%-18s %7.3f ms  wave0 %.0f clk  -> %.2f cycles/wave-instr/SIMD (wave-clock), %.2f GHz\n", name, ms,
	       (double)c, (double)c / per_simd, (double)c / (ms * 1e-3) / 1e9);
}

int main()
{
	int dev = 0, cus = 0;
	hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
	uint32_t* out;
	long long* clk;
	hipMalloc(&out, (size_t)cus * 8 * 256 * 4);
	hipMalloc(&clk, 8);
	printf("CUs %d\n", cus);
	run<0>("v_add_u32", out, clk, cus);
	run<1>("v_pk_add_u16", out, clk, cus);
	run<2>("v_pk_min_u16", out, clk, cus);
	run<3>("v_xor_b32", out, clk, cus);
	run<4>("v_pk_ashrrev_i16", out, clk, cus);
	run<5>("v_lshlrev_b32", out, clk, cus);
	run<6>("v_pk_sub_u16", out, clk, cus);
	run<7>("v_max_i32", out, clk, cus);
	return 0;
}
