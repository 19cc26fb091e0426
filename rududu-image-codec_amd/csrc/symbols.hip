// symbols.hip -- zerotree symbolisation of one pyramid level on the GPU: one
// lane per 4x4 block of the D, H and V bands, writing the block's record at its
// serpentine scan position (symbols.h, restating the encoder side of
// CBandCodec::tree / block_enum, src/lib/bandcodec.cpp:346-589).
#include <hip/hip_runtime.h>
#include "ric_types.h"
#include "ric_kernels.h"
#include "symbols.h"

namespace ric {

namespace {

__constant__ SymTables kSymDev = RIC_SYM_TABLES_INIT;

struct SArgs {
	const void* band[3];
	const void* par[3];
	uint64_t* rec[3];
	int pitch[3], dx[3], dy[3];
	int ppitch[3], pdx[3], pdy[3];
	int first[4];
	int high;
};

template <typename C, typename P>
__global__ void __launch_bounds__(256) k_blocks(SArgs a, int n)
{
	int gid = blockIdx.x * blockDim.x + threadIdx.x;
	if (gid >= n) return;
	int b = gid >= a.first[2] ? 2 : gid >= a.first[1] ? 1 : 0;
	int s = gid - a.first[b];
	int bx, by;
	scan_block(s, a.dx[b], a.dy[b], bx, by);
	a.rec[b][s] = block_record<C, P>(kSymDev, (const C*)a.band[b], a.pitch[b], a.dx[b], a.dy[b],
	                                 (const P*)a.par[b], a.ppitch[b], a.pdx[b], a.pdy[b], a.high != 0, bx, by);
}

}  // namespace

void launch_blocks_level(const Pyramid& P, int l, char* arena, hipStream_t st)
{
	const Level& L = P.L[l];
	SArgs a;
	int n = 0;
	const bool has_par = l + 1 < P.nlev;
	for (int b = 0; b < 3; b++) {
		const Band& B = L.b[b];
		a.band[b] = arena + B.off; a.pitch[b] = B.pitch; a.dx[b] = B.dx; a.dy[b] = B.dy;
		a.rec[b] = (uint64_t*)(arena + P.rec_off[l][b]);
		if (has_par) {
			const Band& Q = P.L[l + 1].b[b];
			a.par[b] = arena + Q.off; a.ppitch[b] = Q.pitch; a.pdx[b] = Q.dx; a.pdy[b] = Q.dy;
		} else {
			a.par[b] = nullptr; a.ppitch[b] = 0; a.pdx[b] = 0; a.pdy[b] = 0;
		}
		a.first[b] = n;
		n += B.bw() * B.bh();
	}
	a.first[3] = n;
	a.high = l == 0;
	if (n == 0) return;
	dim3 grid((n + 255) / 256);
	const bool pint = has_par ? P.L[l + 1].is_int : L.is_int;
	if (!L.is_int && !pint) hipLaunchKernelGGL((k_blocks<int16_t, int16_t>), grid, dim3(256), 0, st, a, n);
	else if (!L.is_int) hipLaunchKernelGGL((k_blocks<int16_t, int32_t>), grid, dim3(256), 0, st, a, n);
	else hipLaunchKernelGGL((k_blocks<int32_t, int32_t>), grid, dim3(256), 0, st, a, n);
}

}  // namespace ric
