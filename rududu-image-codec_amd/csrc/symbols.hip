// symbols.hip -- zerotree symbolisation on the GPU for the levels the fused
// forward+quantiser (dwt.hip k_fwdq) does not cover: one lane per 4x4 block of
// the D, H and V bands of one level, writing the block-local record and/or the
// parent info (symbols.h), both in raster block order.  Restates the encoder
// side of CBandCodec::tree / block_enum (src/lib/bandcodec.cpp:346-589).
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
	uint8_t* pin[3];
	int pitch[3], dx[3], dy[3], bw[3];
	int ppitch[3], pdx[3], pdy[3];
	int first[4];
	int high, do_rec, do_pin;
};

template <typename C, typename P>
__global__ void __launch_bounds__(256) k_blocks(SArgs a, int n)
{
	int gid = blockIdx.x * blockDim.x + threadIdx.x;
	if (gid >= n) return;
	int b = gid >= a.first[2] ? 2 : gid >= a.first[1] ? 1 : 0;
	int s = gid - a.first[b];
	const int by = s / a.bw[b], bx = s - by * a.bw[b];
	if (a.do_rec)
		a.rec[b][s] = block_local<C>(kSymDev, (const C*)a.band[b], a.pitch[b], a.dx[b], a.dy[b], a.high != 0, bx, by);
	if (a.do_pin)
		a.pin[b][s] = (uint8_t)parent_info<P>((const P*)a.par[b], a.ppitch[b], a.pdx[b], a.pdy[b], bx, by);
}

}  // namespace

void launch_blocks_level(const Pyramid& P, int l, bool do_rec, bool do_pin, char* arena, hipStream_t st)
{
	const Level& L = P.L[l];
	SArgs a;
	int n = 0;
	const bool has_par = l + 1 < P.nlev;
	do_pin = do_pin && has_par;
	if (!do_rec && !do_pin) return;
	for (int b = 0; b < 3; b++) {
		const Band& B = L.b[b];
		a.band[b] = arena + B.off; a.pitch[b] = B.pitch; a.dx[b] = B.dx; a.dy[b] = B.dy; a.bw[b] = B.bw();
		a.rec[b] = (uint64_t*)(arena + P.rec_off[l][b]);
		a.pin[b] = (uint8_t*)(arena + P.pin_off[l][b]);
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
	a.do_rec = do_rec;
	a.do_pin = do_pin;
	if (n == 0) return;
	dim3 grid((n + 255) / 256);
	const bool pint = has_par ? P.L[l + 1].is_int : L.is_int;
	if (!L.is_int && !pint) hipLaunchKernelGGL((k_blocks<int16_t, int16_t>), grid, dim3(256), 0, st, a, n);
	else if (!L.is_int) hipLaunchKernelGGL((k_blocks<int16_t, int32_t>), grid, dim3(256), 0, st, a, n);
	else hipLaunchKernelGGL((k_blocks<int32_t, int32_t>), grid, dim3(256), 0, st, a, n);
}

}  // namespace ric
