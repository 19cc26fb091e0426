// compact.h -- the host coder's compacted payload (compact.hip): the values a
// frame's host encoder reads from its 16-bit bands, in walk order.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
#include "ric_types.h"

namespace ric {

struct CmpBand {
	uint32_t off, rec_off;           // band and its block records in the frame's arena
	int dx, dy, pitch;
	int nblk;                        // blocks
	int chunk0;                      // first chunk of 64 blocks (flattened over the bands)
};

// Frames f (blockIdx.z): arena + f * astride; the stream to out + f * ostride
// (int16 values); cnt + f * cstride: per chunk, its count then its offset;
// total[f]: the frame's value count.  band[]: the 16-bit bands in coding
// order (coarse to fine, V, H, D).
struct CmpArgs {
	const char* arena;
	size_t astride;
	char* out;
	size_t ostride;
	uint32_t* cnt;
	size_t cstride;
	uint32_t* total;
	int nb, nchunk;
	CmpBand band[3 * kMaxLevels];
};

// the band table of a pyramid (nb, nchunk, band[]); the pointers are the caller's
void cmp_args(const Pyramid& P, CmpArgs& a);
// the most values a frame's stream can hold (every coefficient of its 16-bit bands)
size_t cmp_values(const Pyramid& P);
// the arena offset from which the rest of the payload stays dense: the int
// bands, the coarsest LL, then region B (status word, records, parent info)
size_t cmp_dense_from(const Pyramid& P);
// the three passes over nframes frames
int launch_compact(const CmpArgs* dev_args, int nchunk, int nframes, hipStream_t st);

}  // namespace ric
