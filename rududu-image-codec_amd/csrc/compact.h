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
// (int16 values); cnt + f * cstride: per chunk, its count then its offset
// (three passes), or the one-pass kernel's ticket and look-back words -- at
// least up(nchunk, 64) words, zeroed when allocated;
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
	// the GPU stream coder's compacted pool (batch.cpp): the bands come from
	// bsrc + f * bstride (the scratch arenas) while the records are the pool's
	// (arena); at most vcap values are written, and a frame with more sets 4 in
	// its status word (status + f * sstride) -- the coder then leaves it to the
	// host.  bsrc null: the bands are in arena; vcap 0: no limit.
	const char* bsrc;
	size_t bstride;
	uint32_t vcap;
	char* status;
	size_t sstride;
};
// a compacted pool frame over its capacity (the status word's bit)
constexpr int32_t kCmpOverCap = 4;
// the one-pass compaction's look-back gave up (the status word's bit; nothing
// written: the frame is then left to the host, or its call fails)
constexpr int32_t kCmpLookback = 8;

// the band table of a pyramid (nb, nchunk, band[]); the pointers are the caller's
void cmp_args(const Pyramid& P, CmpArgs& a);
// the most values a frame's stream can hold (every coefficient of its 16-bit bands)
size_t cmp_values(const Pyramid& P);
// the arena offset from which the rest of the payload stays dense: the int
// bands, the coarsest LL, then region B (status word, records, parent info)
size_t cmp_dense_from(const Pyramid& P);
// the compaction of nframes frames: three passes (count, scan, write), or
// one (k_cmp_one, RIC_CMP_PASS=1)
int launch_compact(const CmpArgs* dev_args, int nchunk, int nframes, hipStream_t st);
// frame f's values (total[f] int16, from src + f * sstride, rounded up to 16
// bytes) to dst + f * dstride: a device-mapped host mirror, written by the kernel
int launch_cmp_to_host(const char* src, size_t sstride, char* dst, size_t dstride, const uint32_t* total, int nframes,
                       hipStream_t st);

// ---- the decode side: the host decoder's finest level (three 16-bit bands
// without children) comes back compacted (decoder.cpp tree_decode_compact)
// and is scattered into the dense bands on the device.  One block per frame:
//   u32 nval[3]           values of each band (coding order V, H, D)
//   u16 mask[nblk_b]      per band, per block in walk order
//   u32 chunk_off[nch_b]  per band, the value count before each 64 blocks
//   i16 vals[]            per band, in walk order, bands back to back
struct DcmpLayout {
	int band[3];                      // BV, BH, BD of level 0
	size_t mask_off[3], coff_off[3], vals_off;
	int nblk[3], nch[3];
	bool ok = false;                  // level 0 is 16-bit and has no int bands
};
DcmpLayout dcmp_layout(const Pyramid& P);
struct DcmpArgs {
	char* arena;                      // frame f: arena + f * astride
	size_t astride;
	const char* in;                   // frame f's block: in + f * istride
	size_t istride;
	uint32_t off[3];                  // band offsets in the arena
	int dx[3], dy[3], pitch[3];
	uint32_t mask_off[3], coff_off[3], vals_off;
	int nblk[3], chunk0[4];           // chunk0[3] = total chunks
	// values readable per block (the compacted pool's capacity: a frame the
	// coder left to the host holds no valid offsets), 0: no limit
	uint32_t vcap = 0;
};
int launch_dcmp_expand(const DcmpArgs& a, int nframes, hipStream_t st);

}  // namespace ric
