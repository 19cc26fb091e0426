// gcoder.h -- launch interface of the GPU stream coder (gcoder.hip): the
// serial .ric coder with one wave per frame's stream.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>
#include "ric_types.h"

namespace ric {

// One band as the stream coder sees it: offsets into the frame's arena.
struct GBandDesc {
	uint32_t off;        // band (pitch elements, is_int ? int32 : int16)
	uint32_t rec_off;    // u64 block records, raster order (symbols.h)
	uint32_t pin_off;    // u8 parent info, raster order
	int dx, dy, pitch, is_int;
	int high;            // finest level (HIGH Huffman tables, k >= 1)
	int has_pin;         // has a parent level (not the coarsest)
	int par;             // decoder: index into b[] of the parent band, or -1
	// the compacted pool (GEncArgs::cmp_rel): 1 + the band's index in the
	// compact block (level 0's V, H, D: DcmpLayout), or 0 (dense at off).
	// The encoder reads the values at the set bits of each block's record mask
	// from the block's value stream; the decoder writes that stream, each
	// block's mask (u16 at cmask_off, walk order) and each chunk's value count
	// before it (u32 at ccoff_off), relative to the compact block.
	int cmp;
	uint32_t cmask_off, ccoff_off;
};
// The compact block of a plane (GEncArgs / GDecArgs::cmp_rel != 0): at the
// plane's arena base + cmp_rel, DcmpLayout (compact.h): u32 nval[3] (written
// by the decoder), the masks, the chunk offsets, then the values of V, H, D
// back to back from cvals_off, at most cvcap of them.

// Frames f = 0..n-1 (blockIdx.x): arena + f * astride, out + f * ostride.
// b[] in coding order: coarsest level first, V, H, D (CodeBand order).
// nplanes 1 (gray) or 3 (Y, Co, Cg: ric.cpp:157-176 codes them in order into
// one stream): plane p's pyramid at arena + f * astride + p * pstride.
struct GEncArgs {
	const char* arena;
	size_t astride;
	size_t pstride;
	int nplanes;
	uint8_t* out;
	size_t ostride;
	size_t cap;                      // bytes available at each out
	uint32_t* res;                   // per frame: file length, status (0 ok, 1 capacity, 2 ring timeout, 3 guard, 4 over a compacted pool's capacity)
	uint32_t status_off;
	int prio;                        // issue priority by progress: 0 off, 1 or 2 (prio_band, gcoder.hip)
	const uint32_t* yield;           // the batch stream's level-kernel flag (coder_yield), or null
	uint64_t* ts;                    // diagnostics: 4 words per frame: the wave's start, end (s_memrealtime, 100 MHz), HW_ID | XCC_ID << 32; or null
	int w, h, q, trans;
	long long cmp_rel;               // compacted pool: the compact block's offset from the plane's base; 0: dense
	uint32_t cvals_off, cvcap;
	int nb;
	GBandDesc ll;
	GBandDesc b[3 * kMaxLevels];
};

// Frames f = 0..n-1 (blockIdx.x): the .ric file at in + f * istride (istride
// bytes readable, a multiple of 16), its length lens[f * lens_stride]; the
// decoded bands to arena + f * astride.  res[f]: 0 ok, 1 the stream ran past
// its end (RIC_E_STREAM, bands still written), 3 LDS staging overrun.
struct GDecArgs {
	char* arena;
	size_t astride;
	size_t pstride;                  // as GEncArgs
	int nplanes;
	const uint8_t* in;
	size_t istride;
	const uint32_t* lens;
	int lens_stride;
	uint32_t* res;
	uint32_t* dbg;                   // diagnostics: 8 words of coder state after the LL and each band, per frame (or null)
	uint64_t* ts;                    // diagnostics: as GEncArgs::ts
	int prio;                        // as GEncArgs::prio
	const uint32_t* yield;           // as GEncArgs::yield
	const uint32_t* etab;            // the enumDecode<16> pattern table (gc_enum16_table())
	int w, h;
	long long cmp_rel;               // as GEncArgs
	uint32_t cvals_off, cvcap;
	int nb;
	GBandDesc ll;
	GBandDesc b[3 * kMaxLevels];
};
int launch_gc_decode(const GDecArgs* dev_args, int nframes, hipStream_t st);
// *flag = v in stream order (a one-wave kernel; the coder waves poll it)
int launch_gc_flag(uint32_t* flag, uint32_t v, hipStream_t st);
// the device address of the decoder's enumDecode<16> table (GDecArgs::etab),
// uploaded on first use on the current device; null on failure
const uint32_t* gc_enum16_table(hipStream_t st);

// k_gc_encode over n frames: the whole .ric file of each (gray, one plane).
// dev_args: the argument block in device memory.
// lossless: q == 0 (the 8 KiB byte ring; lossy streams take a 4 KiB one).
// posted (or null): each frame's result as soon as its stream is in HBM,
// host-visible: posted[2 f] = the coder's end offset, posted[2 f + 1] = status |
// 0x100 | (tag & 0xFFFFF) << 12 -- the caller accepts only its launch's tag.
int launch_gc_encode(const GEncArgs* dev_args, int nframes, int lossless, hipStream_t st, uint32_t* posted = nullptr,
                     uint32_t tag = 0);

// k_gc_roundtrip over n lossy frames: each wave encodes its frame (as
// k_gc_encode), posts its result tagged as launch_gc_encode does, then decodes
// the stream (as k_gc_decode, lens from the encoder) and, with posted_dec,
// posts that its bands are in memory: posted_dec[f] = the decoder's result
// word (0x80 if the encode failed) | 0x100 | (tag & 0xFFFFF) << 12.
int launch_gc_roundtrip(const GEncArgs* dev_eargs, const GDecArgs* dev_dargs, uint32_t* posted, uint32_t* posted_dec,
                        uint32_t tag, int nframes, hipStream_t st);

// Fill the band descriptors (coding order) of a pyramid.
inline void gc_bands(const Pyramid& P, GBandDesc& ll, GBandDesc* b, int& nb)
{
	auto desc = [&](const Band& B, GBandDesc& d) {
		d.off = (uint32_t)B.off; d.dx = B.dx; d.dy = B.dy; d.pitch = B.pitch; d.is_int = B.is_int;
		d.rec_off = d.pin_off = 0; d.high = 0; d.has_pin = 0; d.par = -1;
		d.cmp = 0; d.cmask_off = d.ccoff_off = 0;
	};
	desc(P.L[P.nlev - 1].b[BL], ll);
	nb = 0;
	const int order[3] = {BV, BH, BD};
	for (int l = P.nlev - 1; l >= 0; l--)
		for (int k = 0; k < 3; k++) {
			GBandDesc& d = b[nb];
			desc(P.L[l].b[order[k]], d);
			d.rec_off = (uint32_t)P.rec_off[l][order[k]];
			d.pin_off = (uint32_t)P.pin_off[l][order[k]];
			d.high = l == 0;
			d.has_pin = l + 1 < P.nlev;
			d.par = l + 1 < P.nlev ? nb - 3 : -1;
			nb++;
		}
}

// the compacted pool: level 0's three bands (coding order V, H, D) read from
// / written to the compact block of layout L (compact.h dcmp_layout)
inline void gc_bands_compact(GBandDesc* b, int nb, const size_t* mask_off, const size_t* coff_off)
{
	for (int k = 0; k < 3; k++) {
		GBandDesc& d = b[nb - 3 + k];
		d.cmp = 1 + k;
		d.cmask_off = (uint32_t)mask_off[k];
		d.ccoff_off = (uint32_t)coff_off[k];
	}
}

}  // namespace ric
