// ric_types.h -- band-pyramid geometry and integer helpers shared by the HIP
// kernels and the host coder.  The arithmetic helpers restate
// src/lib/utils.h:79-138 and CWavelet2D::mult08 (src/lib/wavelet2d.cpp:307-318)
// with well-defined forms (no shift UB).
#pragma once
#include <cstdint>
#include <cstddef>

#if defined(__HIPCC__)
#define RIC_HD __host__ __device__ __forceinline__
#else
#define RIC_HD inline
#endif

#if defined(__clang__)
#define RIC_UNROLL _Pragma("unroll")
#else
#define RIC_UNROLL _Pragma("GCC unroll 16")
#endif

namespace ric {

constexpr int kMaxLevels = 16;
constexpr int kInsignif = -0x8000;   // INSIGNIF_BLOCK, src/lib/bandcodec.cpp:113
enum Orient { BD = 0, BH = 1, BV = 2, BL = 3 };
enum Trans { CDF97 = 0, CDF53 = 1, HAAR = 2 };

// C-typed store: SH = band is `short`
template <bool SH> RIC_HD int tr(int v) { return SH ? (int)(int16_t)v : v; }
template <bool SH> RIC_HD uint32_t uc(int v) { return SH ? (uint32_t)(uint16_t)v : (uint32_t)v; }
RIC_HD int trs(bool sh, int v) { return sh ? (int)(int16_t)v : v; }
RIC_HD uint32_t ucs(bool sh, int v) { return sh ? (uint32_t)(uint16_t)v : (uint32_t)v; }

template <bool SH> RIC_HD int mult08(int a)
{
	a = tr<SH>(a);
	a = tr<SH>(a - (a >> 2));
	a = tr<SH>(a + (a >> 4));
	return tr<SH>(a + (a >> 8));
}

RIC_HD int s2u(int s) { int u = (int)(0u - (2u * (uint32_t)s + 1u)); return u ^ (u >> 31); }
RIC_HD int u2s(int u) { return (u >> 1) ^ -(u & 1); }
RIC_HD int s2u_(int s) { int m = s >> 31; return (int)(2u * (uint32_t)s + (uint32_t)m) ^ (m * 2); }
RIC_HD int u2s_(int u) { int m = -(u & 1); return ((u >> 1) + m) ^ m; }
RIC_HD uint32_t popc32(uint32_t m) { return (uint32_t)__builtin_popcount(m); }
RIC_HD int bitlen(uint32_t v) { return v ? 32 - __builtin_clz(v) : 0; }

// One band of the pyramid in the device/host arenas.
struct Band {
	int dx = 0, dy = 0;      // DimX, DimY
	int is_int = 0;          // band_t sint
	int pitch = 0;           // row pitch in elements (arena layout)
	int ref_align = 0;       // the reference's DimXAlign (src/lib/band.cpp:57)
	size_t off = 0;          // byte offset of the band in the arena
	size_t rd_off = 0;       // byte offset of pRD (u32 per 4x4 block)
	float weight = 1.f;      // SetWeight
	int esize() const { return is_int ? 4 : 2; }
	int bw() const { return (dx + 3) / 4; }
	int bh() const { return (dy + 3) / 4; }
	size_t bytes() const { return (size_t)pitch * dy * esize(); }
};

struct Level {
	int w = 0, h = 0;        // input dims of the level
	int is_int = 0;          // band type of this level
	int in_is_int = 0;       // type of the input plane (previous level's LL)
	Band b[4];               // D, H, V, L (L = the next level's input, or the coarsest LL)
};

// CWavelet2D::Init geometry (src/lib/wavelet2d.cpp:69-81, src/lib/band.cpp:51-65).
// Arena layout (one allocation on the device, a pinned mirror on the host):
//   region A [0, a_end):     the coded bands (D/H/V of every level + coarsest LL)
//   region B [a_end, b_end): the device status word, per-block zerotree
//                            records + parent info of the 3*nlev high bands
//   region C [b_end, end):   device-only scratch: intermediate LL planes, pRD
// Encode copies A+B to the host, decode copies A back to the device.
struct Pyramid {
	int nlev = 0;
	int w = 0, h = 0, levels = 0, lc = 0;
	Level L[kMaxLevels];
	size_t arena_bytes = 0, a_end = 0, b_end = 0;
	size_t status_off = 0;                // int: device error word (ring timeout), start of region B
	size_t rec_off[kMaxLevels][3] = {};   // u64 block records (symbols.h), raster order
	size_t pin_off[kMaxLevels][3] = {};   // u8 parent info per block (symbols.h), raster order

	void build(int w_, int h_, int levels_, int lc_)
	{
		w = w_; h = h_; levels = levels_; lc = lc_;
		nlev = 0;
		int lw = w, lh = h, lev = levels;
		auto dims = [](Band& B, int dx, int dy, int is_int) {
			B.dx = dx; B.dy = dy; B.is_int = is_int;
			B.pitch = ((dx + 63) / 64) * 64;
			if (B.pitch == 0) B.pitch = 64;
			int ss = is_int ? 4 : 2;
			B.ref_align = ((dx * ss + 31) & -32) / ss;
		};
		int prev_int = 0;
		while (true) {
			Level& Lv = L[nlev];
			Lv.w = lw; Lv.h = lh;
			Lv.is_int = lev <= lc;
			Lv.in_is_int = nlev == 0 ? 0 : prev_int;   // the image is always short (Transform<short>)
			dims(Lv.b[BD], (lw + 1) >> 1, (lh + 1) >> 1, Lv.is_int);
			dims(Lv.b[BH], lw >> 1, (lh + 1) >> 1, Lv.is_int);
			dims(Lv.b[BV], (lw + 1) >> 1, lh >> 1, Lv.is_int);
			dims(Lv.b[BL], lw >> 1, lh >> 1, Lv.is_int);
			prev_int = Lv.is_int;
			nlev++;
			if (!(lev > 1 && lw > 15 && lh > 15) || nlev == kMaxLevels) break;
			lw >>= 1; lh >>= 1; lev--;
		}
		size_t off = 0;
		auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) / 256 * 256; return o; };
		for (int l = 0; l < nlev; l++)
			for (int b = 0; b < 3; b++) L[l].b[b].off = take(L[l].b[b].bytes());
		L[nlev - 1].b[BL].off = take(L[nlev - 1].b[BL].bytes());
		a_end = off;
		status_off = take(256);
		for (int l = 0; l < nlev; l++)
			for (int b = 0; b < 3; b++) rec_off[l][b] = take((size_t)L[l].b[b].bw() * L[l].b[b].bh() * 8);
		for (int l = 0; l < nlev; l++)
			for (int b = 0; b < 3; b++) pin_off[l][b] = take((size_t)L[l].b[b].bw() * L[l].b[b].bh());
		b_end = off;
		for (int l = 0; l + 1 < nlev; l++) L[l].b[BL].off = take(L[l].b[BL].bytes());
		for (int l = 0; l < nlev; l++)
			for (int b = 0; b < 4; b++) L[l].b[b].rd_off = take((size_t)L[l].b[b].bw() * L[l].b[b].bh() * 4);
		arena_bytes = off;
	}

	// CWavelet2D::SetWeight, src/lib/wavelet2d.cpp:1009-1032 (float32)
	void set_weight(int trans, float base = 1.f)
	{
		float scale = trans == CDF97 ? 1.149604398f * 1.149604398f : 2.f;
		for (int l = 0; l < nlev; l++) {
			Band* B = L[l].b;
			if (l == 0) {
				B[BD].weight = base / scale; B[BV].weight = base; B[BH].weight = base; B[BL].weight = base * scale;
			} else {
				B[BD].weight = L[l - 1].b[BV].weight;
				B[BV].weight = L[l - 1].b[BL].weight;
				B[BH].weight = B[BV].weight;
				B[BL].weight = B[BV].weight * scale;
			}
		}
	}

	Band& coarsest_ll() { return L[nlev - 1].b[BL]; }
	int nbands() const { return 3 * nlev + 1; }
	// canonical band order: levels finest->coarsest, D,H,V; then the coarsest LL
	Band& band(int i) { return i == 3 * nlev ? L[nlev - 1].b[BL] : L[i / 3].b[i % 3]; }
};

}  // namespace ric
