// motion.h -- launchers of the video codec's data-parallel stages (motion.hip):
// the reference's CImage / CImageBuffer pixel work (src/lib/image.cpp,
// imagebuffer.cpp), the EPZS motion search (COBME, src/lib/obme.cpp) and the
// overlapped block motion compensation (COBMC::apply_mv, src/lib/obmc.cpp).
//
// Images keep the reference's CImage memory layout exactly (image.cpp:56-68):
// planes of dimXAlign = (w + 2 * 15 + 31) & -32 samples per row and h + 30
// rows, BORDER = 15 rows / columns of border, the three planes back to back.
// An image is addressed by its pImage[0] (plane 0, row 0, column 0); plane c
// starts P = dimXAlign * (h + 30) samples later.  The border samples are part
// of the codec's state (calc_sub reads a sample past each edge before extend()
// rewrites them, and TransformI leaves part of its level-1 output there), so
// the kernels read and write them at the reference's addresses.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ric {

constexpr int kVidBorder = 15;            // BORDER, src/lib/image.h:27
constexpr uint32_t kVidIntra = 0x80008000u;   // MV_INTRA, src/lib/obmc.h:37

struct VidGeom {
	int w = 0, h = 0;            // image size
	int S = 0;                   // dimXAlign (samples)
	long P = 0;                  // plane stride (samples)
	int bx = 0, by = 0;          // OBMC / motion blocks: w >> 3, h >> 3
	void init(int w_, int h_)
	{
		w = w_; h = h_;
		S = (w + 2 * kVidBorder + 31) & -32;
		P = (long)S * (h + 2 * kVidBorder);
		bx = w >> 3; by = h >> 3;
	}
	size_t image_samples() const { return (size_t)P * 3; }
	long origin() const { return (long)kVidBorder * S + kVidBorder; }   // pImage[0] - allocation start
};

// the 16 quarter-pel images of a reference frame (sub[4 * x_phase + y_phase],
// sub[0] the frame itself: CImageBuffer::calc_sub, imagebuffer.cpp:90-121)
struct VidSubs {
	int16_t* p[16];
};

// CImage::inputSGI<unsigned char> (image.cpp:96-123) with offset -128: planes
// R, G, B of h rows x stride bytes (bottom row first) -> Y, Co, Cg
int launch_vid_input(const VidGeom& g, const uint8_t* rgb, int stride, int16_t* img, hipStream_t st);
// CImage::operator-= / += (image.cpp:216-246): img -= pred (sign < 0) or +=
int launch_vid_addsub(const VidGeom& g, int16_t* img, const int16_t* pred, int sign, hipStream_t st);
// calc_sub's interpolation: interH<1..3> of sub[0] into sub[4], sub[8],
// sub[12], then interV<1..3> of sub[0, 4, 8, 12] into the rest (image.cpp:
// 280-342), reading the samples one past each edge as the reference does
int launch_vid_interp(const VidGeom& g, const VidSubs& s, hipStream_t st);
// CImage::extend (image.cpp:190-214) of n images
int launch_vid_extend(const VidGeom& g, const VidSubs& s, int n, hipStream_t st);
// COBME::EPZS (obme.cpp:171-244): the full-pel predictor + diamond search in
// raster order (a wavefront over the block rows: block (i, j) needs (i - 1, j)
// and (i + 1, j - 1)), then the quarter-pel refinement of every block.
// mv: the motion field, read (the previous frame's vectors are predictors)
// and rewritten; dist: scratch (u16 per block); gran: the rows' hand-off
// granules (u64 per block, {vector, epoch}: zeroed once at allocation, never
// reset); epoch: this search's tag, non-zero and different from the previous
// search's; status: set non-zero if a wait gave up.
int launch_vid_epzs(const VidGeom& g, const int16_t* cur, const VidSubs& ref, uint32_t* mv, uint16_t* dist,
                    uint64_t* gran, uint32_t epoch, uint32_t* status, hipStream_t st);
// COBMC::apply_mv (obmc.cpp:278-332) into pred, reference frame `ref`
// residual != nullptr (the encoder): also residual = residual - prediction over
// the whole w x h plane, in the same pass (CImage::operator-=, k_vid_addsub's -1)
int launch_vid_obmc(const VidGeom& g, const uint32_t* mv, const VidSubs& ref, int16_t* pred, int16_t* residual,
                    hipStream_t st);
// the samples CWavelet2D::TransformI (given the plane's end pointer) leaves
// outside the plane: its level-1 output, dx1 x dy1 at (row h - dy1, column
// dimXAlign - dx1) of the plane, wrapping into the next row's left border
// (wavelet2d.cpp:503-510, 963-969).  ll1: that output (the level-0 LL band
// after the coarse inverse levels), row pitch ll1_pitch.
int launch_vid_tinv_side(const VidGeom& g, int16_t* plane, const int16_t* ll1, long ll1_pitch, int dx1, int dy1,
                         hipStream_t st);

}  // namespace ric
