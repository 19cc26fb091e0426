// ric_kernels.h -- host-side launchers of the HIP kernels (dwt.hip, quant.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <vector>
#include "ric_types.h"

namespace ric {

// Frees that never wait for a stream coder launch (device.cpp).  hipFree and
// hipHostFree synchronise every stream of the device, so a free issued while a
// k_gc_* launch runs (seconds) -- a caller's buffer released by its garbage
// collector, another batch destroyed -- would wait for the whole launch.
// CoderCall marks a library call that may have such a launch in flight; while
// any is active, dev_free / pinned_free park the pointer and the last
// CoderCall to end frees it.  With none active they free at once.
struct CoderCall {
	CoderCall();
	~CoderCall();
	CoderCall(const CoderCall&) = delete;
	CoderCall& operator=(const CoderCall&) = delete;
};
hipError_t dev_free(void* p);       // hipFree, deferred while a CoderCall is active
hipError_t pinned_free(void* p);    // hipHostFree, the same
long deferred_frees();              // frees parked so far (ric_diag_deferred_frees)


// Forward level: src (level input, in_is_int ? int32 : int16, pitch sp) -> the
// level's D/H/V/L bands in the arena.  vec: src rows are 8/16-byte aligned.
void launch_fwd_level(const Level& L, const void* src, long sp, char* arena, int trans, int vec,
                      hipStream_t st);
// Fused forward level + quantiser + block records (dwt.hip k_fwdq): the 9/7
// short->short levels.  Writes level l's quantised D/H/V bands, pRD, block-local
// records, its unquantised LL, and (l > 0) the parent info of level l-1.
struct QuantParams;
// How a level's forward transform + quantiser run: FQ_PACKED = k_fwdq_fast
// (9/7 short levels, sizes multiples of 8, 16-byte aligned rows, rd thresholds
// in the packed range), FQ_GENERIC = k_fwdq_gen (other 9/7 levels), FQ_NONE =
// separate forward / quantiser / record kernels (5/3, Haar).
enum { FQ_NONE = 0, FQ_PACKED = 1, FQ_GENERIC = 2 };
int fwdq_mode(const Level& L, int trans, const QuantParams& qp, int vec16);
// in8: the level-0 input is 8-bit pixels after the ric level shift (|x| <=
// 2048), which bounds every mult08 sum to 16 bits and allows the plain packed
// form at level 0; any other input (the API's Transform, the video residual)
// takes the exact form (dwt.hip mult08x).
void launch_fwdq_level(const Pyramid& P, int l, const void* src, long sp, int vec8, int vec16, const QuantParams& qp,
                       char* arena, hipStream_t st, int in8 = 0);
// Generic fused forward level + quantiser + records (dwt.hip k_fwdq_gen) for
// any 9/7 level (int bands, odd sizes); ll_on: also CBand::TSUQ on the level's
// LL (the coarsest level), with its iQ and dead zone T0.
void launch_fwdq_gen_level(const Pyramid& P, int l, const void* src, long sp, int vec8, const QuantParams& qp,
                           int ll_on, int ll_iQ, int ll_T0, char* arena, hipStream_t st);
// Inverse level: D/H/V bands + lls (the level's LL) -> out (pitch po elements),
// typed int32 if out_is_int else int16.  q (optional): TSUQi multipliers of
// D, H, V, LL applied to the loaded band values (fused dequantiser).
void launch_inv_level(const Level& L, const Band& lls, char* arena, void* out, long po,
                      int out_is_int, int trans, hipStream_t st, const int* q = nullptr);

// Per-band quantiser parameters computed on the host (float32 exactly as the
// reference: src/lib/bandcodec.cpp:243-247, 149-157).
struct QuantParams {
	int Q[3], iQ[3];
	int thres[3][16];
};
// buildTree for the D/H/V bands of one level (finest level first).
void launch_quant_level(const Pyramid& P, int l, const QuantParams& qp, char* arena, hipStream_t st);
// CBand::TSUQ on the coarsest LL (src/lib/band.h:65-92).
void launch_quant_ll(const Pyramid& P, int Q, int iQ, int T, char* arena, hipStream_t st);
// Zerotree block records of the D/H/V bands of level l (symbols.h), written
// at P.rec_off[l][b]; needs every level quantised (parents are read).
// do_rec: the block-local records of level l; do_pin: the parent info of
// level l's blocks, read from level l+1's quantised bands.
void launch_blocks_level(const Pyramid& P, int l, bool do_rec, bool do_pin, char* arena, hipStream_t st);
// CBand::TSUQ on one band, adding its non-zero count to *count (device).
void launch_tsuq_band(const Band& B, int iQ, int T0, char* arena, unsigned int* count, hipStream_t st);
// CBand::TSUQi on one band (src/lib/band.h:94-107).
void launch_dequant_band(const Band& B, int q, char* arena, hipStream_t st);
// CBand::TSUQ with its statistics: stats[0] += non-zeros, stats[1] max=,
// stats[2] min= (device ints, initialised by the caller to 0, 0, 0)
void launch_band_tsuq(const Band& B, int iQ, int T0, char* arena, int* stats, hipStream_t st);
// CBand::Mean's Sum and SSum (device u64[2], zeroed by the caller)
void launch_band_sums(const Band& B, const char* arena, unsigned long long* out, hipStream_t st);
// CBand::Add(val) over the band's rows (padding included)
void launch_band_add(const Band& B, int val, char* arena, hipStream_t st);
// ------------------------------------------------------- batched launches
// nz frames at fixed strides: frame f's arena is arena + f * astride, its
// level input src + f * sstride (bytes, row pitch sp elements), its inverse
// output out + f * ostride (bytes, row pitch po elements).  One grid over all
// frames (blockIdx.z = frame).
struct ZFrames {
	char* arena = nullptr; size_t astride = 0;
	const void* src = nullptr; size_t sstride = 0; long sp = 0;
	void* out = nullptr; size_t ostride = 0; long po = 0;
	int nz = 0;
	// level 0 of the fused forward: the LDS ring hand-off (1: 32 KiB per
	// workgroup, the faster form alone on the chip) or the double buffer (0:
	// 20 KiB, two workgroups per CU fit beside the stream coder's waves)
	int ring = 0;
	// level 0 of a gray batch straight from its u8 pixels (k_fwdq_pc_z8, the
	// ric level shift fused): one device pointer per frame (W bytes per row,
	// 8-byte aligned), sh8 the shift; null: from src (the coding planes)
	const uint8_t* const* pix8 = nullptr;
	int sh8 = 0;
	// the last level on the one-producer form (k_fwdq_pc_z; above it the
	// two-producer k_fwdq_pc2_z): 1 when the level kernels run alone on the
	// chip (measured at C3: level 1 20.4 against 23.2 us per frame), 0 beside
	// the stream coder's waves (the one-producer form holds 128 VGPRs)
	int pc1 = 0;
	// Split arenas (the GPU stream coder's pool): regions A and B (bands,
	// status word, records, parent info: offsets below `split` = Pyramid::b_end)
	// of frame f at arena + f * astride, region C (intermediate LL planes, pRD)
	// at scratch + f * scstride.  scratch null: one arena per frame.
	char* scratch = nullptr; size_t scstride = 0; size_t split = 0;
	// the compacted pool (ric_batch_hybrid_config_ex): the offsets below `lo`
	// (level 0's three bands) are in the scratch arena as well -- the pool
	// holds them compacted, not at their pyramid offsets
	size_t lo = 0;
	char* c_base(int f) const { return scratch ? scratch + (size_t)f * scstride : arena + (size_t)f * astride; }
	// level 0 of a gray 9/7 decode (launch_inv_level_z): the pixel output
	// fused -- frame f's u8 pixels to pix[f] (w bytes per row, 4-byte aligned,
	// w a multiple of 4), unshifted with quantiser pix_q[f]; dig_part (or
	// null): 16 partial digest words per frame (zeroed first), folded by
	// launch_digest_fold.  The int16 plane (out) is not written.
	uint8_t* const* pix = nullptr;
	const int* pix_q = nullptr;
	unsigned long long* dig_part = nullptr;
};
// Per-frame argument array of one batched launch, on the device; uploaded
// only when it changes.  A ring of kRing device / pinned host slots: a new
// image goes to the next slot by an async copy in stream order, so an upload
// never waits for the kernels still reading the previous images (round 5
// synchronised the stream before every upload: the batch stream's host thread
// then waited out each level launch of the step's front, ~1000 per step, with
// the GPU idle while it issued the next).  A slot is reused once the event
// recorded after its last launch has passed (kRing uploads later: at once).
// Images that come back (the serving step's groups reuse the same pool slots,
// scratch arenas and output buffers step after step) are kept in a cache of
// device copies, uploaded once: a step then issues its level launches without
// an argument copy in front of each (round 6: ~1870 copies per step, each a
// small blit kernel in the batch stream's order).  Up to kCacheBytes per
// ZArgs; images past it take the ring.
struct ZArgsImage {
	uint64_t hash;
	char* dev;
	std::vector<char> host;
	hipStream_t st;                  // the stream the upload was queued on
	hipEvent_t ev;                   // after the upload
};
struct ZArgs {
	static constexpr int kRing = 8;
	static constexpr size_t kCacheBytes = 4u << 20, kCacheBlock = 256u << 10;
	void* dev = nullptr;             // the current image's slot (the launches' argument)
	char* dbase = nullptr;           // kRing slots of cap bytes
	char* hbase = nullptr;           // pinned staging, the same
	size_t cap = 0;
	int cur = -1;
	hipStream_t st = nullptr;        // the stream of the current slot's launches
	hipEvent_t ev[kRing] = {};
	bool evset[kRing] = {};
	std::vector<char> img;
	// the cache: images by hash, carved from device / pinned blocks
	std::vector<ZArgsImage> cache;
	std::vector<char*> cdev, chost;  // blocks of kCacheBlock
	size_t cused = 0;                // bytes carved from the last block
	size_t ctotal = 0;               // bytes cached
	int ccur = -1;                   // the cache entry in use (then cur is only the ring's position), or -1
};
int zargs_put(ZArgs& z, const void* data, size_t bytes, hipStream_t st);
void zargs_free(ZArgs& z);
// The batched forms of launch_fwdq_level / launch_fwdq_gen_level /
// launch_inv_level; 0 or -1 (HIP error).  The inverse takes 4 TSUQi factors
// per frame (q + 4 f), or none.
int launch_fwdq_level_z(const Pyramid& P, int l, const ZFrames& fr, int vec8, int vec16, const QuantParams& qp,
                        ZArgs& z, hipStream_t st, int in8 = 0);
int launch_fwdq_gen_level_z(const Pyramid& P, int l, const ZFrames& fr, int vec8, const QuantParams& qp, int ll_on,
                            int ll_iQ, int ll_T0, ZArgs& z, hipStream_t st);
int launch_inv_level_z(const Level& L, const Band& lls, const ZFrames& fr, int out_is_int, int trans, const int* q,
                       ZArgs& z, hipStream_t st);

// diagnostics: the level-0 workgroup trace of the fused level kernel (dwt.hip)
int diag_wgtrace(int device, uint64_t* host, int n);
// fault injection: force a ring hand-off timeout in the next fused launches
void diag_set_fault(int on);

}  // namespace ric
