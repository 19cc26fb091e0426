// batch.cpp -- ric_batch (include/ric_gpu.h): CompressImage / DecompressImage
// (src/ric/ric.cpp:123-251) over a batch of frames of one geometry.
//
// The frames of a group sit in fixed-stride slots of one device arena, one
// pinned host mirror and one set of coding planes, so every GPU stage is one
// launch per level over the whole group (blockIdx.z = frame, dwt.hip *_z
// kernels): the small coarse levels that leave most of the chip idle for a
// single frame fill it for a batch.  A native pool of host threads runs the
// serial coder (entropy.cpp / encoder.cpp / decoder.cpp) of different frames
// in parallel.  Two sets of slots let ric_batch_roundtrip overlap the GPU
// stages of one group with the host coding of the previous one.
//
// Output is byte-identical to ric_codec (the same kernels' arithmetic and the
// same host coder), i.e. to the reference.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ric_gpu.h"
#include "ric_types.h"
#include "ric_kernels.h"
#include "ric_image.h"
#include "entropy.h"
#include "codec_params.h"
#include "gcoder.h"
#include "host_pool.h"
#include "compact.h"

using namespace ric;

namespace {

bool bfail(hipError_t e, const char* what)
{
	if (e == hipSuccess) return false;
	set_last_error(std::string(what) + ": " + hipGetErrorString(e));
	return true;
}
#define BCHK(x) do { if (bfail((x), #x)) return RIC_E_HIP; } while (0)

double now_ms()
{
	return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// counts down the tasks of one group
class Latch {
public:
	void reset(int n) { std::lock_guard<std::mutex> g(mu_); left_ = n; }
	void done()
	{
		std::lock_guard<std::mutex> g(mu_);
		if (--left_ == 0) cv_.notify_all();
	}
	void wait()
	{
		std::unique_lock<std::mutex> lk(mu_);
		cv_.wait(lk, [this] { return left_ <= 0; });
	}
	bool wait_for_ms(int ms)
	{
		std::unique_lock<std::mutex> lk(mu_);
		return cv_.wait_for(lk, std::chrono::milliseconds(ms), [this] { return left_ <= 0; });
	}

private:
	std::mutex mu_;
	std::condition_variable cv_;
	int left_ = 0;
};

// Stage timers: GPU stages by event pairs on the batch's stream (harvested
// after the call's final sync), host stages by a steady clock per frame.
// Stage order: pix_in, fwd level 0..7, d2h, host_enc, host_dec, h2d,
// inv level 0..7, pix_out, gpu stream encode, gpu stream decode
// (RIC_BATCH_STAGES; the stream coder stages are per launch: ms = kernel
// time, frames = streams).
// B_D2HV: the compacted values of host-coded frames, written into the host mirrors by k_cmp_to_host
enum { B_PIXIN = 0, B_FWD = 1, B_D2H = 9, B_HENC = 10, B_HDEC = 11, B_H2D = 12, B_INV = 13, B_PIXOUT = 21, B_GENC = 22, B_GDEC = 23,
       B_D2HV = 24, B_GRT = 25, B_DEXP = 26, B_CMP = 27, B_COUNT = 28 };   // B_CMP: k_cmp_count / scan / write (pool and host payloads)   // B_DEXP: k_dcmp_expand (part of B_H2D)   // B_GRT: the stream coder's encode + decode as one kernel

struct BProf {
	bool on = false;
	struct Rec { int stage; hipEvent_t a, b; int frames; };
	std::vector<Rec> pending;
	std::vector<hipEvent_t> spare;
	double ms[B_COUNT] = {};
	long frames[B_COUNT] = {}, launches[B_COUNT] = {};
	std::mutex mu;

	hipEvent_t ev()
	{
		if (!spare.empty()) { hipEvent_t e = spare.back(); spare.pop_back(); return e; }
		hipEvent_t e = nullptr;
		(void)hipEventCreate(&e);
		return e;
	}
	// brackets one GPU stage of `frames` frames
	struct Span { BProf* p; int stage, frames; hipEvent_t a = nullptr; hipStream_t st; };
	Span begin(int stage, int nfr, hipStream_t st)
	{
		Span s{this, stage, nfr, nullptr, st};
		if (!on) return s;
		s.a = ev();
		(void)hipEventRecord(s.a, st);
		return s;
	}
	void end(const Span& s)
	{
		if (!s.a) return;
		hipEvent_t b = ev();
		(void)hipEventRecord(b, s.st);
		pending.push_back({s.stage, s.a, b, s.frames});
	}
	void harvest()   // after a stream sync
	{
		for (auto& r : pending) {
			float t = 0;
			if (hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
				ms[r.stage] += t; frames[r.stage] += r.frames; launches[r.stage]++;
			}
			spare.push_back(r.a); spare.push_back(r.b);
		}
		pending.clear();
	}
	void host(int stage, double t)
	{
		if (!on) return;
		std::lock_guard<std::mutex> g(mu);
		ms[stage] += t; frames[stage]++; launches[stage]++;
	}
	void reset()
	{
		for (int i = 0; i < B_COUNT; i++) { ms[i] = 0; frames[i] = 0; launches[i] = 0; }
	}
	void destroy()
	{
		for (auto& r : pending) { spare.push_back(r.a); spare.push_back(r.b); }
		pending.clear();
		for (hipEvent_t e : spare) (void)hipEventDestroy(e);
		spare.clear();
	}
};

}  // namespace

struct ric_batch {
	// The level kernels' forms (ZFrames::ring, ::pc1): beside the stream
	// coder's waves level 0 takes the double-buffered hand-off (20 KiB of LDS,
	// two workgroups per CU fit beside them) and level 1 the two-producer
	// kernel; alone on the chip (the step's front, before the coder launch;
	// the diagnostics) the LDS ring hand-off and the one-producer level 1 are
	// faster (C3, 16 frames: level 0 61.6 against 67.3 us per frame, level 1
	// 20.4 against 23.2).  RIC_FQZ_ALONE=0: the beside forms everywhere.
	// Every call but the serving step (ric_batch_roundtrip_hybrid) runs its
	// level kernels alone.
	int fq_ring = 1, fq_pc1 = 1;
	void alone(bool on)
	{
		static const bool en = [] { const char* e = getenv("RIC_FQZ_ALONE"); return !e || atoi(e) != 0; }();
		// alone: the LDS-ring hand-off, levels 0-2 on one producer wave (level 2:
		// 5.8-6.0 against 6.3-6.4 us per C3 frame, profiles/r05_level12_sweep.log)
		fq_ring = on && en ? 1 : 0;
		fq_pc1 = on && en ? 2 : 0;
	}
	ric_batch() { alone(true); }
	// The host encoder's payload compacted on the GPU (compact.hip): the
	// 16-bit bands' values in walk order instead of the dense bands.  Per
	// slot: the stream (d_cmp), chunk counts / offsets, its value count (also
	// pinned on the host); cmp_ok[s]: slot s's last forward pass compacted.
	bool compact = true;
	char* d_cmp = nullptr;
	size_t cmp_stride = 0;
	uint32_t* d_cmp_cnt = nullptr;
	size_t cmp_cstride = 0;
	uint32_t* d_cmp_total = nullptr;
	uint32_t* h_cmp_total = nullptr;
	CmpArgs* d_cmp_args = nullptr;                 // one block per slot set
	int cmp_nchunk = 0;
	size_t cmp_dense = 0;                          // arena offset where the dense part starts
	std::vector<char> cmp_ok;
	// the decode side: the host decoder's finest level compacted
	// (tree_decode_compact), scattered on the device (k_dcmp_expand)
	bool dcompact = false;
	DcmpLayout dl;
	std::vector<size_t> dcmp_bytes;
	std::vector<char> dcmp_ok;
	// ric_batch_set_digests: per frame of a call, the digest of its decoded pixels
	unsigned long long* digest = nullptr;
	long ndigest = 0;
	// the fused pixel output's partial digest words (16 per frame of a group)
	unsigned long long* d_dpart = nullptr;
	// the step's front: a host group's band copies on a stream of their own
	// (xst), after the batch stream's compaction (ev_fork)
	hipStream_t xst = nullptr;
	hipEvent_t ev_fork = nullptr;
	// ric_batch_set_ready: per frame of a call, its .ric file's length once the
	// file is complete in out[i] (host words the caller polls)
	uint32_t* ready = nullptr;
	long nready = 0;
	int device = 0, w = 0, h = 0, channels = 1, slots = 0;
	double hyb_host_ms = 0, hyb_gpu_ms = 0;        // last hybrid call: when each side finished (ms from entry)
	int hyb_fallback = 0;                          // last hybrid call: frames over the pool's value capacity
	bool cmp_dma = false;                          // host frames' compacted values to the host by DMA (d2h_slots)
	Pyramid P;
	size_t astride = 0, hstride = 0, pstride = 0;   // bytes per slot: device arena, host mirror, coding planes
	long pitch = 0;                                // coding plane row pitch (elements)
	char* d_arena = nullptr;                       // 2 * slots slots
	char* h_arena = nullptr;
	char* h_arena_dev = nullptr;                   // the mirror's device-mapped address (k_cmp_to_host)
	int16_t* d_planes = nullptr;
	uint8_t* d_stage = nullptr;                    // host pixels in / out, w*h*channels per slot
	hipStream_t st = nullptr;
	// non-blocking streams for the device -> host copies made while a coder
	// launch runs (the stream copier, host-decoded streams): never the null
	// stream, which waits for every blocking stream of the process
	hipStream_t cst[4] = {nullptr, nullptr, nullptr, nullptr};
	ZArgs zf[2][kMaxLevels], zi[2][kMaxLevels];    // per set: forward / inverse argument arrays
	std::vector<Mux> enc, dec;                     // per slot
	Pool* pool = nullptr;
	// The band-parallel encoder (encode_bands_split, encoder.cpp) for calls
	// with fewer frames in flight than half the host threads (C4's tiles, C5
	// frames over many ranks): a frame's bands are modelled on bpool's threads
	// while its own task writes the stream.  evb: per slot, the bands' event lists.
	Pool* bpool = nullptr;
	bool split = false;
	std::vector<std::vector<EvBuf>> evb;
	void set_split(int frames_in_flight)
	{
		static const bool en = [] { const char* e = getenv("RIC_BATCH_SPLIT"); return !e || atoi(e) != 0; }();
		split = en && pool && frames_in_flight * 2 <= pool->size();
		if (split && !bpool) bpool = new Pool(pool->size());
		if (split && evb.size() < (size_t)nslot()) evb.resize(nslot());
	}
	BProf prof;
	// GPU stream coder (gcoder.hip): argument block, per-slot results
	GEncArgs genc{};
	GEncArgs* d_genc = nullptr;
	GDecArgs gdec{};
	GDecArgs* d_gdec = nullptr;
	uint32_t* d_res = nullptr;                     // 2 per slot
	uint32_t* h_res = nullptr;                     // pinned
	// hybrid round trip: the pool of frames the GPU stream coder works on
	struct CoderPool {
		int n = 0;                                 // frames per coder launch
		size_t abstride = 0, ocap = 0;             // A+B bytes per plane pyramid, stream bytes per frame
		size_t fstride = 0;                        // bytes per frame: channels * abstride
		char* d_ab = nullptr;                      // 2 halves of n frames' bands + records
		uint8_t* d_out = nullptr;                  // 2 halves of n streams
		GEncArgs* d_args = nullptr;                // argument blocks, one per half
		GDecArgs* d_dargs = nullptr;
		GEncArgs args[2];
		GDecArgs dargs[2];
		uint32_t* d_res = nullptr;                 // per half: 2 n encoder words, n decoder words
		uint32_t* h_res = nullptr;                 // pinned mirror
		hipStream_t st[2] = {nullptr, nullptr};    // coder stream of each half
		hipEvent_t ev_fwd[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
		hipEvent_t ev_enc[2] = {nullptr, nullptr};   // a half's encode (and its result words) done
		uint64_t* d_ts = nullptr;                  // RIC_GC_TSTAMP: per half, the waves' start / end stamps
		// k_gc_roundtrip: per frame of both halves, the encoder's end offset and
		// status | 0x100, posted by the kernel into coherent host memory
		uint32_t* h_post = nullptr;
		uint32_t* d_post = nullptr;
		uint32_t* d_yield = nullptr;               // raised while the batch stream runs host frames' level kernels
		uint32_t epoch = 0;                        // the last coder launch's tag (posted words, k_gc_*)
		// Compacted pool (ric_batch_hybrid_config_ex): level 0's three bands of a
		// plane are held as a compact block (compact.h DcmpLayout: cmp_cap bytes,
		// at most vcap values) in front of the rest of its pyramid [lo, b_end);
		// the kernels' arena base of a plane is its region + ashift (= cmp_cap -
		// lo), so the pyramid offsets >= lo land after the block, and level 0
		// passes through the scratch arenas (ZFrames::lo).  vcap 0: dense pool.
		uint32_t vcap = 0;
		size_t lo = 0, cmp_cap = 0;
		long long ashift = 0;
		DcmpLayout dl;
		CmpArgs* d_pcmp = nullptr;                 // the forward compaction's arguments: [half][group][plane]
		int pcmp_groups = 0;
		uint32_t* d_pcnt = nullptr;                // its chunk counts / offsets (slots frames) and totals
		size_t pcnt_stride = 0;
		uint32_t* d_ptotal = nullptr;
	} cp;

	int nslot() const { return 2 * slots; }
	char* arena(int s) const { return d_arena + (size_t)s * astride; }
	char* harena(int s) const { return h_arena + (size_t)s * hstride; }
	int16_t* plane(int s, int p) const { return d_planes + (size_t)s * (pstride / 2) + (size_t)p * pitch * h; }
	uint8_t* stage(int s) const { return d_stage + (size_t)s * w * h * channels; }
	BandView view(int s, const Band& B) const
	{
		BandView v;
		v.p = harena(s) + B.off; v.pitch = B.pitch; v.dx = B.dx; v.dy = B.dy; v.is_int = B.is_int;
		return v;
	}
};

namespace {

// RIC_GC_PRIO: the stream coder waves' issue priority by progress (prio_band, level_step, gcoder.hip):
// 0 one priority, 1 steps at the finest H band of each phase, 2 steps through the decode's finest
// bands, 3 steps at the decode's finest H and D bands and half-way through D, 4 (default; the round-trip
// kernel, else 2's schedule is not applied) by rank among the coder waves of the same SIMD at every chunk,
// 5 the same ranks one priority lower.
// Measured (one C3 serving step, 3072 streams): mode 2 11011 ms per launch, the waves ending in three
// tiers (9.25 / 10.0 / 10.9 s); mode 4 10327 ms, every wave ending within 10.2-10.3 s
int gc_prio()
{
	static const int mode = [] { const char* e = getenv("RIC_GC_PRIO"); return e ? atoi(e) : 4; }();
	return mode;
}

int set_dev(int device) { return bfail(hipSetDevice(device), "hipSetDevice") ? RIC_E_HIP : RIC_OK; }

// The coder's yield flag (coder_yield, gcoder.hip) raised around a run of
// level kernels: lowered on every path out, errors included (a flag left up
// would make the coder waves sleep at every chunk until the next call)
struct YieldFlag {
	uint32_t* f;
	hipStream_t st;
	bool up = false;
	YieldFlag(uint32_t* flag, hipStream_t s) : f(flag), st(s) {}
	int raise()
	{
		if (!f || up) return RIC_OK;
		if (launch_gc_flag(f, 1, st)) return RIC_E_HIP;
		up = true;
		return RIC_OK;
	}
	int lower()
	{
		if (!f || !up) return RIC_OK;
		up = false;
		return launch_gc_flag(f, 0, st) ? RIC_E_HIP : RIC_OK;
	}
	~YieldFlag() { (void)lower(); }
};

// RIC_GC_YIELD 1 (the default since round 6): the coder waves yield around
// every level kernel of the host frames (forward and inverse); 2: only around
// their forward level 0 (the others run beside the coder waves unpaused); 0:
// never.  Round 4 (profiles/r04_yield_ab.json): 1 10491, 2 10561-10576, 0
// 10624 Mpix/s.  Round 6, with the waves levelled by rank (gcoder.hip mode 4)
// and the yield flag read a chunk ahead, same box, 4 timed steps each
// (profiles/r06_yield_ab.txt): 1 11,922-11,947 Mpix/s with the whole encode
// in the step at 0.396 of HBM peak; 2 11,745-11,947 at 0.363; 0 11,928-11,933
// at 0.342.
bool yield_level0_only()
{
	static const bool v = [] { const char* e = getenv("RIC_GC_YIELD"); return e && atoi(e) == 2; }();
	return v;
}

int quant_of(int q, int p) { return q ? quants(q + 20 + (p ? 8 : 0)) : 0; }    // Y, then chroma +C_Q_BOOST (ric.cpp:164-168)
int lambda_of(int q, int p) { return q ? quants(q + 13 + (p ? 8 : 0)) : 0; }

// The GPU half of CompressImage for plane p of n frames of set `set`: pixel
// conversion (p == 0), every forward level + quantiser + block records as one
// launch per level over the group, then the bands + records of every frame
// to the host mirrors (one strided copy).  pix: device pixels of each frame.
// abase / amul: frame i's arena is arena(abase + i * amul) (default: the
// set's slots, abase = set * slots, amul 1); the GPU stream coder of colour
// frames keeps a frame's three plane pyramids side by side (amul 3).
// yflag: the GPU stream coder's yield flag (coder_yield, gcoder.hip), raised
// around the level kernels only (not the copies), or null
int d2h_slots(ric_batch* b, int set, int n, hipStream_t cst = nullptr);

// pool (the GPU stream coder's pool, pstr bytes per frame): regions A and B
// of frame i go to pool + i * pstr instead of its arena -- written there by
// the level kernels directly when every level is a fused one (region C, the
// scratch, stays in the arena), else copied there after the levels.
// lo (a compacted pool, CoderPool): pool is the frames' kernel base and the
// offsets below lo (level 0's bands) stay in the arenas, for the compaction
int gpu_encode_plane(ric_batch* b, int set, int n, int p, const uint8_t* const* pix, int q, int trans, bool d2h = true,
                     int abase = -1, int amul = 1, uint32_t* yflag = nullptr, char* pool = nullptr, size_t pstr = 0,
                     size_t lo = 0)
{
	const bool y0only = yield_level0_only();
	YieldFlag yf(yflag, b->st);
	if (!y0only && yf.raise()) return RIC_E_HIP;
	Pyramid& P = b->P;
	const int s0 = set * b->slots;
	if (abase < 0) abase = s0;
	const size_t ast = (size_t)amul * b->astride;
	bool direct = pool != nullptr;
	if (pool) {
		// direct writes need every level fused, the coarsest with the LL TSUQ
		P.set_weight(trans);
		const int lambda = lambda_of(q, p);
		int qin = quant_of(q, p);
		for (int l = 0; l < P.nlev && direct; l++) {
			const int mode = fwdq_mode(P.L[l], trans, level_qp(P, l, qin, lambda), 1);
			direct = mode != FQ_NONE && (l + 1 < P.nlev || mode == FQ_GENERIC);
		}
		if (direct) BCHK(hipMemset2DAsync(pool + P.status_off, pstr, 0, sizeof(int32_t), n, b->st));
	}
	const int quant = quant_of(q, p), lambda = lambda_of(q, p);
	P.set_weight(trans);
	// a gray frame's level 0 reads its u8 pixels itself (k_fwdq_pc_z8, the
	// level shift fused): no coding plane written or read (RIC_PIX8=0: off)
	static const bool pix8_on = [] { const char* e = getenv("RIC_PIX8"); return !e || atoi(e) != 0; }();
	int q0 = quant;
	bool u8 = pix8_on && p == 0 && b->channels == 1 && n <= 32 && (b->w & 7) == 0 &&
	          fwdq_mode(P.L[0], trans, level_qp(P, 0, q0, lambda), 1) == FQ_PACKED;
	for (int i = 0; i < n && u8; i++) u8 = ((uintptr_t)pix[i] & 7) == 0;
	if (p == 0 && !u8) {
		auto sp = b->prof.begin(B_PIXIN, n, b->st);
		for (int i = 0; i < n; i++) launch_pix_in(pix[i], b->plane(s0 + i, 0), b->w, b->h, b->pitch, b->channels, q, b->st);
		b->prof.end(sp);
	}
	bool fused[kMaxLevels] = {};
	bool ll_done = false;
	int qin = quant;
	for (int l = 0; l < P.nlev; l++) {
		ZFrames fr;
		fr.arena = b->arena(abase); fr.astride = ast; fr.nz = n;
		fr.ring = b->fq_ring;
		fr.pc1 = b->fq_pc1;
		if (direct) {
			fr.arena = pool; fr.astride = pstr;
			fr.scratch = b->arena(abase); fr.scstride = ast; fr.split = P.b_end; fr.lo = lo;
		}
		if (l == 0) {
			fr.src = b->plane(s0, p); fr.sstride = b->pstride; fr.sp = b->pitch;
			if (u8) { fr.pix8 = pix; fr.sh8 = q ? 4 : 0; }   // SHIFT, src/ric/ric.cpp:39,144-148
		} else {
			const Band& LL = P.L[l - 1].b[BL];
			fr.src = b->arena(abase) + LL.off; fr.sstride = ast; fr.sp = LL.pitch;
		}
		// coding planes: 64-element row pitch, 256-byte aligned slots
		const int vec8 = 1, vec16 = 1;
		QuantParams qp = level_qp(P, l, qin, lambda);
		const int mode = fwdq_mode(P.L[l], trans, qp, vec16);
		fused[l] = mode != FQ_NONE;
		// (the yield flag's one-wave kernels outside the level's timed span)
		if (y0only && l == 0 && yf.raise()) return RIC_E_HIP;
		if (y0only && l == 1 && yf.lower()) return RIC_E_HIP;
		auto sp = b->prof.begin(B_FWD + std::min(l, 7), n, b->st);
		if (mode == FQ_PACKED) {
			// the batch's planes are 8-bit pixels after the level shift (in8)
			if (launch_fwdq_level_z(P, l, fr, vec8, vec16, qp, b->zf[set][l], b->st, 1)) return RIC_E_HIP;
		} else if (mode == FQ_GENERIC) {
			const bool coarsest = l + 1 == P.nlev;
			int llQ = 0, lliQ = 0, llT0 = 0;
			if (coarsest) { ll_params(P, quant, llQ, lliQ, llT0); ll_done = true; }
			if (launch_fwdq_gen_level_z(P, l, fr, vec8, qp, coarsest, lliQ, llT0, b->zf[set][l], b->st)) return RIC_E_HIP;
		} else {
			// unfused levels (5/3, Haar): the per-frame kernels
			for (int i = 0; i < n; i++) {
				char* ar = b->arena(abase + i * amul);
				launch_fwd_level(P.L[l], (const char*)fr.src + i * fr.sstride, fr.sp, ar, trans, vec8, b->st);
				launch_quant_level(P, l, qp, ar, b->st);
			}
		}
		b->prof.end(sp);
	}
	for (int i = 0; i < n; i++) {
		char* ar = b->arena(abase + i * amul);
		if (!ll_done) {
			int Q, iQ, T0;
			ll_params(P, quant, Q, iQ, T0);
			launch_quant_ll(P, Q, iQ, T0, ar, b->st);
		}
		for (int l = 0; l < P.nlev; l++)
			if (!fused[l] || (l + 1 < P.nlev && !fused[l + 1]))
				launch_blocks_level(P, l, !fused[l], l + 1 < P.nlev && !fused[l + 1], ar, b->st);
	}
	BCHK(hipGetLastError());
	if (yf.lower()) return RIC_E_HIP;
	if (pool && !direct)
		BCHK(hipMemcpy2DAsync(pool + lo, pstr, b->arena(abase) + lo, ast, P.b_end - lo, n, hipMemcpyDeviceToDevice, b->st));
	if (!d2h || pool) return RIC_OK;
	if (abase != s0 || amul != 1) return RIC_E_ARG;      // the host mirrors follow the slots
	return d2h_slots(b, set, n);
}

// The bands + records of slots set * slots .. + n - 1 (after their forward
// levels) to the host mirrors: the compacted 16-bit values and the dense rest
// (or the dense arenas).  Colour frames of a hybrid host group take C slots
// each (plane p of frame i in slot C i + p), so n counts slots, not frames.
// cst (or null: the batch stream): the stream of the copies (the compaction
// kernels stay on the batch stream; cst waits for them) -- the step's front
// puts its second host group's copies beside the pool's forward levels
int d2h_slots(ric_batch* b, int set, int n, hipStream_t cst)
{
	Pyramid& P = b->P;
	const int s0 = set * b->slots;
	hipStream_t xs = cst ? cst : b->st;
	auto fork = [&]() -> int {
		if (xs == b->st) return RIC_OK;
		if (!b->ev_fork) BCHK(hipEventCreateWithFlags(&b->ev_fork, hipEventDisableTiming));
		BCHK(hipEventRecord(b->ev_fork, b->st));
		BCHK(hipStreamWaitEvent(xs, b->ev_fork, 0));
		return RIC_OK;
	};
	if (b->compact) {
		// the 16-bit bands' values in walk order (compact.hip), written by a
		// kernel into the head of each frame's host mirror (only the values,
		// no per-frame copy on another stream: the host tasks find them there
		// once the group's event has passed); their counts and the dense rest
		// (int bands, LL, region B) by copies
		{
			auto sc = b->prof.begin(B_CMP, n, b->st);
			if (launch_compact(b->d_cmp_args + set, b->cmp_nchunk, n, b->st)) return bfail(hipGetLastError(), "compact") ? RIC_E_HIP : RIC_E_HIP;
			b->prof.end(sc);
		}
		if (int r = fork()) return r;
		BCHK(hipMemcpyAsync(b->h_cmp_total + s0, b->d_cmp_total + s0, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, xs));
		{
			auto sv = b->prof.begin(B_D2HV, n, xs);
			// In the serving step (cmp_dma): the values' whole capacity by the
			// copy engine -- about twice the bytes of the values, but no CUs
			// taken from the stream coder's launch: a kernel writing each frame's
			// count into the device-mapped mirror held CUs for the PCIe writes
			// and slowed the launch by 3 % (C3 step: 11,363-11,382 against
			// 11,168 Mpix/s, profiles/r05_cmp_dma_ab.json).  Elsewhere the kernel
			// (only the values cross PCIe).  RIC_CMP_DMA=0/1 forces either.
			static const int dma_env = [] { const char* e = getenv("RIC_CMP_DMA"); return e ? atoi(e) : -1; }();
			const bool dma = dma_env >= 0 ? dma_env != 0 : b->cmp_dma;
			if (dma || xs != b->st) {
				BCHK(hipMemcpy2DAsync(b->harena(s0), b->hstride, b->d_cmp + (size_t)s0 * b->cmp_stride, b->cmp_stride,
				                      std::min(b->cmp_stride, b->hstride), n, hipMemcpyDeviceToHost, xs));
			} else if (launch_cmp_to_host(b->d_cmp + (size_t)s0 * b->cmp_stride, b->cmp_stride, b->h_arena_dev + (size_t)s0 * b->hstride,
			                              b->hstride, b->d_cmp_total + s0, n, b->st))
				return bfail(hipGetLastError(), "compact to host") ? RIC_E_HIP : RIC_E_HIP;
			b->prof.end(sv);
		}
		auto sp = b->prof.begin(B_D2H, n, xs);
		BCHK(hipMemcpy2DAsync(b->harena(s0) + b->cmp_dense, b->hstride, b->arena(s0) + b->cmp_dense, b->astride,
		                      P.b_end - b->cmp_dense, n, hipMemcpyDeviceToHost, xs));
		b->prof.end(sp);
		for (int i = 0; i < n; i++) b->cmp_ok[s0 + i] = 1;
		return RIC_OK;
	}
	if (int r = fork()) return r;
	auto sp = b->prof.begin(B_D2H, n, xs);
	BCHK(hipMemcpy2DAsync(b->harena(s0), b->hstride, b->arena(s0), b->astride, P.b_end, n, hipMemcpyDeviceToHost, xs));
	b->prof.end(sp);
	return RIC_OK;
}

// The host-decoded bands of slots set * slots .. + n - 1 to the device: one
// strided copy (levels 1.. dense and each slot's compacted finest level,
// scattered by k_dcmp_expand; or the dense arenas).  n counts slots (colour
// frames of a hybrid host group take C slots each).
int h2d_slots(ric_batch* b, int set, int n)
{
	Pyramid& P = b->P;
	const int s0 = set * b->slots;
	{
		bool cmp = b->dcompact;
		for (int i = 0; i < n && cmp; i++) cmp = b->dcmp_ok[s0 + i] != 0;
		auto sp = b->prof.begin(B_H2D, n, b->st);
		if (cmp) {
			// levels 1.. and the LL dense; each frame's compacted finest level,
			// scattered into its three bands on the device
			const size_t d0 = P.L[1].b[BD].off;
			BCHK(hipMemcpy2DAsync(b->arena(s0) + d0, b->astride, b->harena(s0) + d0, b->hstride, P.a_end - d0, n,
			                      hipMemcpyHostToDevice, b->st));
			for (int i = 0; i < n; i++) {
				BCHK(hipMemcpyAsync(b->d_cmp + (size_t)(s0 + i) * b->cmp_stride, b->harena(s0 + i), b->dcmp_bytes[s0 + i],
				                    hipMemcpyHostToDevice, b->st));
				b->dcmp_ok[s0 + i] = 0;
			}
			DcmpArgs a;
			a.arena = b->arena(s0); a.astride = b->astride;
			a.in = b->d_cmp + (size_t)s0 * b->cmp_stride; a.istride = b->cmp_stride;
			int ch = 0;
			for (int k = 0; k < 3; k++) {
				const Band& B = P.L[0].b[b->dl.band[k]];
				a.off[k] = (uint32_t)B.off; a.dx[k] = B.dx; a.dy[k] = B.dy; a.pitch[k] = B.pitch;
				a.mask_off[k] = (uint32_t)b->dl.mask_off[k]; a.coff_off[k] = (uint32_t)b->dl.coff_off[k];
				a.nblk[k] = b->dl.nblk[k];
				a.chunk0[k] = ch;
				ch += b->dl.nch[k];
			}
			a.chunk0[3] = ch;
			a.vals_off = (uint32_t)b->dl.vals_off;
			auto sx = b->prof.begin(B_DEXP, n, b->st);
			if (launch_dcmp_expand(a, n, b->st)) return bfail(hipGetLastError(), "k_dcmp_expand") ? RIC_E_HIP : RIC_E_HIP;
			b->prof.end(sx);
		} else {
			BCHK(hipMemcpy2DAsync(b->arena(s0), b->astride, b->harena(s0), b->hstride, P.a_end, n, hipMemcpyHostToDevice, b->st));
		}
		b->prof.end(sp);
	}
	return RIC_OK;
}

// The GPU half of DecompressImage for plane p of n frames of set `set`: the
// host-decoded bands to the device (one strided copy), then every inverse
// level with the fused TSUQi factors of each frame, as one launch per level.
// pool (as gpu_encode_plane): the decoded bands of frame i are read from
// pool + i * pstr (region A) while the inverse's intermediate LL planes
// (region C) stay in the frame's arena -- no copy of the bands.
// lo (a compacted pool): level 0's bands are read from the arenas (expanded
// there from the pool's compact blocks)
// The pixel output fused into level 0's inverse (a gray 9/7 frame: ZFrames::pix):
// frames' device pixel buffers, their quantisers, and frames idx0.. of the
// call for the digests (ric_batch_set_digests)
struct PixFuse {
	uint8_t* const* pix;
	const int* q;
	long idx0;
};
// RIC_PIX_FUSE=0: the separate pixel output kernel after the inverse
bool pix_fuse_ok(const ric_batch* b, int trans, uint8_t* const* pix, int n)
{
	static const bool on = [] { const char* e = getenv("RIC_PIX_FUSE"); return !e || atoi(e) != 0; }();
	if (!on || b->channels != 1 || trans != CDF97 || (b->w & 3) || b->P.L[0].is_int) return false;
	for (int i = 0; i < n; i++)
		if (!pix[i] || ((uintptr_t)pix[i] & 3)) return false;
	return true;
}

int gpu_decode_plane(ric_batch* b, int set, int n, int p, const int* qs, int trans, bool h2d = true, int abase = -1,
                     int amul = 1, uint32_t* yflag = nullptr, char* pool = nullptr, size_t pstr = 0, size_t lo = 0,
                     const PixFuse* pf = nullptr)
{
	Pyramid& P = b->P;
	const int s0 = set * b->slots;
	if (abase < 0) abase = s0;
	if (h2d && (abase != s0 || amul != 1 || pool)) return RIC_E_ARG;
	const size_t ast = (size_t)amul * b->astride;
	if (h2d) {
		const int r = h2d_slots(b, set, n);
		if (r) return r;
	}
	P.set_weight(trans);
	YieldFlag yf(yield_level0_only() ? nullptr : yflag, b->st);
	if (yf.raise()) return RIC_E_HIP;                                    // (after the copies)
	std::vector<int> qf(4 * n);
	for (int l = P.nlev - 1; l >= 0; l--) {
		const Level& L = P.L[l];
		ZFrames fr;
		fr.arena = b->arena(abase); fr.astride = ast; fr.nz = n;
		if (pool) {
			fr.arena = pool; fr.astride = pstr;
			fr.scratch = b->arena(abase); fr.scstride = ast; fr.split = P.b_end; fr.lo = lo;
		}
		int out_int;
		long ndig = 0;
		if (l == 0) {
			fr.out = b->plane(s0, p); fr.ostride = b->pstride; fr.po = b->pitch; out_int = 0;
			if (pf) {
				fr.pix = pf->pix; fr.pix_q = pf->q;
				ndig = b->digest && pf->idx0 >= 0 ? std::max(0L, std::min((long)n, b->ndigest - pf->idx0)) : 0;
				if (ndig) {
					if (!b->d_dpart) BCHK(hipMalloc(&b->d_dpart, sizeof(unsigned long long) * 16 * 2 * (size_t)b->slots));
					if (n > 2 * b->slots) return RIC_E_ARG;
					BCHK(hipMemsetAsync(b->d_dpart, 0, sizeof(unsigned long long) * 16 * (size_t)n, b->st));
					fr.dig_part = b->d_dpart;
				}
			}
		} else {
			const Band& LL = P.L[l - 1].b[BL];
			fr.out = b->arena(abase) + LL.off; fr.ostride = ast; fr.po = LL.pitch; out_int = LL.is_int;
		}
		for (int i = 0; i < n; i++) {
			const int quant = quant_of(qs[i], p);
			int* f = &qf[4 * i];
			if (quant) {
				f[0] = tsuqi_factor(L.b[BD], quant); f[1] = tsuqi_factor(L.b[BH], quant); f[2] = tsuqi_factor(L.b[BV], quant);
				f[3] = l + 1 == P.nlev ? tsuqi_factor(L.b[BL], quant) : 1;
			} else {
				f[0] = f[1] = f[2] = f[3] = 1;    // lossless: no TSUQi (ric.cpp:213)
			}
		}
		auto si = b->prof.begin(B_INV + std::min(l, 7), n, b->st);
		if (launch_inv_level_z(L, L.b[BL], fr, out_int, trans, qf.data(), b->zi[set][l], b->st)) return RIC_E_HIP;
		b->prof.end(si);
		if (ndig) launch_digest_fold(b->d_dpart, b->digest + pf->idx0, (int)ndig, b->st);
	}
	if (yf.lower()) return RIC_E_HIP;
	BCHK(hipGetLastError());
	return RIC_OK;
}

// pixel output of n frames of set `set` (after every plane's inverse)
// idx0 >= 0: these are frames idx0.. of the call, whose digests
// (ric_batch_set_digests) are taken right after their pixels are written.
int gpu_pix_out(ric_batch* b, int set, int n, const int* qs, uint8_t* const* pix_out, int on_device, long idx0 = -1)
{
	const int s0 = set * b->slots;
	auto sp = b->prof.begin(B_PIXOUT, n, b->st);
	// every frame of the group below ndigest gets its digest (a group may
	// straddle the limit)
	const long ndig = b->digest && idx0 >= 0 ? std::max(0L, std::min((long)n, b->ndigest - idx0)) : 0;
	if (ndig) BCHK(hipMemsetAsync(b->digest + idx0, 0, sizeof(unsigned long long) * ndig, b->st));
	for (int i = 0; i < n; i++) {
		if (!pix_out[i]) continue;
		uint8_t* dst = on_device ? pix_out[i] : b->stage(s0 + i);
		launch_pix_out(b->plane(s0 + i, 0), b->pitch, b->w, b->h, b->channels, qs[i], dst, nullptr, b->st,
		               i < ndig ? b->digest + idx0 + i : nullptr);
	}
	b->prof.end(sp);
	BCHK(hipGetLastError());
	if (!on_device)
		for (int i = 0; i < n; i++)
			if (pix_out[i])
				BCHK(hipMemcpyAsync(pix_out[i], b->stage(s0 + i), (size_t)b->w * b->h * b->channels, hipMemcpyDeviceToHost, b->st));
	return RIC_OK;
}

// Host coder of plane p of the frame in slot s.  Encode: the .ric file is
// written in place into out (the coder buffer starts at out + 7, so the
// payload lands at out + 9 and the two dropped leading coder bytes are
// overwritten by the header at the end).  ms: the slot whose coder carries
// the frame's stream across its planes (default s; a hybrid colour frame keeps
// each plane in a slot of its own, the stream in its first).
int host_encode_plane(ric_batch* b, int s, int p, int q, int trans, uint8_t* out, size_t cap, size_t* len, int ms = -1)
{
	Pyramid& P = b->P;
	Mux& m = b->enc[ms < 0 ? s : ms];
	if (p == 0) {
		if (cap < 16) return RIC_E_CAPACITY;
		m.init_encoder(out + 7, cap - 7, 0);
	}
	int32_t* status = (int32_t*)(b->harena(s) + P.status_off);
	if (*status) {
		*status = 0;
		set_last_error("device status word set: a fused level kernel's LDS ring hand-off or the compaction's look-back timed out; output discarded");
		return RIC_E_HIP;
	}
	const int16_t* cp = nullptr;
	if (b->compact && b->cmp_ok[s]) {
		// this frame's compacted values, already in the mirror's head (k_cmp_to_host)
		if ((size_t)b->h_cmp_total[s] * 2 > b->cmp_stride)
			return set_last_error("compacted payload larger than its slot"), RIC_E_HIP;
		cp = (const int16_t*)b->harena(s);
	}
	const double t0 = now_ms();
	if (b->split && b->bpool) {
		// the bands modelled in parallel (a compacted band's values start where
		// the walk's previous compacted bands' end), the stream written here
		BandRecs bands[3 * kMaxLevels];
		int nb = 0;
		const int16_t* c0 = cp;
		for (int l = P.nlev - 1; l >= 0; l--) {
			const int order[3] = {BV, BH, BD};
			for (int k = 0; k < 3; k++) {
				const Band& B = P.L[l].b[order[k]];
				BandRecs& r = bands[nb++];
				r.rec = (const uint64_t*)(b->harena(s) + P.rec_off[l][order[k]]);
				r.pin = l + 1 < P.nlev ? (const uint8_t*)(b->harena(s) + P.pin_off[l][order[k]]) : nullptr;
				r.v = b->view(s, B);
				r.high = l == 0;
				r.cvals = nullptr;
				if (c0 && !B.is_int) {
					r.cvals = c0;
					c0 += band_value_count(r.rec, r.v);
				}
			}
		}
		encode_bands_split(m, *b->bpool, b->evb[ms < 0 ? s : ms], b->view(s, P.coarsest_ll()), bands, nb);
	} else {
		pred_encode(m, b->view(s, P.coarsest_ll()));
		for (int l = P.nlev - 1; l >= 0; l--) {
			const int order[3] = {BV, BH, BD};
			for (int k = 0; k < 3; k++) {
				const Band& B = P.L[l].b[order[k]];
				const uint64_t* rec = (const uint64_t*)(b->harena(s) + P.rec_off[l][order[k]]);
				const uint8_t* pin = l + 1 < P.nlev ? (const uint8_t*)(b->harena(s) + P.pin_off[l][order[k]]) : nullptr;
				if (cp && !B.is_int) tree_encode_records_compact(m, rec, pin, b->view(s, B), l == 0, &cp);
				else tree_encode_records_fast(m, rec, pin, b->view(s, B), l == 0);
			}
		}
	}
	if (p + 1 == b->channels) {
		uint8_t* e = m.end_coding();
		if (m.overflow()) return RIC_E_CAPACITY;
		const size_t n = (size_t)(e - (out + 7));
		*len = 9 + n - 2;
		memcpy(out, "RUD2", 4);
		out[4] = b->w & 255; out[5] = (b->w >> 8) & 255; out[6] = b->h & 255; out[7] = (b->h >> 8) & 255;
		out[8] = (uint8_t)((q & 31) | ((b->channels == 3) << 5) | ((trans & 3) << 6));
	}
	b->prof.host(B_HENC, now_ms() - t0);
	return RIC_OK;
}

// Host decoder of plane p of one .ric file into the host mirror of slot s
// (CWavelet2D::DecodeBand, src/lib/wavelet2d.cpp:179-222).
int host_decode_plane(ric_batch* b, int s, int p, const uint8_t* ric, size_t len, int ms = -1)
{
	Pyramid& P = b->P;
	Mux& m = b->dec[ms < 0 ? s : ms];
	if (p == 0) {
		// the reference reads W*H*C payload bytes (ric.cpp:203-205)
		const size_t pay = std::min(len - 9, (size_t)b->w * b->h * b->channels);
		m.init_decoder_payload(ric + 9, pay);
	}
	const double t0 = now_ms();
	// the finest level compacted into the mirror's level-0 area (DcmpLayout)
	const bool cmp = b->dcompact;
	char* blk = b->harena(s);
	uint32_t* nval = (uint32_t*)blk;
	pred_decode(m, b->view(s, P.coarsest_ll()));
	for (int l = P.nlev - 1; l >= 0; l--) {
		const int order[3] = {BV, BH, BD};
		uint32_t vsum = 0;
		for (int k = 0; k < 3; k++) {
			BandView par;
			if (l + 1 < P.nlev) par = b->view(s, P.L[l + 1].b[order[k]]);
			if (cmp && l == 0) {
				const DcmpLayout& L = b->dl;
				nval[k] = tree_decode_compact(m, b->view(s, P.L[l].b[order[k]]), par, (uint16_t*)(blk + L.mask_off[k]),
				                              (uint32_t*)(blk + L.coff_off[k]), (int16_t*)(blk + L.vals_off) + vsum);
				vsum += nval[k];
				b->dcmp_bytes[s] = L.vals_off + (size_t)vsum * 2;
			} else {
				tree_decode_fast(m, b->view(s, P.L[l].b[order[k]]), par, l == 0, l > 0);
			}
		}
	}
	if (cmp) b->dcmp_ok[s] = 1;
	b->prof.host(B_HDEC, now_ms() - t0);
	return m.overflow() ? RIC_E_STREAM : RIC_OK;
}

// keeps the first error of a group's tasks (RIC_E_STREAM only if nothing worse)
struct FirstErr {
	std::atomic<int> rc{RIC_OK};
	std::mutex mu;
	std::string msg;
	void put(int r)
	{
		if (r == RIC_OK) return;
		std::lock_guard<std::mutex> g(mu);
		const int cur = rc.load();
		if (cur == RIC_OK || (cur == RIC_E_STREAM && r != RIC_E_STREAM)) {
			rc.store(r);
			msg = ric_last_error();    // the worker thread's message
		}
	}
	int get()
	{
		const int r = rc.load();
		if (r != RIC_OK && r != RIC_E_STREAM) set_last_error(msg);
		return r;
	}
};

// Two frames of one call must not share an output buffer: different threads
// (host coders, the stream copier) write them concurrently.
bool outputs_distinct(uint8_t* const* out, int n)
{
	std::vector<uint8_t*> v(out, out + n);
	std::sort(v.begin(), v.end());
	return std::adjacent_find(v.begin(), v.end()) == v.end();
}

// a device -> host copy on one of the batch's copy streams (lane: any
// integer), waited for on that stream alone
hipError_t d2h(ric_batch* b, long lane, void* dst, const void* src, size_t n)
{
	hipStream_t st = b->cst[lane & 3];
	const hipError_t e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, st);
	return e != hipSuccess ? e : hipStreamSynchronize(st);
}

// frame f's .ric file is complete in its host buffer (ric_batch_set_ready)
void mark_ready(ric_batch* b, long f, size_t len)
{
	if (b->ready && f < b->nready) __atomic_store_n(b->ready + f, (uint32_t)len, __ATOMIC_RELEASE);
}

int check_header(ric_batch* b, const uint8_t* ric, size_t len, int* q, int* trans)
{
	int w, h, ch;
	int rc = ric_read_header(ric, len, &w, &h, &ch, q, trans);
	if (rc) return rc;
	if (w != b->w || h != b->h || ch != b->channels || *trans > 2) return RIC_E_ARG;
	return RIC_OK;
}

// after a failed call: clear every slot's device status word (a fused
// kernel's ring timeout, see host_encode_plane) so the next call starts clean
void clear_status(ric_batch* b)
{
	for (int s = 0; s < b->nslot(); s++)
		(void)hipMemsetAsync(b->arena(s) + b->P.status_off, 0, sizeof(int32_t), b->st);
	(void)hipStreamSynchronize(b->st);
}

// device pixel pointers of n frames, staging host pixels through the slots
int stage_pixels(ric_batch* b, int set, int n, const uint8_t* const* pix, int on_device, std::vector<const uint8_t*>& dpix)
{
	dpix.resize(n);
	for (int i = 0; i < n; i++) {
		if (on_device) { dpix[i] = pix[i]; continue; }
		uint8_t* d = b->stage(set * b->slots + i);
		BCHK(hipMemcpyAsync(d, pix[i], (size_t)b->w * b->h * b->channels, hipMemcpyHostToDevice, b->st));
		dpix[i] = d;
	}
	return RIC_OK;
}

}  // namespace

extern "C" {

int ric_batch_create(ric_batch** out, int w, int h, int channels, int slots, int threads, int device)
{
	if (!out || w < 8 || h < 8 || w > 65535 || h > 65535 || (channels != 1 && channels != 3) || slots < 1 || slots > 4096 ||
	    threads < 1 || threads > 1024)
		return RIC_E_ARG;
	*out = nullptr;
	if (set_dev(device)) return RIC_E_HIP;
	ric_batch* b = new ric_batch;
	b->device = device; b->w = w; b->h = h; b->channels = channels; b->slots = slots;
	b->P.build(w, h, 5, 1);     // WAV_LEVELS 5, level_chg 1 (ric.cpp:159)
	b->P.set_weight(CDF97);
	auto up = [](size_t v, size_t a) { return (v + a - 1) / a * a; };
	b->astride = up(b->P.arena_bytes, 1 << 16);
	b->hstride = up(b->P.b_end, 4096);
	b->pitch = ((long)w + 63) / 64 * 64;
	b->pstride = up((size_t)b->pitch * h * channels * 2, 1 << 16);
	const size_t ns = (size_t)b->nslot();
	if (bfail(hipMalloc(&b->d_arena, ns * b->astride), "hipMalloc batch arena") ||
	    bfail(hipHostMalloc(&b->h_arena, ns * b->hstride, 0), "hipHostMalloc batch mirror") ||
	    bfail(hipMalloc(&b->d_planes, ns * b->pstride), "hipMalloc batch planes") ||
	    bfail(hipMalloc(&b->d_stage, ns * (size_t)w * h * channels), "hipMalloc batch staging") ||
	    bfail(hipStreamCreateWithFlags(&b->st, hipStreamNonBlocking), "hipStreamCreate") ||
	    bfail(hipStreamCreateWithFlags(&b->cst[0], hipStreamNonBlocking), "hipStreamCreate") ||
	    bfail(hipStreamCreateWithFlags(&b->cst[1], hipStreamNonBlocking), "hipStreamCreate") ||
	    bfail(hipStreamCreateWithFlags(&b->cst[2], hipStreamNonBlocking), "hipStreamCreate") ||
	    bfail(hipStreamCreateWithFlags(&b->cst[3], hipStreamNonBlocking), "hipStreamCreate") ||
	    bfail(hipMemsetAsync(b->d_arena, 0, ns * b->astride, b->st), "hipMemset batch arena") ||
	    bfail(hipStreamSynchronize(b->st), "hipStreamSynchronize")) {
		ric_batch_destroy(b);
		return RIC_E_HIP;
	}
	memset(b->h_arena, 0, ns * b->hstride);
	// compacted payloads (RIC_COMPACT=0: dense bands to the host)
	static const bool cmp_env = [] { const char* e = getenv("RIC_COMPACT"); return !e || atoi(e) != 0; }();
	b->compact = cmp_env;
	if (b->compact) {
		CmpArgs a{};
		cmp_args(b->P, a);
		b->cmp_nchunk = a.nchunk;
		b->cmp_dense = cmp_dense_from(b->P);
		b->cmp_stride = up(cmp_values(b->P) * 2, 256);
		b->cmp_cstride = up((size_t)a.nchunk, 64);
		b->cmp_ok.assign(ns, 0);
		bool bad = b->cmp_stride > b->cmp_dense ||      // the values land in the mirror's band area
		           bfail(hipMalloc(&b->d_cmp, ns * b->cmp_stride), "hipMalloc compact") ||
		           bfail(hipMalloc(&b->d_cmp_cnt, ns * b->cmp_cstride * sizeof(uint32_t)), "hipMalloc compact") ||
		           bfail(hipMemset(b->d_cmp_cnt, 0, ns * b->cmp_cstride * sizeof(uint32_t)), "hipMemset compact") ||
		           bfail(hipMalloc(&b->d_cmp_total, ns * sizeof(uint32_t)), "hipMalloc compact") ||
		           bfail(hipHostMalloc(&b->h_cmp_total, ns * sizeof(uint32_t), 0), "hipHostMalloc compact") ||
		           bfail(hipMalloc(&b->d_cmp_args, 2 * sizeof(CmpArgs)), "hipMalloc compact");
		if (!bad) bad = bfail(hipHostGetDevicePointer((void**)&b->h_arena_dev, b->h_arena, 0), "hipHostGetDevicePointer");
		CmpArgs h[2];
		for (int set = 0; set < 2 && !bad; set++) {
			h[set] = a;
			const size_t s0 = (size_t)set * slots;
			h[set].arena = b->arena((int)s0); h[set].astride = b->astride;
			h[set].out = b->d_cmp + s0 * b->cmp_stride; h[set].ostride = b->cmp_stride;
			h[set].cnt = b->d_cmp_cnt + s0 * b->cmp_cstride; h[set].cstride = b->cmp_cstride;
			h[set].total = b->d_cmp_total + s0;
			// (the one-pass kernel's kCmpLookback: the status word fails the frame)
			h[set].status = b->arena((int)s0) + b->P.status_off; h[set].sstride = b->astride;
		}
		if (!bad) bad = bfail(hipMemcpy(b->d_cmp_args, h, sizeof(h), hipMemcpyHostToDevice), "hipMemcpy compact");
		if (bad) {
			ric_batch_destroy(b);
			return RIC_E_HIP;
		}
		// decode side: the block must fit the mirror's level-0 area and a device slot
		b->dl = dcmp_layout(b->P);
		size_t l0 = 0;
		for (int k = 0; k < 3; k++) l0 += (size_t)b->P.L[0].b[k].dx * b->P.L[0].b[k].dy;
		const size_t most = b->dl.vals_off + l0 * 2;
		b->dcompact = b->dl.ok && most <= b->P.L[1].b[BD].off && most <= b->cmp_stride;
		b->dcmp_bytes.assign(ns, 0);
		b->dcmp_ok.assign(ns, 0);
	}
	b->enc = std::vector<Mux>(ns);
	b->dec = std::vector<Mux>(ns);
	b->pool = new Pool(threads);
	*out = b;
	return RIC_OK;
}

void ric_batch_destroy(ric_batch* b)
{
	if (!b) return;
	delete b->pool;
	delete b->bpool;
	(void)hipSetDevice(b->device);
	if (b->st) (void)hipStreamSynchronize(b->st);
	for (int s = 0; s < 2; s++)
		for (int l = 0; l < kMaxLevels; l++) { zargs_free(b->zf[s][l]); zargs_free(b->zi[s][l]); }
	b->prof.destroy();
	if (b->d_arena) (void)dev_free(b->d_arena);
	if (b->h_arena) (void)pinned_free(b->h_arena);
	if (b->d_cmp) (void)dev_free(b->d_cmp);
	if (b->d_cmp_cnt) (void)dev_free(b->d_cmp_cnt);
	if (b->d_cmp_total) (void)dev_free(b->d_cmp_total);
	if (b->h_cmp_total) (void)pinned_free(b->h_cmp_total);
	if (b->d_cmp_args) (void)dev_free(b->d_cmp_args);
	if (b->d_planes) (void)dev_free(b->d_planes);
	if (b->d_stage) (void)dev_free(b->d_stage);
	if (b->d_genc) (void)dev_free(b->d_genc);
	if (b->d_gdec) (void)dev_free(b->d_gdec);
	if (b->d_res) (void)dev_free(b->d_res);
	if (b->h_res) (void)pinned_free(b->h_res);
	{
		auto& c = b->cp;
		for (int h = 0; h < 2; h++)
			if (c.st[h]) (void)hipStreamSynchronize(c.st[h]);
		if (c.d_ab) (void)dev_free(c.d_ab);
		if (c.d_out) (void)dev_free(c.d_out);
		if (c.d_args) (void)dev_free(c.d_args);
		if (c.d_dargs) (void)dev_free(c.d_dargs);
		if (c.h_res) (void)pinned_free(c.h_res);
		if (c.d_ts) (void)dev_free(c.d_ts);
		if (c.h_post) (void)pinned_free(c.h_post);
		if (c.d_yield) (void)dev_free(c.d_yield);
		if (b->d_dpart) (void)dev_free(b->d_dpart);
		if (b->xst) (void)hipStreamSynchronize(b->xst);
		if (b->ev_fork) (void)hipEventDestroy(b->ev_fork);
		if (b->xst) (void)hipStreamDestroy(b->xst);
		if (c.d_pcmp) (void)dev_free(c.d_pcmp);
		if (c.d_pcnt) (void)dev_free(c.d_pcnt);
		if (c.d_ptotal) (void)dev_free(c.d_ptotal);
		for (int h = 0; h < 2; h++) {
			if (c.ev_fwd[h]) (void)hipEventDestroy(c.ev_fwd[h]);
			if (c.ev_done[h]) (void)hipEventDestroy(c.ev_done[h]);
			if (c.ev_enc[h]) (void)hipEventDestroy(c.ev_enc[h]);
			if (c.st[h]) (void)hipStreamDestroy(c.st[h]);
		}
	}
	if (b->st) (void)hipStreamDestroy(b->st);
	for (hipStream_t& x : b->cst)
		if (x) (void)hipStreamDestroy(x);
	delete b;
}

int ric_batch_encode(ric_batch* b, const uint8_t* const* pix, int n, int pix_on_device, int q, int trans,
                     uint8_t* const* out, const size_t* cap, size_t* len)
{
	if (!b || !pix || !out || !cap || !len || n < 0 || n > b->slots || q < 0 || q > 31 || trans < 0 || trans > 2)
		return RIC_E_ARG;
	if (n == 0) return RIC_OK;
	if (set_dev(b->device)) return RIC_E_HIP;
	b->set_split(n);
	struct SplitGuard { ric_batch* b; ~SplitGuard() { b->split = false; } } split_guard{b};
	std::vector<const uint8_t*> dpix;
	int rc = stage_pixels(b, 0, n, pix, pix_on_device, dpix);
	if (rc) return rc;
	for (int p = 0; p < b->channels; p++) {
		rc = gpu_encode_plane(b, 0, n, p, dpix.data(), q, trans);
		if (rc) return rc;
		BCHK(hipStreamSynchronize(b->st));
		FirstErr err;
		Latch done;
		done.reset(n);
		for (int i = 0; i < n; i++)
			b->pool->submit([=, &err, &done] {
				err.put(host_encode_plane(b, i, p, q, trans, out[i], cap[i], &len[i]));
				done.done();
			});
		done.wait();
		rc = err.get();
		if (rc == RIC_E_HIP) clear_status(b);
		if (rc) return rc;
	}
	b->prof.harvest();
	return RIC_OK;
}

int ric_batch_decode(ric_batch* b, const uint8_t* const* ric, const size_t* len, int n, uint8_t* const* pix_out,
                     int pix_on_device)
{
	if (!b || !ric || !len || !pix_out || n < 0 || n > b->slots) return RIC_E_ARG;
	if (n == 0) return RIC_OK;
	if (set_dev(b->device)) return RIC_E_HIP;
	std::vector<int> qs(n), ts(n);
	for (int i = 0; i < n; i++) {
		int rc = check_header(b, ric[i], len[i], &qs[i], &ts[i]);
		if (rc) return rc;
		if (ts[i] != ts[0]) return RIC_E_ARG;    // one transform per call (one kernel per level)
	}
	int result = RIC_OK;
	for (int p = 0; p < b->channels; p++) {
		FirstErr err;
		Latch done;
		done.reset(n);
		for (int i = 0; i < n; i++)
			b->pool->submit([=, &err, &done] {
				err.put(host_decode_plane(b, i, p, ric[i], len[i]));
				done.done();
			});
		done.wait();
		const int rc = err.get();
		if (rc && rc != RIC_E_STREAM) return rc;
		if (rc) result = rc;
		int r2 = gpu_decode_plane(b, 0, n, p, qs.data(), ts[0]);
		if (r2) return r2;
		// the next plane's host decode rewrites the mirrors the copy reads
		BCHK(hipStreamSynchronize(b->st));
	}
	int rc = gpu_pix_out(b, 0, n, qs.data(), pix_out, pix_on_device, 0);
	if (rc) return rc;
	BCHK(hipStreamSynchronize(b->st));
	b->prof.harvest();
	return result;
}

int ric_batch_roundtrip(ric_batch* b, const uint8_t* const* pix, int n, int q, int trans, uint8_t* const* out,
                        const size_t* cap, size_t* len, uint8_t* const* pix_out)
{
	if (!b || !pix || !out || !cap || !len || !pix_out || n < 0 || q < 0 || q > 31 || trans < 0 || trans > 2)
		return RIC_E_ARG;
	if (n == 0) return RIC_OK;
	if (!outputs_distinct(out, n)) return set_last_error("ric_batch_roundtrip: out[] buffers must be distinct"), RIC_E_ARG;
	if (set_dev(b->device)) return RIC_E_HIP;
	const int S = b->slots;
	const int G = (n + S - 1) / S;
	b->set_split(std::min(n, 2 * S));                    // (two groups in flight)
	struct SplitGuard { ric_batch* b; ~SplitGuard() { b->split = false; } } split_guard{b};
	if (b->channels != 1) {
		// colour: plane-sequential groups (each plane's host coding needs the
		// previous plane's bands out of the mirror first)
		std::vector<size_t> l2(S);
		for (int g = 0; g < G; g++) {
			const int f0 = g * S, m = std::min(S, n - f0);
			int rc = ric_batch_encode(b, pix + f0, m, 1, q, trans, out + f0, cap + f0, len + f0);
			if (rc) return rc;
			for (int i = 0; i < m; i++) mark_ready(b, f0 + i, len[f0 + i]);
			std::vector<const uint8_t*> rics(out + f0, out + f0 + m);
			// the group's digests are frames f0.. of this call
			unsigned long long* const dg = b->digest;
			const long nd = b->ndigest;
			if (dg) { b->digest = nd > f0 ? dg + f0 : nullptr; b->ndigest = nd > f0 ? nd - f0 : 0; }
			rc = ric_batch_decode(b, rics.data(), len + f0, m, pix_out + f0, 1);
			b->digest = dg;
			b->ndigest = nd;
			if (rc && rc != RIC_E_STREAM) return rc;
		}
		return RIC_OK;
	}
	// gray: group g uses slot set g % 2.  The stream runs enc(0), enc(1),
	// then for each g: dec(g), enc(g + 2) -- enc(g + 2) reuses dec(g)'s set
	// and follows it in stream order.  Host tasks of group g wait for enc(g)'s
	// event, encode their frame, then decode the stream just written into the
	// same slot's mirror; dec(g) starts once all of group g's tasks are done.
	std::vector<hipEvent_t> ev(G, nullptr);
	for (auto& e : ev) BCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
	std::vector<Latch> done(G);
	std::vector<FirstErr> err(G);
	std::vector<int> qs(S, q);
	int rc = RIC_OK;
	auto launch_enc = [&](int g) -> int {
		const int f0 = g * S, m = std::min(S, n - f0), set = g & 1;
		int r = gpu_encode_plane(b, set, m, 0, pix + f0, q, trans);
		if (r) return r;
		BCHK(hipEventRecord(ev[g], b->st));
		done[g].reset(m);
		for (int i = 0; i < m; i++) {
			const int slot = set * S + i, f = f0 + i;
			b->pool->submit([=, &ev, &err, &done] {
				int r1 = bfail(hipEventSynchronize(ev[g]), "hipEventSynchronize") ? RIC_E_HIP : RIC_OK;
				if (!r1) r1 = host_encode_plane(b, slot, 0, q, trans, out[f], cap[f], &len[f]);
				if (!r1) mark_ready(b, f, len[f]);
				if (!r1) r1 = host_decode_plane(b, slot, 0, out[f], len[f]);
				err[g].put(r1);
				done[g].done();
			});
		}
		return RIC_OK;
	};
	int launched = 0;
	std::vector<char> waited(G, 0);
	bool stream_err = false;
	for (; launched < std::min(G, 2); launched++) {
		rc = launch_enc(launched);
		if (rc) break;
	}
	for (int g = 0; g < launched && rc == RIC_OK; g++) {
		done[g].wait();
		waited[g] = 1;
		const int r = err[g].get();
		if (r && r != RIC_E_STREAM) { rc = r; break; }
		stream_err |= r == RIC_E_STREAM;
		const int f0 = g * S, m = std::min(S, n - f0), set = g & 1;
		if (pix_fuse_ok(b, trans, pix_out + f0, m)) {
			const PixFuse pf{pix_out + f0, qs.data(), f0};
			rc = gpu_decode_plane(b, set, m, 0, qs.data(), trans, true, -1, 1, nullptr, nullptr, 0, 0, &pf);
		} else {
			rc = gpu_decode_plane(b, set, m, 0, qs.data(), trans);
			if (!rc) rc = gpu_pix_out(b, set, m, qs.data(), pix_out + f0, 1, f0);
		}
		if (!rc && launched < G) rc = launch_enc(launched++);
	}
	// on an error, the tasks already queued still run: wait for them
	for (int k = 0; k < launched; k++)
		if (!waited[k]) done[k].wait();
	const bool ok = !bfail(hipStreamSynchronize(b->st), "hipStreamSynchronize");
	for (auto& e : ev) (void)hipEventDestroy(e);
	if (rc == RIC_E_HIP) clear_status(b);
	if (rc) return rc;
	if (!ok) return RIC_E_HIP;
	b->prof.harvest();
	return stream_err ? RIC_E_STREAM : RIC_OK;
}

// The whole CompressImage of n gray frames on the GPU: pixel conversion,
// fused forward levels, then the serial coder of every frame's stream on one
// wave each (gcoder.hip k_gc_encode).  pix: device pixels; the .ric file of
// frame i goes to out + i * ostride (device, cap bytes each), its size to
// len[i] (host).  Byte-identical to ric_batch_encode.
int ric_batch_encode_gpu(ric_batch* b, const uint8_t* const* pix, int n, int q, int trans, uint8_t* out, size_t ostride,
                         size_t cap, size_t* len)
{
	const CoderCall coder_call;   // frees from other threads park until this call ends (ric_kernels.h)
	// the coder stores 16-byte chunks (gcoder.hip GEnc::flush_to): a capacity or
	// stride off a multiple of 16 would drop the stream's last bytes unflagged
	if (!b || !pix || !out || !len || n < 0 || n > b->slots || q < 0 || q > 31 || trans < 0 || trans > 2 || cap > ostride ||
	    cap > 0xFFFFFFF0u || (cap & 15) || (ostride & 15))
		return RIC_E_ARG;
	// colour: a frame's three plane pyramids sit in arenas 3i, 3i + 1, 3i + 2
	const int C = b->channels;
	if (C == 3 && 3 * n > b->nslot()) return RIC_E_ARG;
	if (n == 0) return RIC_OK;
	if (set_dev(b->device)) return RIC_E_HIP;
	for (int p = 0; p < C; p++) {
		int rc = C == 1 ? gpu_encode_plane(b, 0, n, 0, pix, q, trans, false)
		                : gpu_encode_plane(b, 0, n, p, pix, q, trans, false, p, 3);
		if (rc) return rc;
	}
	if (!b->d_genc) {
		BCHK(hipMalloc(&b->d_genc, sizeof(GEncArgs)));
		BCHK(hipMalloc(&b->d_res, sizeof(uint32_t) * 2 * b->nslot()));
		BCHK(hipHostMalloc(&b->h_res, sizeof(uint32_t) * 2 * b->nslot(), 0));
	}
	GEncArgs& a = b->genc;
	a.ts = nullptr;
	a.yield = nullptr;
	a.prio = gc_prio();
	a.arena = b->arena(0); a.astride = (size_t)C * b->astride;
	a.pstride = b->astride; a.nplanes = C;
	a.out = out; a.ostride = ostride; a.cap = cap;
	a.res = b->d_res;
	a.status_off = (uint32_t)b->P.status_off;
	a.w = b->w; a.h = b->h; a.q = q; a.trans = trans;
	gc_bands(b->P, a.ll, a.b, a.nb);
	BCHK(hipMemcpyAsync(b->d_genc, &a, sizeof(GEncArgs), hipMemcpyHostToDevice, b->st));
	auto sp = b->prof.begin(B_GENC, n, b->st);
	if (launch_gc_encode(b->d_genc, n, q == 0, b->st)) return bfail(hipGetLastError(), "k_gc_encode") ? RIC_E_HIP : RIC_E_HIP;
	b->prof.end(sp);
	BCHK(hipMemcpyAsync(b->h_res, b->d_res, sizeof(uint32_t) * 2 * n, hipMemcpyDeviceToHost, b->st));
	BCHK(hipStreamSynchronize(b->st));
	b->prof.harvest();
	for (int i = 0; i < n; i++) {
		len[i] = b->h_res[2 * i];
		if (b->h_res[2 * i + 1] == 2) {
			clear_status(b);
			set_last_error("device status word set: a fused level kernel's LDS ring hand-off or the compaction's look-back timed out; output discarded");
			return RIC_E_HIP;
		}
		if (b->h_res[2 * i + 1]) return RIC_E_CAPACITY;
	}
	return RIC_OK;
}

// diagnostics: device buffer for the stream decoder's per-band state dumps
static void* g_gdec_dbg = nullptr;
extern "C" int ric_diag_gdec_dbg(void* dev_buf)
{
	g_gdec_dbg = dev_buf;
	return RIC_OK;
}

// The whole DecompressImage of n gray frames on the GPU: the serial decoder
// of every stream on one wave each (gcoder.hip k_gc_decode) into the bands of
// slot set 0, then the inverse levels and the pixel conversion.  in: the .ric
// files at in + i * istride (device, istride a multiple of 16), len[i] their
// sizes (host); pix_out[i] device pixels.  RIC_E_STREAM when a stream ran past
// its end (the frames are still written), as ric_batch_decode.
int ric_batch_decode_gpu(ric_batch* b, const uint8_t* in, size_t istride, const size_t* len, int n, uint8_t* const* pix_out)
{
	const CoderCall coder_call;   // frees from other threads park until this call ends (ric_kernels.h)
	if (!b || !in || !len || !pix_out || n < 0 || n > b->slots || (istride & 15) || istride > 0xFFFFFFF0u) return RIC_E_ARG;
	const int C = b->channels;
	if (C == 3 && 3 * n > b->nslot()) return RIC_E_ARG;
	if (n == 0) return RIC_OK;
	if (set_dev(b->device)) return RIC_E_HIP;
	if (!b->d_genc) {
		BCHK(hipMalloc(&b->d_genc, sizeof(GEncArgs)));
		BCHK(hipMalloc(&b->d_res, sizeof(uint32_t) * 2 * b->nslot()));
		BCHK(hipHostMalloc(&b->h_res, sizeof(uint32_t) * 2 * b->nslot(), 0));
	}
	if (!b->d_gdec) BCHK(hipMalloc(&b->d_gdec, sizeof(GDecArgs)));
	int q0 = -1, t0 = -1;
	std::vector<int> qs(n);
	for (int i = 0; i < n; i++) {
		if (len[i] > istride || len[i] > 0xFFFFFFF0u) return RIC_E_ARG;
		// the header: the host reads it from device memory (9 bytes per frame)
		uint8_t hd[9];
		BCHK(hipMemcpy(hd, in + (size_t)i * istride, 9, hipMemcpyDeviceToHost));
		int w, h, ch, q, t;
		int rc = ric_read_header(hd, len[i], &w, &h, &ch, &q, &t);
		if (rc) return rc;
		if (w != b->w || h != b->h || ch != C || t > 2) return RIC_E_ARG;
		if (t0 >= 0 && t != t0) return RIC_E_ARG;
		t0 = t; q0 = q; qs[i] = q;
	}
	(void)q0;
	// lengths to the device (the coder reads them per frame)
	for (int i = 0; i < n; i++) b->h_res[2 * i] = (uint32_t)len[i];
	BCHK(hipMemcpyAsync(b->d_res, b->h_res, sizeof(uint32_t) * 2 * n, hipMemcpyHostToDevice, b->st));
	GDecArgs& a = b->gdec;
	a.arena = b->arena(0); a.astride = (size_t)C * b->astride;
	a.pstride = b->astride; a.nplanes = C;
	a.in = in; a.istride = istride;
	a.lens = b->d_res; a.lens_stride = 2;
	a.res = b->d_res + 2 * b->slots;          // after the lengths (2 words per frame)
	a.dbg = (uint32_t*)g_gdec_dbg;
	a.ts = nullptr;
	a.yield = nullptr;
	a.prio = gc_prio();
	a.etab = gc_enum16_table(b->st);
	if (!a.etab) return set_last_error("GPU stream decoder: enumDecode table upload failed"), RIC_E_HIP;
	a.w = b->w; a.h = b->h;
	gc_bands(b->P, a.ll, a.b, a.nb);
	BCHK(hipMemcpyAsync(b->d_gdec, &a, sizeof(GDecArgs), hipMemcpyHostToDevice, b->st));
	auto sp = b->prof.begin(B_GDEC, n, b->st);
	if (launch_gc_decode(b->d_gdec, n, b->st)) return bfail(hipGetLastError(), "k_gc_decode") ? RIC_E_HIP : RIC_E_HIP;
	b->prof.end(sp);
	int rc = RIC_OK;
	for (int p = 0; p < C && !rc; p++)
		rc = C == 1 ? gpu_decode_plane(b, 0, n, 0, qs.data(), t0, false) : gpu_decode_plane(b, 0, n, p, qs.data(), t0, false, p, 3);
	if (rc) return rc;
	rc = gpu_pix_out(b, 0, n, qs.data(), pix_out, 1, 0);
	if (rc) return rc;
	BCHK(hipMemcpyAsync(b->h_res + 2 * b->slots, b->d_res + 2 * b->slots, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, b->st));
	BCHK(hipStreamSynchronize(b->st));
	b->prof.harvest();
	int result = RIC_OK;
	for (int i = 0; i < n; i++) {
		const uint32_t r = b->h_res[2 * b->slots + i];
		if ((r & 15) == 3) {
			set_last_error("GPU stream decoder: staging overrun (pathological stream) at byte " + std::to_string(r >> 4));
			return RIC_E_CAPACITY;
		}
		if (r == 1) result = RIC_E_STREAM;
	}
	return result;
}

// ------------------------------------------------------------ hybrid
// Round trips with the serial coder on the GPU (gcoder.hip: one wave per
// frame's stream).  Frames go to the GPU coder in launches of `pool_frames`:
// their forward levels run in groups of `slots` on the batch stream and each
// group's bands + records are copied into one half of the pool; then, on that
// half's coder stream, k_gc_encode codes them all and (gpu_decode) k_gc_decode
// decodes the streams back into the pool, whose bands go through the inverse
// levels in groups.  Without gpu_decode the host pool decodes the streams;
// gpu_decode 2 decides per launch (host pool first, the GPU for the excess).
// A coder launch takes seconds (a wave codes one whole stream), so two
// launches are in flight (the two halves) and the host threads meanwhile do
// whole round trips of the first n_host frames.
int ric_batch_set_digests(ric_batch* b, unsigned long long* dev_digests, long n)
{
	if (!b || n < 0 || (n > 0 && !dev_digests)) return RIC_E_ARG;
	b->digest = n ? dev_digests : nullptr;
	b->ndigest = n;
	return RIC_OK;
}

int ric_batch_set_ready(ric_batch* b, uint32_t* host_words, long n)
{
	if (!b || n < 0 || (n > 0 && !host_words)) return RIC_E_ARG;
	b->ready = n ? host_words : nullptr;
	b->nready = n;
	return RIC_OK;
}

int ric_batch_hybrid_config(ric_batch* b, int pool_frames, size_t stream_cap)
{
	return ric_batch_hybrid_config_ex(b, pool_frames, stream_cap, -1);
}

int ric_batch_hybrid_config_ex(ric_batch* b, int pool_frames, size_t stream_cap, long value_cap)
{
	if (!b || pool_frames < 1 || pool_frames > 65536 || stream_cap < 64 || (stream_cap & 15) || stream_cap > 0xFFFFFFF0u)
		return RIC_E_ARG;
	if (set_dev(b->device)) return RIC_E_HIP;
	auto& c = b->cp;
	for (int h = 0; h < 2; h++)
		if (c.st[h]) BCHK(hipStreamSynchronize(c.st[h]));
	if (c.d_ab) { BCHK(dev_free(c.d_ab)); c.d_ab = nullptr; }
	if (c.d_out) { BCHK(dev_free(c.d_out)); c.d_out = nullptr; }
	if (c.h_res) { BCHK(pinned_free(c.h_res)); c.h_res = c.d_res = nullptr; }
	if (c.d_ts) { BCHK(dev_free(c.d_ts)); c.d_ts = nullptr; }
	if (c.h_post) { BCHK(pinned_free(c.h_post)); c.h_post = c.d_post = nullptr; }
	if (c.d_pcmp) { BCHK(dev_free(c.d_pcmp)); c.d_pcmp = nullptr; }
	if (c.d_pcnt) { BCHK(dev_free(c.d_pcnt)); c.d_pcnt = nullptr; }
	if (c.d_ptotal) { BCHK(dev_free(c.d_ptotal)); c.d_ptotal = nullptr; }
	if (!c.d_yield) {
		BCHK(hipMalloc(&c.d_yield, 256));
		BCHK(hipMemset(c.d_yield, 0, 256));
	}
	c.n = pool_frames;
	const Pyramid& P = b->P;
	// the compacted pool: level 0 16-bit (the 9/7 ric path), a value capacity
	// per plane (default 9 of a block's 16 coefficients) below the dense bands
	c.dl = dcmp_layout(P);
	size_t l0 = 0;
	for (int k = 0; k < 3; k++) l0 += (size_t)P.L[0].b[k].dx * P.L[0].b[k].dy;
	const long vdef = (long)(l0 * 9 / 16);
	const long vc = value_cap < 0 ? vdef : std::min(value_cap, (long)l0);
	c.vcap = 0; c.lo = 0; c.cmp_cap = 0; c.ashift = 0;
	if (vc > 0 && c.dl.ok && P.nlev >= 2) {
		c.vcap = (uint32_t)vc;
		c.lo = P.L[1].b[BD].off;                           // level 0's bands: [0, lo)
		c.cmp_cap = (c.dl.vals_off + 2 * (size_t)c.vcap + 255) / 256 * 256;
		if (c.cmp_cap == c.lo) c.cmp_cap += 256;           // (GEncArgs::cmp_rel 0 means dense)
		c.ashift = (long long)c.cmp_cap - (long long)c.lo;
	}
	// colour: a frame's Y, Co, Cg plane pyramids side by side (the coder codes
	// them into one stream on one wave, ric.cpp:157-176)
	c.abstride = ((c.vcap ? c.cmp_cap + (P.b_end - c.lo) : P.b_end) + 65535) / 65536 * 65536;
	c.fstride = (size_t)b->channels * c.abstride;
	c.ocap = stream_cap;
	// out of memory: nothing stays allocated and the error is not left
	// pending (a caller may retry with a smaller pool)
	if (hipMalloc(&c.d_ab, 2 * c.fstride * c.n) != hipSuccess || hipMalloc(&c.d_out, 2 * c.ocap * c.n) != hipSuccess) {
		const hipError_t e = hipGetLastError();
		if (c.d_ab) (void)dev_free(c.d_ab);
		c.d_ab = nullptr;
		c.d_out = nullptr;
		set_last_error(std::string("ric_batch_hybrid_config: pool of ") + std::to_string(pool_frames) +
		               " frames: " + hipGetErrorString(e));
		return e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation ? RIC_E_CAPACITY : RIC_E_HIP;
	}
	// the rest; on any failure the pool is released again (a half-configured
	// pool would let ric_batch_roundtrip_hybrid launch coder kernels that post
	// through null result pointers)
	auto rest = [&]() -> int {
		// the coder kernels write their result words straight into host memory: a
		// copy queued behind a coder kernel on its stream held up the batch
		// stream's own copies until the kernel ended (seconds)
		BCHK(hipHostMalloc(&c.h_res, sizeof(uint32_t) * 6 * c.n, hipHostMallocMapped | hipHostMallocCoherent));
		BCHK(hipHostGetDevicePointer((void**)&c.d_res, c.h_res, 0));
		// posted words: the encoder's two per frame of both halves, then the
		// round trip's decode word per frame of both
		BCHK(hipHostMalloc(&c.h_post, sizeof(uint32_t) * 6 * c.n, hipHostMallocCoherent | hipHostMallocMapped));
		BCHK(hipHostGetDevicePointer((void**)&c.d_post, c.h_post, 0));
		memset(c.h_post, 0, sizeof(uint32_t) * 6 * c.n);
		if (!c.d_args) BCHK(hipMalloc(&c.d_args, 3 * sizeof(GEncArgs)));   // the halves, then both as one launch
		if (!c.d_dargs) BCHK(hipMalloc(&c.d_dargs, 3 * sizeof(GDecArgs)));
		if (c.vcap) {
			// the forward compaction's argument blocks, one per (half, group, plane)
			c.pcmp_groups = (c.n + b->slots - 1) / b->slots;
			BCHK(hipMalloc(&c.d_pcmp, sizeof(CmpArgs) * 2 * (size_t)c.pcmp_groups * b->channels));
			int nch = 0;
			for (int k = 0; k < 3; k++) nch += c.dl.nch[k];
			c.pcnt_stride = (size_t)(nch + 63) / 64 * 64;
			BCHK(hipMalloc(&c.d_pcnt, sizeof(uint32_t) * c.pcnt_stride * b->slots));
			BCHK(hipMemset(c.d_pcnt, 0, sizeof(uint32_t) * c.pcnt_stride * b->slots));
			BCHK(hipMalloc(&c.d_ptotal, sizeof(uint32_t) * b->slots));
			std::vector<CmpArgs> ca(2 * (size_t)c.pcmp_groups * b->channels);
			for (int h = 0; h < 2; h++)
				for (int g = 0; g < c.pcmp_groups; g++)
					for (int p = 0; p < b->channels; p++) {
						CmpArgs& a = ca[((size_t)h * c.pcmp_groups + g) * b->channels + p];
						memset(&a, 0, sizeof a);
						char* region = c.d_ab + ((size_t)h * c.n + (size_t)g * b->slots) * c.fstride + (size_t)p * c.abstride;
						a.arena = region + c.ashift; a.astride = c.fstride;      // the records (pool region B)
						a.bsrc = b->arena(0); a.bstride = b->astride;             // level 0's dense bands (scratch)
						a.out = region + c.dl.vals_off; a.ostride = c.fstride;
						a.cnt = c.d_pcnt; a.cstride = c.pcnt_stride;
						a.total = c.d_ptotal;
						a.vcap = c.vcap;
						a.status = region + c.ashift + P.status_off; a.sstride = c.fstride;
						int ch = 0;
						for (int k = 0; k < 3; k++) {                             // level 0, coding order V, H, D
							const Band& B = P.L[0].b[c.dl.band[k]];
							CmpBand& d = a.band[k];
							d.off = (uint32_t)B.off; d.rec_off = (uint32_t)P.rec_off[0][c.dl.band[k]];
							d.dx = B.dx; d.dy = B.dy; d.pitch = B.pitch;
							d.nblk = B.bw() * B.bh();
							d.chunk0 = ch;
							ch += (d.nblk + 63) / 64;
						}
						a.nb = 3; a.nchunk = ch;
					}
			BCHK(hipMemcpy(c.d_pcmp, ca.data(), sizeof(CmpArgs) * ca.size(), hipMemcpyHostToDevice));
		}
		for (int h = 0; h < 2; h++) {
			if (!c.st[h]) BCHK(hipStreamCreateWithFlags(&c.st[h], hipStreamNonBlocking));
			if (!c.ev_fwd[h]) BCHK(hipEventCreateWithFlags(&c.ev_fwd[h], hipEventDisableTiming));
			if (!c.ev_done[h]) BCHK(hipEventCreateWithFlags(&c.ev_done[h], hipEventDisableTiming));
			if (!c.ev_enc[h]) BCHK(hipEventCreateWithFlags(&c.ev_enc[h], hipEventDisableTiming));
		}
		return RIC_OK;
	};
	const int rc = rest();
	if (rc) {
		(void)dev_free(c.d_ab);
		(void)dev_free(c.d_out);
		c.d_ab = nullptr;
		c.d_out = nullptr;
		if (c.h_res) (void)pinned_free(c.h_res);
		if (c.h_post) (void)pinned_free(c.h_post);
		if (c.d_pcmp) (void)dev_free(c.d_pcmp);
		if (c.d_pcnt) (void)dev_free(c.d_pcnt);
		if (c.d_ptotal) (void)dev_free(c.d_ptotal);
		c.h_res = c.d_res = c.h_post = c.d_post = nullptr;
		c.d_pcmp = nullptr; c.d_pcnt = c.d_ptotal = nullptr;
		c.n = 0;
	}
	return rc;
}

namespace {

// one group of at most `slots` frames through a slot set
struct HGroup {
	int f0 = 0, m = 0;
	bool gpu = false;         // stream coded on the GPU (tasks: decode only)
	int half = 0;             // its streams' half of cp.d_out
	int k0 = 0;               // index of f0 in that half
};

}  // namespace

int ric_batch_roundtrip_hybrid(ric_batch* b, const uint8_t* const* pix, int n, int n_host, int gpu_decode, int q,
                               int trans, uint8_t* const* out, const size_t* cap, size_t* len, uint8_t* const* pix_out)
{
	const CoderCall coder_call;   // frees from other threads park until this call ends (ric_kernels.h)
	if (!b || !pix || !out || !cap || !len || !pix_out || n < 0 || n_host < 0 || n_host > n || q < 0 || q > 31 ||
	    trans < 0 || trans > 2)
		return RIC_E_ARG;
	if (n_host < n && (!b->cp.d_ab || !b->cp.h_res || !b->cp.d_post)) return RIC_E_ARG;    // ric_batch_hybrid_config first
	// colour frames round-tripped or decoded on the host keep each plane's
	// bands in a slot of its own: a host group is slots / 3 frames
	const int C = b->channels;
	// (a compacted pool can leave any frame to a host round trip: over its value capacity)
	if (C == 3 && b->slots < 3 && (n_host > 0 || gpu_decode != 1 || b->cp.vcap)) return RIC_E_ARG;
	if (n == 0) return RIC_OK;
	if (!outputs_distinct(out, n))
		return set_last_error("ric_batch_roundtrip_hybrid: out[] buffers must be distinct"), RIC_E_ARG;
	if (set_dev(b->device)) return RIC_E_HIP;
	// the level kernels run beside the stream coder's waves (the step's front,
	// before the coder launch, switches to the alone forms)
	struct FormGuard {
		ric_batch* b;
		~FormGuard() { b->alone(true); b->cmp_dma = false; }
	} form_guard{b};
	b->alone(false);
	b->cmp_dma = true;
	b->split = false;                                      // every host thread codes frames of its own here
	auto& c = b->cp;
	Pyramid& P = b->P;
	const int S = b->slots;
	const int SG = S / C;                                  // frames per host group (slots per frame: C)
	// word offsets into d_res / h_res: the encoder's 2 words per frame of both
	// halves, then the decoder's word per frame of both (so the two halves can
	// also run as one launch over 2 n frames)
	auto res_enc = [&](int h) { return (size_t)h * 2 * c.n; };
	auto res_dec = [&](int h) { return (size_t)4 * c.n + (size_t)h * c.n; };
	// RIC_GC_YIELD=0: the coder waves do not pause for the host frames' level
	// kernels (coder_yield, gcoder.hip)
	static const bool yield_on = [] { const char* e = getenv("RIC_GC_YIELD"); return !e || atoi(e) != 0; }();
	if (c.d_yield) BCHK(hipMemsetAsync(c.d_yield, 0, 4, b->st));
	uint32_t* yflag = yield_on ? c.d_yield : nullptr;   // host frames' level kernels raise it
	// RIC_GC_TSTAMP=1: every coder wave's start and end, summarised per launch
	// on stderr at its harvest (when the waves end: the launch's tail)
	static const bool tstamp = [] { const char* e = getenv("RIC_GC_TSTAMP"); return e && atoi(e) > 0; }();
	if (tstamp && c.d_ab && !c.d_ts) BCHK(hipMalloc(&c.d_ts, sizeof(uint64_t) * 16 * (size_t)c.n));
	if (c.d_ab) {
		for (int h = 0; h < 2; h++) {
			GEncArgs& a = c.args[h];
			a.ts = tstamp ? c.d_ts + (size_t)h * 4 * c.n : nullptr;
			a.prio = gc_prio();
			a.yield = yield_on ? c.d_yield : nullptr;
			a.arena = c.d_ab + (size_t)h * c.n * c.fstride + c.ashift; a.astride = c.fstride;
			a.pstride = c.abstride; a.nplanes = C;
			a.out = c.d_out + (size_t)h * c.n * c.ocap; a.ostride = c.ocap; a.cap = c.ocap;
			a.res = c.d_res + res_enc(h);
			a.status_off = (uint32_t)P.status_off;
			a.w = b->w; a.h = b->h; a.q = q; a.trans = trans;
			gc_bands(P, a.ll, a.b, a.nb);
			a.cmp_rel = c.vcap ? -c.ashift : 0;
			a.cvals_off = (uint32_t)c.dl.vals_off; a.cvcap = c.vcap;
			if (c.vcap) gc_bands_compact(a.b, a.nb, c.dl.mask_off, c.dl.coff_off);
			GDecArgs& d = c.dargs[h];
			d.arena = (char*)a.arena; d.astride = a.astride;
			d.pstride = a.pstride; d.nplanes = C;
			d.in = a.out; d.istride = c.ocap;
			d.lens = a.res; d.lens_stride = 2;
			d.res = c.d_res + res_dec(h);
			d.dbg = nullptr;
			d.prio = gc_prio();
			d.yield = yield_on ? c.d_yield : nullptr;
			d.etab = gc_enum16_table(b->st);
			if (!d.etab) return set_last_error("GPU stream decoder: enumDecode table upload failed"), RIC_E_HIP;
			d.ts = tstamp ? c.d_ts + (size_t)8 * c.n + (size_t)h * 4 * c.n : nullptr;
			d.w = b->w; d.h = b->h;
			gc_bands(P, d.ll, d.b, d.nb);
			d.cmp_rel = a.cmp_rel; d.cvals_off = a.cvals_off; d.cvcap = a.cvcap;
			if (c.vcap) gc_bands_compact(d.b, d.nb, c.dl.mask_off, c.dl.coff_off);
		}
		// entry 2: both halves as one launch (frames 0 .. 2 n - 1 of the pool;
		// the arenas, streams and result words of the halves are contiguous)
		GEncArgs ea[3] = {c.args[0], c.args[1], c.args[0]};
		GDecArgs da[3] = {c.dargs[0], c.dargs[1], c.dargs[0]};
		BCHK(hipMemcpy(c.d_args, ea, sizeof(ea), hipMemcpyHostToDevice));
		BCHK(hipMemcpy(c.d_dargs, da, sizeof(da), hipMemcpyHostToDevice));
	}
	// RIC_HYBRID_TRACE=1: the step's timeline on stderr (kicks, encode ends,
	// harvests, host groups, the end), ms from entry
	static const int trace = [] { const char* e = getenv("RIC_HYBRID_TRACE"); return e ? atoi(e) : 0; }();   // 2: every group
	const double t_entry = now_ms();
	auto tr = [&](const char* what, int j) {
		if (trace) fprintf(stderr, "[hybrid] %9.1f ms %s %d\n", now_ms() - t_entry, what, j);
	};
	int host_groups_done = 0;
	b->hyb_host_ms = b->hyb_gpu_ms = 0;
	// the GPU side's end: the coder frames' last harvest kernel, timed on the
	// batch stream from the call's start (the host side's end is host time)
	struct EvPair {
		hipEvent_t a = nullptr, b = nullptr;
		~EvPair() { if (a) (void)hipEventDestroy(a); if (b) (void)hipEventDestroy(b); }
	} evt;
	hipEvent_t& ev_t0 = evt.a;
	hipEvent_t& ev_t1 = evt.b;
	bool t1_set = false;
	BCHK(hipEventCreate(&ev_t0));
	BCHK(hipEventCreate(&ev_t1));
	BCHK(hipEventRecord(ev_t0, b->st));
	b->hyb_fallback = 0;
	std::deque<HGroup> ready_host, ready_dec;
	for (int f0 = 0; f0 < n_host; f0 += SG) ready_host.push_back({f0, std::min(SG, n_host - f0), false, 0, 0});
	const int ng = n - n_host;
	const int nbatch = ng > 0 ? (ng + c.n - 1) / c.n : 0;
	int kicked = 0, finished = 0;
	std::vector<Latch> copied(nbatch > 0 ? nbatch : 1);   // host decode: a batch's streams are out of d_out
	// per batch: decoded on the GPU (1) or by the host pool (0).  gpu_decode 2
	// decides at each launch: the host pool takes a batch when its own backlog
	// would run dry before the batch's encode ends, the GPU decodes the rest.
	std::vector<char> bgpu(nbatch > 0 ? nbatch : 1, 0);
	std::vector<double> t_kick(nbatch > 0 ? nbatch : 1, 0.0);
	const double px = (double)b->w * b->h;
	double enc_ms_est = px * 1.3e-4;                      // a stream coder launch (C3: ~4.3 s), refined as launches end
	std::atomic<long> dec_us{0}, dec_n{0};                // host decode time per frame, measured
	auto host_dec_ms = [&]() { const long k = dec_n.load(); return k > 0 ? dec_us.load() * 1e-3 / k : px * 4e-6; };
	int rc = RIC_OK;
	bool stream_err = false;
	std::vector<int> qs(S, q);
	auto batch_f0 = [&](int j) { return n_host + j * c.n; };
	auto batch_m = [&](int j) { return std::min(c.n, n - batch_f0(j)); };
	auto abslot = [&](int h, int k) { return c.d_ab + ((size_t)h * c.n + k) * c.fstride; };   // frame k of half h, plane 0
	// its kernels' arena base (a compacted pool: the offsets >= lo after the compact block)
	auto kbase = [&](int h, int k) { return abslot(h, k) + c.ashift; };
	int pcmp_nch = 0;
	for (int k = 0; k < 3; k++) pcmp_nch += c.dl.nch[k];
	int n_fallback = 0;                                    // frames over the compacted pool's capacity: coded on the host
	// RIC_FWD_AHEAD=0: each batch's coder launch starts after its own forward
	// levels (the second batch's then run beside the first batch's coder waves)
	static const bool fwd_ahead = [] { const char* e = getenv("RIC_FWD_AHEAD"); return !e || atoi(e) != 0; }();
	// RIC_GC_MERGE=0: the two halves' coder kernels as two launches side by side
	static const bool merge = [] { const char* e = getenv("RIC_GC_MERGE"); return !e || atoi(e) != 0; }();
	// RIC_GC_FUSE=0: the merged launch as an encode kernel, then a decode kernel
	// (1: k_gc_roundtrip, each wave goes on to decode its stream as soon as it
	// is encoded)
	static const bool fuse = [] { const char* e = getenv("RIC_GC_FUSE"); return !e || atoi(e) != 0; }();
	// each coder launch's tag (launch_gc_encode): its posted result words carry it
	std::vector<uint32_t> tagj(nbatch > 0 ? nbatch : 1, 0);
	bool fused = false;                                    // batches 0 and 1 run as one k_gc_roundtrip
	auto next_tag = [&]() {
		c.epoch = (c.epoch + 1) & 0xFFFFFu;
		if (!c.epoch) c.epoch = 1;
		return c.epoch;
	};
	// batch j's coder launches are done: (host decode) its decode groups become
	// ready; (gpu_decode) its frames go through the inverse levels right away
	// A GPU-decoded batch's .ric files leave for the host as soon as its encode
	// is done, from a thread of their own (the host buffers are pageable: the
	// copies block their caller), while the batch decodes on the GPU.
	std::vector<std::thread> copier(nbatch > 0 ? nbatch : 1);
	std::vector<int> copy_rc(nbatch > 0 ? nbatch : 1, RIC_OK);
	int enc_seen = 0;                                      // batches whose encode event was handled
	auto copy_out = [&](int j) {
		if (copier[j].joinable()) return;                          // (fused: started at the kick)
		const int f0 = batch_f0(j), m = batch_m(j), h = j & 1;
		// the launch posts each stream's result once the stream is in HBM, tagged
		// with the launch's tag (k_gc_encode / k_gc_roundtrip): a word is this
		// launch's only if it carries the tag, whatever an earlier launch left
		const uint32_t* po = c.h_post + res_enc(h);
		const uint32_t want = 0x100u | tagj[j] << 12;
		hipEvent_t done = c.ev_enc[h];                         // the encoding kernel's end
		copier[j] = std::thread([=, &copy_rc, &c] {
			int r = set_dev(b->device);
			for (int k = 0; k < m && !r; k++) {
				uint32_t st_k;
				// the kernel's end (normal or not) stops the wait
				while (((st_k = __atomic_load_n(po + 2 * k + 1, __ATOMIC_ACQUIRE)) & ~0xFFu) != want) {
					if (hipEventQuery(done) != hipErrorNotReady) {
						st_k = __atomic_load_n(po + 2 * k + 1, __ATOMIC_ACQUIRE);
						break;
					}
					std::this_thread::sleep_for(std::chrono::microseconds(500));
				}
				if ((st_k & ~0xFFu) != want) break;                  // harvest reports it
				if ((st_k & 0xFFu) == 4) continue;                    // left to the host (harvest)
				const uint32_t len_k = __atomic_load_n(po + 2 * k, __ATOMIC_RELAXED);
				if ((st_k & 0xFFu) || len_k > cap[f0 + k]) break;   // harvest reports it
				if (bfail(d2h(b, j, out[f0 + k], c.d_out + ((size_t)h * c.n + k) * c.ocap, len_k), "hipMemcpy stream"))
					r = RIC_E_HIP;
				else
					mark_ready(b, f0 + k, len_k);
			}
			copy_rc[j] = r;
		});
	};
	// batch j: forward levels in groups of S (slot set 0; stream order keeps it
	// clear of the groups using the arenas), bands + records into pool half
	// j & 1, then the coder launches on that half's stream
	auto kick_fwd = [&](int j) -> int {
		const int f0 = batch_f0(j), m = batch_m(j), h = j & 1;
		for (int g0 = 0; g0 < m; g0 += S) {
			const int gm = std::min(S, m - g0);
			for (int p = 0; p < C; p++) {                   // (p 0 converts every plane's pixels)
				// the bands + records straight into the pool (the arenas keep the scratch)
				int r = gpu_encode_plane(b, 0, gm, p, pix + f0 + g0, q, trans, false, -1, 1, nullptr,
				                         kbase(h, g0) + (size_t)p * c.abstride, c.fstride, c.lo);
				if (r) return r;
				// a compacted pool: level 0's values (from the arenas) into each frame's compact block
				if (c.vcap) {
					auto sc = b->prof.begin(B_CMP, gm, b->st);
					if (launch_compact(c.d_pcmp + ((size_t)h * c.pcmp_groups + g0 / S) * C + p, pcmp_nch, gm, b->st))
						return bfail(hipGetLastError(), "pool compaction") ? RIC_E_HIP : RIC_E_HIP;
					b->prof.end(sc);
				}
			}
		}
		BCHK(hipEventRecord(c.ev_fwd[h], b->st));
		return RIC_OK;
	};
	// wait_other: the launch also waits for the other half's forward levels
	// (the first two batches: every forward level of both, and of the first
	// host groups, runs before any coder wave takes the CUs)
	auto kick_coder = [&](int j, bool wait_other) -> int {
		const int m = batch_m(j), h = j & 1;
		BCHK(hipStreamWaitEvent(c.st[h], c.ev_fwd[h], 0));
		if (wait_other) BCHK(hipStreamWaitEvent(c.st[h], c.ev_fwd[h ^ 1], 0));
		tagj[j] = next_tag();
		auto sp = b->prof.begin(B_GENC, m, c.st[h]);
		if (launch_gc_encode(c.d_args + h, m, q == 0, c.st[h], c.d_post + res_enc(h), tagj[j]))
			return bfail(hipGetLastError(), "k_gc_encode") ? RIC_E_HIP : RIC_E_HIP;
		b->prof.end(sp);
		BCHK(hipEventRecord(c.ev_enc[h], c.st[h]));
		if (gpu_decode == 1) bgpu[j] = 1;
		else if (gpu_decode == 2) {
			// the host pool's backlog (frames to decode, round trips queued), in seconds of its threads
			long dec_frames = 0;
			for (const auto& g : ready_dec) dec_frames += g.m;
			for (int k = finished; k < j; k++)
				if (!bgpu[k]) dec_frames += batch_m(k);
			long rt_frames = 0;
			for (const auto& g : ready_host) rt_frames += g.m;
			const double thr = (double)b->pool->size();
			const double backlog_ms = (dec_frames * host_dec_ms() + rt_frames * 2.0 * host_dec_ms()) / thr;
			bgpu[j] = backlog_ms > enc_ms_est ? 1 : 0;
		}
		t_kick[j] = now_ms();
		tr("kick", j);
		if (bgpu[j]) {
			auto sd = b->prof.begin(B_GDEC, m, c.st[h]);
			if (launch_gc_decode(c.d_dargs + h, m, c.st[h]))
				return bfail(hipGetLastError(), "k_gc_decode") ? RIC_E_HIP : RIC_E_HIP;
			b->prof.end(sd);
		}
		BCHK(hipEventRecord(c.ev_done[h], c.st[h]));
		copied[j].reset(bgpu[j] ? 0 : m);
		return RIC_OK;
	};
	// batches 0 and 1 (both GPU-decoded) as one launch of both pool halves:
	// dispatched at once onto an idle chip, the waves spread evenly over the
	// SIMDs (two launches side by side each spread on their own, so SIMDs
	// held two to four coder waves, and the four-wave ones set each phase's end)
	auto kick_both = [&]() -> int {
		const int m = batch_m(0) + batch_m(1);
		BCHK(hipStreamWaitEvent(c.st[0], c.ev_fwd[0], 0));
		BCHK(hipStreamWaitEvent(c.st[0], c.ev_fwd[1], 0));
		tagj[0] = tagj[1] = next_tag();
		if (fuse && q != 0) {
			// one kernel: each wave encodes its frame, posts the stream (the
			// copiers take it from there at once) and decodes it
			fused = true;
			auto sp = b->prof.begin(B_GRT, m, c.st[0]);
			if (launch_gc_roundtrip(c.d_args + 2, c.d_dargs + 2, c.d_post, c.d_post + 4 * (size_t)c.n, tagj[0], m, c.st[0]))
				return bfail(hipGetLastError(), "k_gc_roundtrip") ? RIC_E_HIP : RIC_E_HIP;
			b->prof.end(sp);
			for (int j = 0; j < 2; j++) {
				BCHK(hipEventRecord(c.ev_enc[j], c.st[0]));
				BCHK(hipEventRecord(c.ev_done[j], c.st[0]));
				bgpu[j] = 1;
				t_kick[j] = now_ms();
				tr("kick", j);
				copied[j].reset(0);
				copy_out(j);
			}
			return RIC_OK;
		}
		auto sp = b->prof.begin(B_GENC, m, c.st[0]);
		if (launch_gc_encode(c.d_args + 2, m, q == 0, c.st[0], c.d_post, tagj[0]))
			return bfail(hipGetLastError(), "k_gc_encode") ? RIC_E_HIP : RIC_E_HIP;
		b->prof.end(sp);
		BCHK(hipEventRecord(c.ev_enc[0], c.st[0]));
		BCHK(hipEventRecord(c.ev_enc[1], c.st[0]));
		for (int j = 0; j < 2; j++) {
			bgpu[j] = 1;
			t_kick[j] = now_ms();
			tr("kick", j);
		}
		auto sd = b->prof.begin(B_GDEC, m, c.st[0]);
		if (launch_gc_decode(c.d_dargs + 2, m, c.st[0])) return bfail(hipGetLastError(), "k_gc_decode") ? RIC_E_HIP : RIC_E_HIP;
		b->prof.end(sd);
		BCHK(hipEventRecord(c.ev_done[0], c.st[0]));
		BCHK(hipEventRecord(c.ev_done[1], c.st[0]));
		copied[0].reset(0);
		copied[1].reset(0);
		return RIC_OK;
	};
	auto kick = [&](int j) -> int {
		const int r = kick_fwd(j);
		return r ? r : kick_coder(j, false);
	};
	// The inverse levels + pixel output of frames g0 .. g0 + S - 1 of GPU-decoded
	// batch j (the inverse reads the decoded bands in the pool)
	std::vector<std::vector<char>> hv_done(nbatch > 0 ? nbatch : 1);
	for (int j = 0; j < nbatch; j++) hv_done[j].assign((batch_m(j) + S - 1) / S, 0);
	int hv_early = 0;
	auto harvest_group = [&](int j, int g0) -> int {
		const int f0 = batch_f0(j), m = batch_m(j), h = j & 1;
		const int gm = std::min(S, m - g0);
		for (int p = 0; p < C; p++) {
			if (c.vcap) {
				// level 0 from the compact blocks into the arenas' dense bands
				DcmpArgs x;
				x.arena = b->arena(0); x.astride = b->astride;
				x.in = abslot(h, g0) + (size_t)p * c.abstride; x.istride = c.fstride;
				int ch = 0;
				for (int k = 0; k < 3; k++) {
					const Band& B = P.L[0].b[c.dl.band[k]];
					x.off[k] = (uint32_t)B.off; x.dx[k] = B.dx; x.dy[k] = B.dy; x.pitch[k] = B.pitch;
					x.mask_off[k] = (uint32_t)c.dl.mask_off[k]; x.coff_off[k] = (uint32_t)c.dl.coff_off[k];
					x.nblk[k] = c.dl.nblk[k];
					x.chunk0[k] = ch;
					ch += c.dl.nch[k];
				}
				x.chunk0[3] = ch;
				x.vals_off = (uint32_t)c.dl.vals_off;
				x.vcap = c.vcap;
				auto sx = b->prof.begin(B_DEXP, gm, b->st);
				if (launch_dcmp_expand(x, gm, b->st)) return bfail(hipGetLastError(), "k_dcmp_expand") ? RIC_E_HIP : RIC_E_HIP;
				b->prof.end(sx);
			}
			const bool fuse = pix_fuse_ok(b, trans, pix_out + f0 + g0, gm);
			const PixFuse pf{pix_out + f0 + g0, qs.data(), f0 + g0};
			int r = gpu_decode_plane(b, 0, gm, p, qs.data(), trans, false, -1, 1, nullptr,
			                         kbase(h, g0) + (size_t)p * c.abstride, c.fstride, c.lo, fuse ? &pf : nullptr);
			if (r) return r;
			if (fuse) {
				hv_done[j][g0 / S] = 1;
				return RIC_OK;
			}
		}
		const int r = gpu_pix_out(b, 0, gm, qs.data(), pix_out + f0 + g0, 1, f0 + g0);
		if (r == RIC_OK) hv_done[j][g0 / S] = 1;          // a failed group is not taken for harvested
		return r;
	};
	// While the fused launch runs: a group whose frames have all posted their
	// decode (k_gc_roundtrip's posted_dec words, this launch's tag, no failure)
	// is harvested at once, beside the waves still decoding, instead of after
	// the launch (RIC_EARLY_HARVEST=0: after the launch only)
	static const bool early_on = [] { const char* e = getenv("RIC_EARLY_HARVEST"); return !e || atoi(e) != 0; }();
	auto early_harvest = [&]() -> int {
		if (!fused || !early_on) return RIC_OK;
		const uint32_t want = 0x100u | tagj[0] << 12;
		const uint32_t* pd = c.h_post + 4 * (size_t)c.n;       // frames of both halves, in pool order
		for (int j = finished; j < 2 && j < nbatch; j++) {
			const int m = batch_m(j);
			for (int g0 = 0; g0 < m; g0 += S) {
				if (hv_done[j][g0 / S]) continue;
				const int gm = std::min(S, m - g0);
				bool ok = true;
				for (int k = 0; k < gm && ok; k++) {
					const uint32_t w = __atomic_load_n(pd + (size_t)j * c.n + g0 + k, __ATOMIC_ACQUIRE);
					ok = (w & ~0xFFu) == want && !(w & 0x80u) && (w & 15u) != 3u;
				}
				if (!ok) continue;
				const int r = harvest_group(j, g0);
				if (r) return r;
				hv_early++;
			}
		}
		return RIC_OK;
	};
	auto harvest = [&](int j) -> int {
		const int f0 = batch_f0(j), m = batch_m(j), h = j & 1;
		const uint32_t* re = c.h_res + res_enc(h);
		const uint32_t* rd = c.h_res + res_dec(h);
		if (copier[j].joinable()) copier[j].join();
		if (copy_rc[j]) return copy_rc[j];
		if (tstamp) {
			// per kernel: waves' end times from the kernel's first start, ms (p0 p10 p50 p90 p100),
			// the mean wave duration, and the waves per SIMD they ran beside (this launch's own)
			std::vector<uint64_t> t(8 * (size_t)m);
			BCHK(d2h(b, j, t.data(), c.d_ts + (size_t)h * 4 * c.n, sizeof(uint64_t) * 4 * m));
			BCHK(d2h(b, j, t.data() + 4 * m, c.d_ts + (size_t)8 * c.n + (size_t)h * 4 * c.n, sizeof(uint64_t) * 4 * m));
			static std::mutex ts_mu;
			std::lock_guard<std::mutex> g(ts_mu);
			// RIC_GC_TSTAMP_FILE: every wave as a line (call, batch, kernel, frame, start, end, HW_ID, XCC_ID)
			static FILE* tsf = [] { const char* e = getenv("RIC_GC_TSTAMP_FILE"); return e ? fopen(e, "a") : (FILE*)nullptr; }();
			static int ts_call = 0;
			if (j == 0) ts_call++;
			if (tsf) {
				for (int kk = 0; kk < (bgpu[j] ? 2 : 1); kk++)
					for (int k = 0; k < m; k++) {
						const uint64_t* w = t.data() + (size_t)kk * 4 * m + 4 * (size_t)k;
						fprintf(tsf, "%d %d %d %d %llu %llu %llu %llu\n", ts_call, j, kk, k, (unsigned long long)w[0],
						        (unsigned long long)w[1], (unsigned long long)(w[2] & 0xFFFFFFFFu), (unsigned long long)(w[2] >> 32));
					}
				fflush(tsf);
			}
			for (int kk = 0; kk < (bgpu[j] ? 2 : 1); kk++) {
				const uint64_t* w = t.data() + (size_t)kk * 4 * m;
				uint64_t t0 = ~0ull;
				double dur = 0;
				std::vector<double> e(m);
				std::map<uint64_t, int> simd, cu;
				for (int k = 0; k < m; k++) t0 = std::min(t0, w[4 * k]);
				for (int k = 0; k < m; k++) {
					e[k] = (double)(w[4 * k + 1] - t0) * 1e-5;
					dur += (double)(w[4 * k + 1] - w[4 * k]) * 1e-5;
					const uint64_t hw = w[4 * k + 2];
					const uint64_t where = (hw >> 32) << 16 | ((hw >> 8) & 0xFF) | ((hw >> 13) & 7) << 8;   // xcc, se, cu
					cu[where]++;
					simd[where << 2 | ((hw >> 4) & 3)]++;
				}
				std::sort(e.begin(), e.end());
				auto pc = [&](double q) { return e[std::min((size_t)(q * (m - 1) + 0.5), (size_t)m - 1)]; };
				int hs[17] = {0}, hc[33] = {0};
				for (auto& x : simd) hs[std::min(x.second, 16)]++;
				for (auto& x : cu) hc[std::min(x.second, 32)]++;
				fprintf(stderr, "[tstamp] batch %d %s: wave ends (ms from first start) p0 %.0f p10 %.0f p50 %.0f p90 %.0f p100 %.0f; mean wave %.0f; CUs %zu SIMDs %zu\n",
				        j, kk ? "decode" : "encode", pc(0), pc(0.1), pc(0.5), pc(0.9), pc(1.0), dur / m, cu.size(), simd.size());
				fprintf(stderr, "[tstamp]   SIMDs by waves:");
				for (int i = 1; i <= 16; i++) if (hs[i]) fprintf(stderr, " %d:%d", i, hs[i]);
				fprintf(stderr, "   CUs by waves:");
				for (int i = 1; i <= 32; i++) if (hc[i]) fprintf(stderr, " %d:%d", i, hc[i]);
				fprintf(stderr, "\n");
				// mean duration by the waves on the same SIMD
				std::map<int, std::pair<double, int>> by;
				for (int k = 0; k < m; k++) {
					const uint64_t hw = w[4 * k + 2];
					const uint64_t where = (hw >> 32) << 16 | ((hw >> 8) & 0xFF) | ((hw >> 13) & 7) << 8;
					auto& q = by[simd[where << 2 | ((hw >> 4) & 3)]];
					q.first += (double)(w[4 * k + 1] - w[4 * k]) * 1e-5; q.second++;
				}
				fprintf(stderr, "[tstamp]   mean wave ms by waves on its SIMD:");
				for (auto& x : by) fprintf(stderr, " %d:%.0f(%d)", x.first, x.second.first / x.second.second, x.second.second);
				fprintf(stderr, "\n");
			}
		}
		std::vector<char> left(m, 0);                      // frames over the compacted pool's capacity
		for (int k = 0; k < m; k++) {
			if (re[2 * k + 1] == 2) {
				clear_status(b);
				set_last_error("device status word set: a fused level kernel's LDS ring hand-off or the compaction's look-back timed out; output discarded");
				return RIC_E_HIP;
			}
			if (re[2 * k + 1] == 4 && c.vcap) {
				// more level-0 values than the pool holds: the frame goes round
				// trip on the host (its GPU harvest output is overwritten then)
				left[k] = 1;
				n_fallback++;
				tr("left to the host (over the pool's value capacity)", f0 + k);
				if (!bgpu[j]) copied[j].done();                    // (no host decode task copies its stream)
				continue;
			}
			if (re[2 * k + 1]) {
				set_last_error("GPU stream coder: a stream larger than the pool's stream capacity");
				return RIC_E_CAPACITY;
			}
			if (re[2 * k] > cap[f0 + k]) return RIC_E_CAPACITY;
			len[f0 + k] = re[2 * k];
			if (bgpu[j]) {
				if ((rd[k] & 15) == 3) {
					set_last_error("GPU stream decoder: staging overrun at byte " + std::to_string(rd[k] >> 4) + " of frame " +
					               std::to_string(f0 + k) + " (stream " + std::to_string(re[2 * k]) + " bytes)");
					return RIC_E_CAPACITY;
				}
				stream_err |= rd[k] == 1;
			}
		}
		// the frames left to the host go round trip in host groups of up to SG
		// consecutive frames (a group per frame would hold the host threads to
		// two frames at a time: the two slot sets)
		for (int g0 = 0; g0 < m;) {
			if (!left[g0]) { g0++; continue; }
			int e = g0;
			while (e < m && e - g0 < SG && left[e]) e++;
			ready_host.push_back({f0 + g0, e - g0, false, 0, 0});
			g0 = e;
		}
		if (!bgpu[j]) {
			enc_ms_est = 0.5 * enc_ms_est + 0.5 * (now_ms() - t_kick[j]);
			// runs of up to SG coded frames (the ones left to the host excluded)
			for (int g0 = 0; g0 < m;) {
				if (left[g0]) { g0++; continue; }
				int e = g0;
				while (e < m && e - g0 < SG && !left[e]) e++;
				ready_dec.push_back({f0 + g0, e - g0, true, h, g0});
				g0 = e;
			}
			return RIC_OK;
		}
		for (int g0 = 0; g0 < m; g0 += S) {
			if (hv_done[j][g0 / S]) continue;                  // harvested while the launch ran
			const int r = harvest_group(j, g0);
			if (r) return r;
		}
		return RIC_OK;
	};
	struct Flight {
		HGroup g;
		int set;
		hipEvent_t ev;
		Latch done;
		FirstErr err;
	};
	std::deque<Flight> fl;
	std::vector<hipEvent_t> evs(2, nullptr);
	for (auto& e : evs) BCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
	bool set_busy[2] = {false, false};
	// RIC_SIDE_COPY: the host groups' band copies on a side stream -- 0 none
	// (stream order), 1 (default) the step's front only, 2 every host group (measured
	// the same or lower: 11,691-11,913 against 11,907-11,969 Mpix/s, r6sc2)
	static const int side_copy_mode = [] { const char* e = getenv("RIC_SIDE_COPY"); return e ? atoi(e) : 1; }();
	const bool side_copy_on = side_copy_mode >= 1;
	bool pool_direct = C == 1;                           // (gpu_encode_plane's direct-write condition)
	{
		P.set_weight(trans);
		const int lambda = lambda_of(q, 0);
		int qin = quant_of(q, 0);
		for (int l = 0; l < P.nlev && pool_direct; l++) {
			const int mode = fwdq_mode(P.L[l], trans, level_qp(P, l, qin, lambda), 1);
			pool_direct = mode != FQ_NONE && (l + 1 < P.nlev || mode == FQ_GENERIC);
		}
	}
	// side_copy: the group's band copies on a stream of their own (the step's
	// front: slot set 1's copies beside the pool's forward levels, which use
	// slot set 0 as scratch and would otherwise wait for them in stream order)
	auto launch_group = [&](const HGroup& g, bool side_copy = false) -> int {
		const int set = set_busy[0] ? 1 : 0;
		set_busy[set] = true;
		fl.emplace_back();
		Flight& F = fl.back();
		F.g = g; F.set = set; F.ev = evs[set];
		// set 0 too when the pool's forward levels write it straight (every
		// level fused): the scratch the pool front and the harvests use in slot
		// set 0 ([0, lo) and region C) is then disjoint from what the copies
		// read ([cmp_dense, b_end) and d_cmp)
		side_copy = side_copy && C == 1 && !g.gpu && (set == 1 || pool_direct);
		if (side_copy && !b->xst) BCHK(hipStreamCreateWithFlags(&b->xst, hipStreamNonBlocking));
		if (!g.gpu) {
			if (C == 1) {
				int r = gpu_encode_plane(b, set, g.m, 0, pix + g.f0, q, trans, !side_copy, -1, 1, yflag);
				if (!r && side_copy) r = d2h_slots(b, set, g.m, b->xst);
				if (r) return r;
			} else {
				// plane p of frame i in slot C i + p, then every slot's bands to the host
				const int s0 = set * S;
				for (int p = 0; p < C; p++) {
					int r = gpu_encode_plane(b, set, g.m, p, pix + g.f0, q, trans, false, s0 + p, C, yflag);
					if (r) return r;
				}
				int r = d2h_slots(b, set, C * g.m);
				if (r) return r;
			}
			BCHK(hipEventRecord(F.ev, side_copy ? b->xst : b->st));
			if (trace > 2) tr("  forward issued", g.f0);
		}
		F.done.reset(g.m);
		if (trace > 1) tr(g.gpu ? "decode group launched" : "host group launched", g.f0);
		for (int i = 0; i < g.m; i++) {
			const int slot = set * S + C * i, f = g.f0 + i;    // colour: the frame's planes in slots slot .. slot + 2
			Flight* pf = &F;
			if (!g.gpu) {
				b->pool->submit([=] {
					int r1 = bfail(hipEventSynchronize(pf->ev), "hipEventSynchronize") ? RIC_E_HIP : RIC_OK;
					if (trace > 2 && i == 0) tr("  task: forward passed", f);
					for (int p = 0; p < C && !r1; p++) r1 = host_encode_plane(b, slot + p, p, q, trans, out[f], cap[f], &len[f], slot);
					if (!r1) mark_ready(b, f, len[f]);
					for (int p = 0; p < C && !r1; p++) {
						const int rp = host_decode_plane(b, slot + p, p, out[f], len[f], slot);
						if (rp == RIC_E_STREAM && p + 1 < C) continue;     // (the last plane reports the overrun)
						r1 = rp;
					}
					pf->err.put(r1);
					pf->done.done();
				});
			} else {
				const uint8_t* src = c.d_out + ((size_t)g.half * c.n + g.k0 + i) * c.ocap;
				Latch* cl = &copied[(f - n_host) / c.n];
				std::atomic<long>* pdec_us = &dec_us;
				std::atomic<long>* pdec_n = &dec_n;
				b->pool->submit([=] {
					int r1 = set_dev(b->device);
					if (!r1) r1 = bfail(d2h(b, (int)f, out[f], src, len[f]), "hipMemcpy stream") ? RIC_E_HIP : RIC_OK;
					if (!r1) mark_ready(b, f, len[f]);
					cl->done();
					// the set's mirrors: the previous group's H2D from them has passed
					if (!r1) r1 = bfail(hipEventSynchronize(pf->ev), "hipEventSynchronize") ? RIC_E_HIP : RIC_OK;
					const double t0 = now_ms();
					for (int p = 0; p < C && !r1; p++) {
						const int rp = host_decode_plane(b, slot + p, p, out[f], len[f], slot);
						if (rp == RIC_E_STREAM && p + 1 < C) continue;     // (the last plane reports the overrun)
						r1 = rp;
					}
					pdec_us->fetch_add((long)((now_ms() - t0) * 1e3));
					pdec_n->fetch_add(1);
					pf->err.put(r1);
					pf->done.done();
				});
			}
		}
		return RIC_OK;
	};
	auto finish_group = [&]() -> int {
		Flight& F = fl.front();
		const int r = F.err.get();
		int r2 = RIC_OK;
		if (r && r != RIC_E_STREAM) r2 = r;
		stream_err |= r == RIC_E_STREAM;
		if (!F.g.gpu) {
			b->hyb_host_ms = now_ms() - t_entry;
			if (++host_groups_done == 1 || host_groups_done == (n_host + S - 1) / S || trace > 1) tr("host group done", host_groups_done);
		} else if (trace > 1) {
			tr("decode group done", F.g.f0);
		}
		const bool fuse = C == 1 && pix_fuse_ok(b, trans, pix_out + F.g.f0, F.g.m);
		const PixFuse pf{pix_out + F.g.f0, qs.data(), F.g.f0};
		if (!r2 && C == 1) r2 = gpu_decode_plane(b, F.set, F.g.m, 0, qs.data(), trans, true, -1, 1, yflag, nullptr, 0, 0,
		                                         fuse ? &pf : nullptr);
		if (!r2 && C > 1) {
			r2 = h2d_slots(b, F.set, C * F.g.m);
			for (int p = 0; p < C && !r2; p++)
				r2 = gpu_decode_plane(b, F.set, F.g.m, p, qs.data(), trans, false, F.set * S + p, C, yflag);
		}
		if (trace > 2) tr("  inverse issued", F.g.f0);
		if (!r2 && !fuse) r2 = gpu_pix_out(b, F.set, F.g.m, qs.data(), pix_out + F.g.f0, 1, F.g.f0);
		if (trace > 2) tr("  pix out issued", F.g.f0);
		if (!r2) BCHK(hipEventRecord(F.ev, b->st));   // the set's mirrors are free once this passes
		set_busy[F.set] = false;
		fl.pop_front();
		return r2;
	};
	bool running[2] = {false, false};
	while (rc == RIC_OK && (finished < nbatch || !ready_host.empty() || !ready_dec.empty() || !fl.empty())) {
		// the oldest batch whose encode is still out: a GPU-decoded batch's
		// streams start for the host
		if (enc_seen < kicked) {
			const hipError_t e = hipEventQuery(c.ev_enc[enc_seen & 1]);
			if (e == hipSuccess) {
				tr("encoded", enc_seen);
				if (bgpu[enc_seen]) copy_out(enc_seen);
				enc_seen++;
			} else if (e != hipErrorNotReady) {
				rc = bfail(e, "coder stream") ? RIC_E_HIP : RIC_E_HIP;
				break;
			}
		}
		// the oldest coder batch (batches finish in order: one per half, alternating)
		if (finished < kicked && enc_seen > finished) {
			const int h = finished & 1;
			const hipError_t e = hipEventQuery(c.ev_done[h]);
			if (e == hipSuccess) {
				running[h] = false;
				b->hyb_gpu_ms = now_ms() - t_entry;
				tr("decoded", finished);
				rc = harvest(finished);
				finished++;
				if (rc == RIC_OK && finished == nbatch) t1_set = hipEventRecord(ev_t1, b->st) == hipSuccess;
				if (rc) break;
			} else if (e != hipErrorNotReady) {
				rc = bfail(e, "coder stream") ? RIC_E_HIP : RIC_E_HIP;
				break;
			}
		}
		// kick the next batch when its half is free: the batch before it on that
		// half has been harvested and (host decode) its streams copied out
		if (fwd_ahead && kicked == 0 && nbatch >= 2) {
			// the step's start: the first host groups' and both coder batches'
			// forward levels, then both coder launches (level 0 runs alone on
			// the CUs, not beside the coder waves: the alone forms)
			b->alone(true);
			while (rc == RIC_OK && fl.size() < 2 && !ready_host.empty()) {
				const HGroup g = ready_host.front();
				ready_host.pop_front();
				rc = launch_group(g, side_copy_on);
			}
			if (rc == RIC_OK) rc = kick_fwd(0);
			if (rc == RIC_OK) rc = kick_fwd(1);
			b->alone(false);                       // the coder's waves from here on
			if (rc == RIC_OK && merge && gpu_decode == 1) {
				rc = kick_both();
				running[0] = running[1] = rc == RIC_OK;
				kicked = 2;
			}
			for (int j = kicked; j < 2 && rc == RIC_OK; j++) {
				rc = kick_coder(j, j == 0);
				running[j] = rc == RIC_OK;
				kicked++;
			}
			if (rc) break;
		}
		while (rc == RIC_OK && kicked < nbatch && kicked - finished < 2 &&
		       (kicked < 2 || copied[kicked - 2].wait_for_ms(0))) {
			rc = kick(kicked);
			running[kicked & 1] = rc == RIC_OK;
			kicked++;
		}
		if (rc) break;
		while (fl.size() < 2 && (!ready_dec.empty() || !ready_host.empty())) {
			HGroup g;
			if (!ready_dec.empty()) { g = ready_dec.front(); ready_dec.pop_front(); }
			else { g = ready_host.front(); ready_host.pop_front(); }
			rc = launch_group(g, side_copy_mode >= 2);
			if (rc) break;
		}
		if (rc) break;
		if (finished < kicked) {
			rc = early_harvest();
			if (rc) break;
		}
		if (!fl.empty()) {
			if (fl.front().done.wait_for_ms(finished < kicked ? 2 : 20)) {
				rc = finish_group();
				if (rc) break;
			}
		} else {
			std::this_thread::sleep_for(std::chrono::milliseconds(1));
		}
	}
	// on an error: let queued tasks, copies and the coder finish before returning
	while (!fl.empty()) { fl.front().done.wait(); fl.pop_front(); }
	for (auto& t : copier)
		if (t.joinable()) t.join();
	for (int h = 0; h < 2; h++)
		if (c.st[h]) (void)hipStreamSynchronize(c.st[h]);
	const bool ok = !bfail(hipStreamSynchronize(b->st), "hipStreamSynchronize");
	if (ok && t1_set) {
		float ms = 0;
		if (hipEventElapsedTime(&ms, ev_t0, ev_t1) == hipSuccess) b->hyb_gpu_ms = ms;
	}
	b->hyb_fallback = n_fallback;
	if (trace)
		fprintf(stderr, "[hybrid] %d coder-frame groups harvested while the launch ran; %d frames left to the host "
		                "(over the compacted pool's value capacity)\n", hv_early, n_fallback);
	tr("end", rc);
	for (auto& e : evs) (void)hipEventDestroy(e);
	if (rc == RIC_E_HIP) clear_status(b);
	if (rc) return rc;
	if (!ok) return RIC_E_HIP;
	b->prof.harvest();
	return stream_err ? RIC_E_STREAM : RIC_OK;
}

// Diagnostics: the GPU stages alone, `iters` times over n frames (slot set
// 0): pixel conversion + fused forward levels + D2H, then H2D + inverse
// levels of the quantised bands just copied + pixel output (no host coding;
// the decode's values are not a real decode).  For kernel timing
// (ric_batch_prof_*, rocprofv3).
int ric_batch_diag_gpu(ric_batch* b, const uint8_t* const* pix, int n, int q, int trans, int iters, uint8_t* const* pix_out)
{
	if (!b || !pix || n < 1 || n > b->slots || iters < 0) return RIC_E_ARG;
	if (set_dev(b->device)) return RIC_E_HIP;
	std::vector<int> qs(n, q);
	for (int it = 0; it < iters; it++) {
		int rc = gpu_encode_plane(b, 0, n, 0, pix, q, trans);
		if (!rc) rc = gpu_decode_plane(b, 0, n, 0, qs.data(), trans);
		if (!rc && pix_out) rc = gpu_pix_out(b, 0, n, qs.data(), pix_out, 1);
		if (rc) return rc;
	}
	BCHK(hipStreamSynchronize(b->st));
	b->prof.harvest();
	return RIC_OK;
}

int ric_batch_diag_gpu_encode(ric_batch* b, const uint8_t* const* pix, int n, int q, int trans, int iters)
{
	if (!b || !pix || n < 1 || n > b->slots || iters < 0) return RIC_E_ARG;
	if (set_dev(b->device)) return RIC_E_HIP;
	for (int it = 0; it < iters; it++)
		if (int rc = gpu_encode_plane(b, 0, n, 0, pix, q, trans)) return rc;
	BCHK(hipStreamSynchronize(b->st));
	b->prof.harvest();
	return RIC_OK;
}

int ric_batch_prof_enable(ric_batch* b, int on)
{
	if (!b) return RIC_E_ARG;
	if (set_dev(b->device)) return RIC_E_HIP;
	BCHK(hipStreamSynchronize(b->st));
	b->prof.harvest();
	b->prof.on = on != 0;
	b->prof.reset();
	return RIC_OK;
}

int ric_batch_prof_read(ric_batch* b, double* ms, long* frames, long* launches, int n)
{
	if (!b || !ms || !frames || !launches) return RIC_E_ARG;
	for (int i = 0; i < n && i < B_COUNT; i++) { ms[i] = b->prof.ms[i]; frames[i] = b->prof.frames[i]; launches[i] = b->prof.launches[i]; }
	return B_COUNT;
}

}  // extern "C"

// When each side of the last ric_batch_roundtrip_hybrid finished: its last
// host round-trip group and its last stream-coder batch (ms from entry).
int ric_batch_hybrid_times(ric_batch* b, double* host_ms, double* gpu_ms)
{
	if (!b || !host_ms || !gpu_ms) return RIC_E_ARG;
	*host_ms = b->hyb_host_ms;
	*gpu_ms = b->hyb_gpu_ms;
	return RIC_OK;
}

// Frames of the last ric_batch_roundtrip_hybrid the stream coder left to a
// host round trip (over the compacted pool's value capacity)
int ric_batch_hybrid_fallbacks(ric_batch* b, int* frames)
{
	if (!b || !frames) return RIC_E_ARG;
	*frames = b->hyb_fallback;
	return RIC_OK;
}
