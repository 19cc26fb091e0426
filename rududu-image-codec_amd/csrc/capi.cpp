// capi.cpp -- the C-ABI (include/ric_gpu.h): object lifetimes, HBM arenas,
// and the orchestration of the GPU stages and the host serial coder.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>
#include <chrono>
#include <mutex>

#include "ric_gpu.h"
#include "ric_types.h"
#include "ric_kernels.h"
#include "ric_image.h"
#include "entropy.h"
#include "codec_params.h"
#include "wavelet_api.h"
#include "host_pool.h"
#include <memory>

using namespace ric;

namespace {

thread_local std::string g_err;

bool hip_fail(hipError_t e, const char* what)
{
	if (e == hipSuccess) return false;
	g_err = std::string(what) + ": " + hipGetErrorString(e);
	return true;
}

#define HIPCHK(x) do { if (hip_fail((x), #x)) return RIC_E_HIP; } while (0)

// Stage timers (ric_prof_*): GPU stages by hipEvents on the object's stream,
// host stages by a steady clock.  Harvested at the sync points that already
// exist (no extra synchronisation in the timed path).
enum Stage { S_FWD0, S_FWD, S_QUANT, S_D2H, S_HENC, S_HDEC, S_H2D, S_DEQ, S_INV, S_PIXIN, S_PIXOUT, S_COUNT };

struct Prof {
	bool on = false;
	hipEvent_t a[S_COUNT] = {}, b[S_COUNT] = {};
	bool pending[S_COUNT] = {};
	double ms[S_COUNT] = {};
	long n[S_COUNT] = {};
	void enable(bool e)
	{
		on = e;
		if (e && !a[0])
			for (int i = 0; i < S_COUNT; i++) { (void)hipEventCreate(&a[i]); (void)hipEventCreate(&b[i]); }
	}
	void destroy()
	{
		if (!a[0]) return;
		for (int i = 0; i < S_COUNT; i++) { (void)hipEventDestroy(a[i]); (void)hipEventDestroy(b[i]); }
		a[0] = nullptr;
	}
	void begin(int s, hipStream_t st) { if (on && !pending[s]) (void)hipEventRecord(a[s], st); }
	void end(int s, hipStream_t st) { if (on && !pending[s]) { (void)hipEventRecord(b[s], st); pending[s] = true; } }
	void harvest()
	{
		if (!on) return;
		for (int i = 0; i < S_COUNT; i++)
			if (pending[i] && hipEventQuery(b[i]) == hipSuccess) {
				float t = 0;
				if (hipEventElapsedTime(&t, a[i], b[i]) == hipSuccess) { ms[i] += t; n[i]++; }
				pending[i] = false;
			}
	}
	void host(int s, double t_ms) { if (on) { ms[s] += t_ms; n[s]++; } }
	void reset() { for (int i = 0; i < S_COUNT; i++) { ms[i] = 0; n[i] = 0; } }
};

double now_ms()
{
	return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct ric_wavelet {
	Prof prof;
	int device = 0;
	Pyramid P;
	char* d_arena = nullptr;
	char* h_arena = nullptr;          // pinned mirror of the band arena
	int16_t* d_img = nullptr;         // scratch for host-resident images
	size_t img_pitch = 0;             // elements
	hipStream_t st = nullptr;
	bool own_stream = false;
	bool host_valid = false;          // bands live on the host (after a decode)
	// A Transform of a host image is deferred until the next call, so that a
	// CodeBand right after it runs as one fused forward+quantiser pass.
	bool pend = false;
	int pend_trans = 0;
	// CodeBand's serial half with the bands modelled on host_threads - 1
	// pool threads (encode_bands_split); 1: one thread, no split
	int host_threads = 1;
	std::unique_ptr<Pool> pool;
	std::vector<EvBuf> evbufs;
	// the one-band reductions' result words (ric_band_tsuq / ric_band_sums):
	// a device block and its pinned mirror, allocated with the arena
	char* d_small = nullptr;
	char* h_small = nullptr;
	// ric_band_host_ref: bands handed out in the reference's layout (row stride
	// DimXAlign: DimX rounded up to 32 bytes, src/lib/band.cpp:57), each a
	// stable host buffer; active ones are written back into the mirror before
	// the mirror goes to the device, and refreshed when the mirror is rewritten
	std::vector<std::vector<char>> ref_buf;
	std::vector<char> ref_active;
};

struct ric_mux {
	Mux m;
	uint8_t* buf = nullptr;
	bool encoder = true;
};

struct ric_codec {
	int device = 0;
	int w = 0, h = 0, channels = 1;
	ric_wavelet* wav = nullptr;
	int16_t* d_planes = nullptr;      // channels coding planes, pitch
	uint8_t* d_pix = nullptr;         // staging for host pixels
	int16_t* d_out = nullptr;         // staging for host int16 output planes
	long pitch = 0;
	std::vector<uint8_t> stream;      // coder buffer
	std::vector<uint8_t> dstream;     // decoder input (2 zero bytes + payload), reused per frame
};

namespace {

int set_dev(int device) { return hip_fail(hipSetDevice(device), "hipSetDevice") ? RIC_E_HIP : RIC_OK; }

// The device status word (Pyramid::status_off): a fused level kernel whose
// LDS ring hand-off timed out raised it (dwt.hip ring_wait_ge); its bands and
// records are not trusted.  in_copy: the word already came with a region-B
// copy, else it is read here (the caller has synchronised the stream).
int take_status(ric_wavelet* w, bool in_copy)
{
	int32_t* hs = (int32_t*)(w->h_arena + w->P.status_off);
	if (!in_copy) {
		HIPCHK(hipMemcpyAsync(hs, w->d_arena + w->P.status_off, sizeof(int32_t), hipMemcpyDeviceToHost, w->st));
		HIPCHK(hipStreamSynchronize(w->st));
	}
	if (*hs == 0) return RIC_OK;
	*hs = 0;
	HIPCHK(hipMemsetAsync(w->d_arena + w->P.status_off, 0, sizeof(int32_t), w->st));
	HIPCHK(hipStreamSynchronize(w->st));
	g_err = "fused level kernel: LDS ring hand-off timed out (device status word set; output discarded)";
	return RIC_E_HIP;
}

// the reference's row stride of band B in samples (CBand::Init, src/lib/band.cpp:57, ALIGN 32)
int ref_stride(const Band& B)
{
	const int ss = B.is_int ? 4 : 2;
	return ((B.dx * ss + 31) & ~31) / ss;
}

// active reference-layout views <-> the host mirror (rows of dx samples)
void ref_copy(ric_wavelet* w, bool to_mirror)
{
	for (size_t i = 0; i < w->ref_active.size(); i++) {
		if (!w->ref_active[i]) continue;
		const Band& B = w->P.band((int)i);
		const size_t ss = B.is_int ? 4 : 2, rs = (size_t)ref_stride(B) * ss, ms = (size_t)B.pitch * ss;
		char* m = w->h_arena + B.off;
		char* r = w->ref_buf[i].data();
		for (int y = 0; y < B.dy; y++) {
			if (to_mirror) memcpy(m + y * ms, r + y * rs, (size_t)B.dx * ss);
			else memcpy(r + y * rs, m + y * ms, (size_t)B.dx * ss);
		}
	}
}

// region A (+ B with records): see Pyramid in ric_types.h
int to_host(ric_wavelet* w, bool records = false)
{
	const size_t lo = 0, hi = records ? w->P.b_end : w->P.a_end;
	w->prof.begin(S_D2H, w->st);
	HIPCHK(hipMemcpyAsync(w->h_arena + lo, w->d_arena + lo, hi - lo, hipMemcpyDeviceToHost, w->st));
	w->prof.end(S_D2H, w->st);
	HIPCHK(hipStreamSynchronize(w->st));
	w->prof.harvest();
	return records ? take_status(w, true) : RIC_OK;
}

int to_device(ric_wavelet* w)
{
	if (!w->host_valid) return RIC_OK;
	ref_copy(w, true);            // what the caller wrote through reference-layout pBand views
	const size_t lo = 0, hi = w->P.a_end;
	w->prof.begin(S_H2D, w->st);
	HIPCHK(hipMemcpyAsync(w->d_arena + lo, w->h_arena + lo, hi - lo, hipMemcpyHostToDevice, w->st));
	w->prof.end(S_H2D, w->st);
	// the host arena is rewritten by the next DecodeBand: wait for the copy
	HIPCHK(hipStreamSynchronize(w->st));
	w->prof.harvest();
	w->host_valid = false;
	return RIC_OK;
}

BandView view(ric_wavelet* w, const Band& B)
{
	BandView v;
	v.p = w->h_arena + B.off; v.pitch = B.pitch; v.dx = B.dx; v.dy = B.dy; v.is_int = B.is_int;
	return v;
}

int forward(ric_wavelet* w, const int16_t* dimg, long stride, int trans)
{
	Pyramid& P = w->P;
	w->prof.begin(S_FWD, w->st);
	for (int l = 0; l < P.nlev; l++) {
		const void* src;
		long sp;
		int vec;
		if (l == 0) {
			src = dimg; sp = stride;
			vec = (stride % 4 == 0) && ((uintptr_t)dimg % 8 == 0);
		} else {
			const Band& LL = P.L[l - 1].b[BL];
			src = w->d_arena + LL.off; sp = LL.pitch; vec = 1;
		}
		if (l == 0) w->prof.begin(S_FWD0, w->st);
		launch_fwd_level(P.L[l], src, sp, w->d_arena, trans, vec, w->st);
		if (l == 0) w->prof.end(S_FWD0, w->st);
	}
	w->prof.end(S_FWD, w->st);
	HIPCHK(hipGetLastError());
	w->host_valid = false;
	return RIC_OK;
}

int inverse(ric_wavelet* w, int16_t* dimg, long stride, int trans)
{
	Pyramid& P = w->P;
	int rc = to_device(w);
	if (rc) return rc;
	w->prof.begin(S_INV, w->st);
	for (int l = P.nlev - 1; l >= 0; l--) {
		const Level& L = P.L[l];
		void* out;
		long po;
		int out_int;
		if (l == 0) { out = dimg; po = stride; out_int = 0; }
		else { const Band& LL = P.L[l - 1].b[BL]; out = w->d_arena + LL.off; po = LL.pitch; out_int = LL.is_int; }
		launch_inv_level(L, L.b[BL], w->d_arena, out, po, out_int, trans, w->st);
	}
	w->prof.end(S_INV, w->st);
	HIPCHK(hipGetLastError());
	return RIC_OK;
}

void ll_params(ric_wavelet* w, int quant, int& Q, int& iQ, int& T0) { ll_params(w->P, quant, Q, iQ, T0); }
void quant_ll(ric_wavelet* w, int quant)
{
	int Q, iQ, T0;
	ll_params(w, quant, Q, iQ, T0);
	launch_quant_ll(w->P, Q, iQ, T0, w->d_arena, w->st);
}

// The GPU half of CWavelet2D::CodeBand (src/lib/wavelet2d.cpp:83-177) on a
// pyramid already transformed: buildTree on every level, the LL TSUQ, and the
// zerotree block records.
int quantize_gpu(ric_wavelet* w, int quant, int lambda)
{
	Pyramid& P = w->P;
	int rc = to_device(w);   // bands a caller wrote through CBand::pBand
	if (rc) return rc;
	// buildTree on every level, finest first (bandcodec.cpp:239-319)
	int qin = quant;
	w->prof.begin(S_QUANT, w->st);
	for (int l = 0; l < P.nlev; l++) {
		QuantParams qp = level_qp(P, l, qin, lambda);
		launch_quant_level(P, l, qp, w->d_arena, w->st);
	}
	quant_ll(w, quant);
	// zerotree symbolisation of every level (parents must be quantised first)
	for (int l = 0; l < P.nlev; l++) launch_blocks_level(P, l, true, true, w->d_arena, w->st);
	w->prof.end(S_QUANT, w->st);
	HIPCHK(hipGetLastError());
	w->host_valid = false;
	return RIC_OK;
}

// Transform + the GPU half of CodeBand in one pass over the pyramid: every 9/7
// short level runs the fused forward+quantiser (dwt.hip k_fwdq), the others the
// separate forward level, quantiser and record kernels.
// in8: dimg holds 8-bit pixels after the ric level shift (the codec's own
// planes), so level 0 may take the plain packed mult08 (ric_kernels.h)
int encode_gpu(ric_wavelet* w, const int16_t* dimg, long stride, int trans, int quant, int lambda, bool in8 = false)
{
	Pyramid& P = w->P;
	bool fused[kMaxLevels] = {};
	bool ll_done = false;
	int qin = quant;
	w->prof.begin(S_FWD, w->st);
	for (int l = 0; l < P.nlev; l++) {
		const void* src;
		long sp;
		int vec8, vec16;
		if (l == 0) {
			src = dimg; sp = stride;
			vec8 = (stride % 4 == 0) && ((uintptr_t)dimg % 8 == 0);
			vec16 = (stride % 8 == 0) && ((uintptr_t)dimg % 16 == 0);
		} else {
			const Band& LL = P.L[l - 1].b[BL];
			src = w->d_arena + LL.off; sp = LL.pitch; vec8 = vec16 = 1;
		}
		QuantParams qp = level_qp(P, l, qin, lambda);
		const int mode = fwdq_mode(P.L[l], trans, qp, vec16);
		fused[l] = mode != FQ_NONE;
		if (l == 0) w->prof.begin(S_FWD0, w->st);
		if (mode == FQ_PACKED) {
			launch_fwdq_level(P, l, src, sp, vec8, vec16, qp, w->d_arena, w->st, in8 ? 1 : 0);
		} else if (mode == FQ_GENERIC) {
			const bool coarsest = l + 1 == P.nlev;
			int llQ = 0, lliQ = 0, llT0 = 0;
			if (coarsest) { ll_params(w, quant, llQ, lliQ, llT0); ll_done = true; }
			launch_fwdq_gen_level(P, l, src, sp, vec8, qp, coarsest, lliQ, llT0, w->d_arena, w->st);
		} else {
			launch_fwd_level(P.L[l], src, sp, w->d_arena, trans, vec8, w->st);
			launch_quant_level(P, l, qp, w->d_arena, w->st);
		}
		if (l == 0) w->prof.end(S_FWD0, w->st);
	}
	if (!ll_done) quant_ll(w, quant);
	// records of the unfused levels, parent info below the unfused levels
	for (int l = 0; l < P.nlev; l++)
		launch_blocks_level(P, l, !fused[l], l + 1 < P.nlev && !fused[l + 1], w->d_arena, w->st);
	w->prof.end(S_FWD, w->st);
	HIPCHK(hipGetLastError());
	w->host_valid = false;
	w->pend = false;
	return RIC_OK;
}

// run a deferred Transform (see ric_wavelet::pend) before anything else
int flush_pending(ric_wavelet* w)
{
	if (!w->pend) return RIC_OK;
	w->pend = false;
	return forward(w, w->d_img, (long)w->img_pitch, w->pend_trans);
}

// The host half: bands + records to the pinned mirror (unless the caller
// copied them already), then the serial coder.  state: also leave the bands
// in the state the reference's CodeBand leaves them in (sign-magnitude, the
// INSIGNIF markers the scan consumes cleared: src/lib/bandcodec.cpp:510-588),
// for API callers that read the bands or run TSUQi next
// (src/lib/rududucodec.cpp:70-73); the codec's .ric path does not need it.
int code_band_host(ric_wavelet* w, Mux& m, bool copy = true, bool state = false)
{
	Pyramid& P = w->P;
	if (copy) {
		int rc = to_host(w, true);
		if (rc) return rc;
	}
	// serial part: LL DPCM, then coarse -> fine, V, H, D (wavelet2d.cpp:119-159)
	const double t0 = now_ms();
	if (w->host_threads > 1) {
		std::vector<BandRecs> bands;
		for (int l = P.nlev - 1; l >= 0; l--) {
			const int order[3] = {BV, BH, BD};
			for (int k = 0; k < 3; k++) {
				const Band& B = P.L[l].b[order[k]];
				bands.push_back({(const uint64_t*)(w->h_arena + P.rec_off[l][order[k]]),
				                 l + 1 < P.nlev ? (const uint8_t*)(w->h_arena + P.pin_off[l][order[k]]) : nullptr,
				                 view(w, B), l == 0});
			}
		}
		encode_bands_split(m, *w->pool, w->evbufs, view(w, P.coarsest_ll()), bands.data(), (int)bands.size());
	} else {
		pred_encode(m, view(w, P.coarsest_ll()));
		for (int l = P.nlev - 1; l >= 0; l--) {
			const int order[3] = {BV, BH, BD};
			for (int k = 0; k < 3; k++) {
				const Band& B = P.L[l].b[order[k]];
				const uint64_t* rec = (const uint64_t*)(w->h_arena + P.rec_off[l][order[k]]);
				const uint8_t* pin = l + 1 < P.nlev ? (const uint8_t*)(w->h_arena + P.pin_off[l][order[k]]) : nullptr;
				tree_encode_records_fast(m, rec, pin, view(w, B), l == 0);
			}
		}
	}
	w->prof.host(S_HENC, now_ms() - t0);
	if (state) {
		for (int l = P.nlev - 1; l >= 0; l--) {
			const int order[3] = {BV, BH, BD};
			for (int k = 0; k < 3; k++) {
				BandView par;
				if (l + 1 < P.nlev) par = view(w, P.L[l + 1].b[order[k]]);
				tree_encode_state(view(w, P.L[l].b[order[k]]), par, l > 0);
			}
		}
	}
	// the host mirror is now the reference: CodeBand's final state with
	// `state`, else buildTree's (the codec path never reads it back)
	w->host_valid = true;
	ref_copy(w, false);
	return RIC_OK;
}

// CWavelet2D::DecodeBand, src/lib/wavelet2d.cpp:179-222
int decode_band(ric_wavelet* w, Mux& m)
{
	Pyramid& P = w->P;
	// every band is overwritten: pred writes the LL, tree() Clear()s its band first
	const double t0 = now_ms();
	BandView ll = view(w, P.coarsest_ll());
	pred_decode(m, ll);
	for (int l = P.nlev - 1; l >= 0; l--) {
		const int order[3] = {BV, BH, BD};
		for (int k = 0; k < 3; k++) {
			BandView par;
			if (l + 1 < P.nlev) par = view(w, P.L[l + 1].b[order[k]]);
			tree_decode_fast(m, view(w, P.L[l].b[order[k]]), par, l == 0, l > 0);
		}
	}
	w->prof.host(S_HDEC, now_ms() - t0);
	w->host_valid = true;
	ref_copy(w, false);
	return m.overflow() ? RIC_E_STREAM : RIC_OK;
}

// DecodeBand + TSUQi + TransformI of one plane, pipelined by level (the
// codec's decode path).  The reference decodes coarse -> fine
// (src/lib/wavelet2d.cpp:179-222) and inverts coarsest level first (:960-990).
// Decoding level l also rewrites level l + 1: the zerotree scan clears the
// parent markers it consumes (src/lib/bandcodec.cpp:528-531).  So once the
// host has decoded level l, level l + 1 is final: its bands go to the device
// and its inverse (TSUQi fused, quant != 0) is queued while the host decodes
// level l - 1; level 0 follows the last host step.  One stream sync, at the end.
int decode_inverse_pipelined(ric_wavelet* w, Mux& m, int16_t* dimg, long stride, int trans, int quant)
{
	Pyramid& P = w->P;
	auto put = [&](size_t lo, size_t hi) -> int {
		HIPCHK(hipMemcpyAsync(w->d_arena + lo, w->h_arena + lo, hi - lo, hipMemcpyHostToDevice, w->st));
		return RIC_OK;
	};
	auto issue = [&](int l) -> int {
		// the coarsest level's D, H, V and the LL (contiguous in region A) go
		// here; a finer level's bands went one by one as each became final
		const Level& L = P.L[l];
		if (l + 1 == P.nlev) {
			int rc = put(L.b[BD].off, P.a_end);
			if (rc) return rc;
		}
		void* out;
		long po;
		int out_int;
		if (l == 0) { out = dimg; po = stride; out_int = 0; }
		else { const Band& LL = P.L[l - 1].b[BL]; out = w->d_arena + LL.off; po = LL.pitch; out_int = LL.is_int; }
		if (quant) {
			const int q[4] = {tsuqi_factor(L.b[BD], quant), tsuqi_factor(L.b[BH], quant), tsuqi_factor(L.b[BV], quant),
			                  l + 1 == P.nlev ? tsuqi_factor(L.b[BL], quant) : 1};
			launch_inv_level(L, L.b[BL], w->d_arena, out, po, out_int, trans, w->st, q);
		} else {
			launch_inv_level(L, L.b[BL], w->d_arena, out, po, out_int, trans, w->st);
		}
		return RIC_OK;
	};
	const double t0 = now_ms();
	pred_decode(m, view(w, P.coarsest_ll()));
	for (int l = P.nlev - 1; l >= 0; l--) {
		const int order[3] = {BV, BH, BD};
		for (int k = 0; k < 3; k++) {
			BandView par;
			if (l + 1 < P.nlev) par = view(w, P.L[l + 1].b[order[k]]);
			tree_decode_fast(m, view(w, P.L[l].b[order[k]]), par, l == 0, l > 0);
			// final now: the parent band (this scan cleared its markers) below
			// the coarsest level, and a finest band (no children) itself --
			// their copies overlap the next bands' decoding
			const Band* done[2] = {l + 2 < P.nlev ? &P.L[l + 1].b[order[k]] : nullptr, l == 0 ? &P.L[0].b[order[k]] : nullptr};
			for (const Band* B : done)
				if (B) {
					int rc = put(B->off, B->off + B->bytes());
					if (rc) return rc;
				}
		}
		if (l + 1 < P.nlev) {
			int rc = issue(l + 1);
			if (rc) return rc;
		}
	}
	w->prof.host(S_HDEC, now_ms() - t0);
	int rc = issue(0);
	if (rc) return rc;
	HIPCHK(hipGetLastError());
	// the host mirror is rewritten by the next DecodeBand: wait for the copies
	HIPCHK(hipStreamSynchronize(w->st));
	w->host_valid = false;    // the device now holds these bands
	return m.overflow() ? RIC_E_STREAM : RIC_OK;
}

// CWavelet2D::TSUQi / CBand::TSUQi (src/lib/wavelet2d.cpp:248-268, band.h:94-107)
int tsuqi(ric_wavelet* w, int quant)
{
	int rc = to_device(w);
	if (rc) return rc;
	Pyramid& P = w->P;
	w->prof.begin(S_DEQ, w->st);
	for (int i = 0; i < P.nbands(); i++) {
		const Band& B = P.band(i);
		const bool sh = !B.is_int;
		int q = tr_any(sh, quant);
		q = tr_any(sh, (int)((float)q / B.weight));
		if (q == 0) q = 1;
		launch_dequant_band(B, q, w->d_arena, w->st);
	}
	w->prof.end(S_DEQ, w->st);
	HIPCHK(hipGetLastError());
	return RIC_OK;
}

// CWavelet2D::CodeBand, src/lib/wavelet2d.cpp:83-177
int code_band(ric_wavelet* w, Mux& m, int quant, int lambda)
{
	int rc = w->pend ? encode_gpu(w, w->d_img, (long)w->img_pitch, w->pend_trans, quant, lambda)
	                 : quantize_gpu(w, quant, lambda);
	return rc ? rc : code_band_host(w, m, true, true);
}

// Exclusive GPU sections: the codec's device stages (pixel conversion, DWT,
// quantiser, records; dequantiser, inverse DWT) of concurrent codecs on one
// device run one at a time, each at full chip width, while the host coder
// threads overlap them.  Kernel timings stay uncontended.  RIC_GPU_SHARED=1
// lets sections of different codecs overlap instead.
std::mutex g_gpu_mu[64];
const bool g_gpu_shared = [] { const char* e = getenv("RIC_GPU_SHARED"); return e && atoi(e) != 0; }();

struct GpuSection {
	std::unique_lock<std::mutex> lk;
	explicit GpuSection(int device)
	{
		if (!g_gpu_shared) lk = std::unique_lock<std::mutex>(g_gpu_mu[device & 63]);
	}
};

int ensure_img(ric_wavelet* w)
{
	if (w->d_img) return RIC_OK;
	w->img_pitch = ((size_t)w->P.w + 63) / 64 * 64;
	HIPCHK(hipMalloc(&w->d_img, w->img_pitch * w->P.h * sizeof(int16_t)));
	return RIC_OK;
}

}  // namespace

namespace ric {
namespace wapi {

hipStream_t stream(ric_wavelet* w) { return w->st; }

int encode_plane(ric_wavelet* w, Mux& m, int16_t* plane, long stride, int trans, int quant, int lambda, int dq)
{
	if (set_dev(w->device)) return RIC_E_HIP;
	w->pend = false;
	int rc = encode_gpu(w, plane, stride, trans, quant, lambda);     // Transform + buildTree + records
	if (!rc) rc = code_band_host(w, m, true, true);                 // CodeBand's serial half + its band state
	if (!rc && m.overflow()) rc = RIC_E_CAPACITY;
	if (!rc) rc = tsuqi(w, dq);
	if (!rc) rc = inverse(w, plane, stride, trans);
	return rc;
}

int decode_plane(ric_wavelet* w, Mux& m, int16_t* plane, long stride, int trans, int dq)
{
	if (set_dev(w->device)) return RIC_E_HIP;
	w->pend = false;
	return decode_inverse_pipelined(w, m, plane, stride, trans, dq);
}

bool ll1(ric_wavelet* w, const int16_t** p, long* pitch, int* dx, int* dy)
{
	if (w->P.nlev < 2) return false;
	const Band& B = w->P.L[0].b[BL];
	if (B.is_int) return false;
	*p = (const int16_t*)(w->d_arena + B.off);
	*pitch = B.pitch;
	*dx = B.dx;
	*dy = B.dy;
	return true;
}

}  // namespace wapi
}  // namespace ric

extern "C" {

const char* ric_version(void) { return "rududu-image-codec_amd 0.1 (gfx950)"; }

int ric_device_count(void)
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess) return 0;
	return n;
}

const char* ric_last_error(void) { return g_err.c_str(); }

}  // extern "C"

void ric::set_last_error(const std::string& msg) { g_err = msg; }

extern "C" {

int ric_wavelet_create(ric_wavelet** out, int x, int y, int level, int level_chg, int device)
{
	if (!out || x < 8 || y < 8 || x > 65535 || y > 65535 || level < 1) return RIC_E_ARG;
	*out = nullptr;
	if (set_dev(device)) return RIC_E_HIP;
	ric_wavelet* w = new ric_wavelet;
	w->device = device;
	w->P.build(x, y, level, level_chg);
	w->P.set_weight(CDF97);
	// the memset runs on the object's own (non-blocking) stream: a null-stream
	// memset would not be ordered before this stream's copies and kernels
	if (hip_fail(hipMalloc(&w->d_arena, w->P.arena_bytes), "hipMalloc arena") ||
	    hip_fail(hipHostMalloc(&w->h_arena, w->P.arena_bytes, 0), "hipHostMalloc arena") ||
	    hip_fail(hipMalloc(&w->d_small, 64), "hipMalloc small") ||
	    hip_fail(hipHostMalloc(&w->h_small, 64, 0), "hipHostMalloc small") ||
	    hip_fail(hipStreamCreateWithFlags(&w->st, hipStreamNonBlocking), "hipStreamCreate") ||
	    hip_fail(hipMemsetAsync(w->d_arena, 0, w->P.arena_bytes, w->st), "hipMemset arena") ||
	    hip_fail(hipStreamSynchronize(w->st), "hipStreamSynchronize")) {
		ric_wavelet_destroy(w);
		return RIC_E_HIP;
	}
	memset(w->h_arena, 0, w->P.arena_bytes);
	w->own_stream = true;
	*out = w;
	return RIC_OK;
}

void ric_wavelet_destroy(ric_wavelet* w)
{
	if (!w) return;
	(void)hipSetDevice(w->device);
	if (w->st) (void)hipStreamSynchronize(w->st);
	w->prof.destroy();
	if (w->d_arena) (void)dev_free(w->d_arena);
	if (w->d_img) (void)dev_free(w->d_img);
	if (w->h_arena) (void)pinned_free(w->h_arena);
	if (w->d_small) (void)dev_free(w->d_small);
	if (w->h_small) (void)pinned_free(w->h_small);
	if (w->own_stream && w->st) (void)hipStreamDestroy(w->st);
	delete w;
}

int ric_wavelet_set_stream(ric_wavelet* w, void* s)
{
	if (!w) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	if (flush_pending(w)) return RIC_E_HIP;
	HIPCHK(hipStreamSynchronize(w->st));
	if (w->own_stream) (void)hipStreamDestroy(w->st);
	if (s) { w->st = (hipStream_t)s; w->own_stream = false; }
	else { HIPCHK(hipStreamCreateWithFlags(&w->st, hipStreamNonBlocking)); w->own_stream = true; }
	return RIC_OK;
}

int ric_wavelet_sync(ric_wavelet* w)
{
	if (!w) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	if (flush_pending(w)) return RIC_E_HIP;
	HIPCHK(hipStreamSynchronize(w->st));
	return RIC_OK;
}

int ric_set_weight(ric_wavelet* w, int trans, float base_weight)
{
	if (!w || trans < 0 || trans > 2) return RIC_E_ARG;
	w->P.set_weight(trans, base_weight);
	return RIC_OK;
}

int ric_transform(ric_wavelet* w, const int16_t* image, int stride, int trans, int on_device)
{
	if (!w || !image || stride < w->P.w || trans < 0 || trans > 2) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	if (!on_device) {
		int rc = ensure_img(w);
		if (rc) return rc;
		HIPCHK(hipMemcpy2DAsync(w->d_img, w->img_pitch * 2, image, (size_t)stride * 2, (size_t)w->P.w * 2,
		                        w->P.h, hipMemcpyHostToDevice, w->st));
		// deferred: a CodeBand next runs it fused with the quantiser (encode_gpu)
		w->pend = true;
		w->pend_trans = trans;
		w->host_valid = false;
		return RIC_OK;
	}
	w->pend = false;   // superseded: this transform rewrites every band
	return forward(w, image, stride, trans);
}

int ric_transform_inv(ric_wavelet* w, int16_t* image, int stride, int trans, int on_device)
{
	if (!w || !image || stride < w->P.w || trans < 0 || trans > 2) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	if (flush_pending(w)) return RIC_E_HIP;
	if (!on_device) {
		int rc = ensure_img(w);
		if (rc) return rc;
		rc = inverse(w, w->d_img, (long)w->img_pitch, trans);
		if (rc) return rc;
		HIPCHK(hipMemcpy2DAsync(image, (size_t)stride * 2, w->d_img, w->img_pitch * 2, (size_t)w->P.w * 2,
		                        w->P.h, hipMemcpyDeviceToHost, w->st));
		HIPCHK(hipStreamSynchronize(w->st));
		return RIC_OK;
	}
	return inverse(w, image, stride, trans);
}

int ric_code_band(ric_wavelet* w, ric_mux* m, int quant, int lambda)
{
	if (!w || !m || !m->encoder) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	int rc = code_band(w, m->m, quant, lambda);
	if (rc) return rc;
	return m->m.overflow() ? RIC_E_CAPACITY : RIC_OK;
}

int ric_quantize(ric_wavelet* w, int quant, int lambda)
{
	if (!w) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	int rc = w->pend ? encode_gpu(w, w->d_img, (long)w->img_pitch, w->pend_trans, quant, lambda)
	                 : quantize_gpu(w, quant, lambda);
	if (rc) return rc;
	HIPCHK(hipStreamSynchronize(w->st));
	return take_status(w, false);
}

int ric_transform_quantize(ric_wavelet* w, const int16_t* image, int stride, int trans, int on_device,
                           int quant, int lambda)
{
	if (!w || !image || stride < w->P.w || trans < 0 || trans > 2) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	w->pend = false;
	const int16_t* src = image;
	long sp = stride;
	if (!on_device) {
		int rc = ensure_img(w);
		if (rc) return rc;
		HIPCHK(hipMemcpy2DAsync(w->d_img, w->img_pitch * 2, image, (size_t)stride * 2, (size_t)w->P.w * 2,
		                        w->P.h, hipMemcpyHostToDevice, w->st));
		src = w->d_img; sp = (long)w->img_pitch;
	}
	int rc = encode_gpu(w, src, sp, trans, quant, lambda);
	if (rc) return rc;
	HIPCHK(hipStreamSynchronize(w->st));
	w->prof.harvest();
	return take_status(w, false);
}

int ric_decode_band(ric_wavelet* w, ric_mux* m)
{
	if (!w || !m || m->encoder) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	w->pend = false;   // every band is rewritten
	return decode_band(w, m->m);
}

// CWavelet2D::TSUQ (src/lib/wavelet2d.cpp:224-246): CBand::TSUQ on every band
// (band.h:65-92, Thres for the high bands, 0.5 for the LL); returns the count.
int ric_tsuq(ric_wavelet* w, int quant, float thres, unsigned int* count)
{
	if (!w) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	if (flush_pending(w)) return RIC_E_HIP;
	int rc = to_device(w);
	if (rc) return rc;
	unsigned int* d_count = (unsigned int*)w->d_small;
	HIPCHK(hipMemsetAsync(d_count, 0, sizeof(unsigned int), w->st));
	Pyramid& P = w->P;
	for (int i = 0; i < P.nbands(); i++) {
		const Band& B = P.band(i);
		const float th = i == 3 * P.nlev ? 0.5f : thres;
		int Q = (int)((float)quant / B.weight);
		if (Q == 0) Q = 1;
		const int iQ = (1 << 16) / Q;
		const int T0 = tr_any(!B.is_int, (int)(th * (float)Q));
		launch_tsuq_band(B, iQ, T0, w->d_arena, d_count, w->st);
	}
	unsigned int& h = *(unsigned int*)w->h_small;
	HIPCHK(hipMemcpyAsync(&h, d_count, sizeof(unsigned int), hipMemcpyDeviceToHost, w->st));
	HIPCHK(hipStreamSynchronize(w->st));
	if (count) *count = h;
	return RIC_OK;
}

int ric_tsuqi(ric_wavelet* w, int quant)
{
	if (!w) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	if (flush_pending(w)) return RIC_E_HIP;
	return tsuqi(w, quant);
}

// ---- one band on the device (CBand, src/lib/band.h:65-141).  Bands a caller
// wrote through pBand go to the device first; the host mirror is stale after.
namespace {
int band_begin(ric_wavelet* w, int index)
{
	if (!w || index < 0 || index >= w->P.nbands()) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	if (flush_pending(w)) return RIC_E_HIP;
	return to_device(w);
}
}  // namespace

int ric_band_tsuq(ric_wavelet* w, int index, int quant, float thres, unsigned int* count, int* max, int* min)
{
	int rc = band_begin(w, index);
	if (rc) return rc;
	const Band& B = w->P.band(index);
	// band.h:68-72: Quant = (int)(Quant / Weight), at least 1; T = (C)(Thres * Quant)
	int Q = (int)((float)quant / B.weight);
	if (Q == 0) Q = 1;
	const int iQ = (1 << 16) / Q;
	const int T0 = tr_any(!B.is_int, (int)(thres * (float)Q));
	int* d = (int*)w->d_small;
	int* h = (int*)w->h_small;
	HIPCHK(hipMemsetAsync(d, 0, 3 * sizeof(int), w->st));
	launch_band_tsuq(B, iQ, T0, w->d_arena, d, w->st);
	HIPCHK(hipGetLastError());
	HIPCHK(hipMemcpyAsync(h, d, 3 * sizeof(int), hipMemcpyDeviceToHost, w->st));
	HIPCHK(hipStreamSynchronize(w->st));
	w->host_valid = false;
	if (count) *count = (unsigned int)h[0];
	if (max) *max = h[1];
	if (min) *min = h[2];
	return RIC_OK;
}

int ric_band_tsuqi(ric_wavelet* w, int index, int quant)
{
	int rc = band_begin(w, index);
	if (rc) return rc;
	const Band& B = w->P.band(index);
	launch_dequant_band(B, tsuqi_factor(B, quant), w->d_arena, w->st);   // band.h:94-107
	HIPCHK(hipGetLastError());
	HIPCHK(hipStreamSynchronize(w->st));
	w->host_valid = false;
	return RIC_OK;
}

int ric_band_sums(ric_wavelet* w, int index, int64_t* sum, int64_t* ssum)
{
	int rc = band_begin(w, index);
	if (rc) return rc;
	unsigned long long* d = (unsigned long long*)w->d_small;
	unsigned long long* h = (unsigned long long*)w->h_small;
	HIPCHK(hipMemsetAsync(d, 0, 2 * sizeof(unsigned long long), w->st));
	launch_band_sums(w->P.band(index), w->d_arena, d, w->st);
	HIPCHK(hipGetLastError());
	HIPCHK(hipMemcpyAsync(h, d, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, w->st));
	HIPCHK(hipStreamSynchronize(w->st));
	if (sum) *sum = (int64_t)h[0];
	if (ssum) *ssum = (int64_t)h[1];
	return RIC_OK;
}

int ric_band_add(ric_wavelet* w, int index, int val)
{
	int rc = band_begin(w, index);
	if (rc) return rc;
	launch_band_add(w->P.band(index), val, w->d_arena, w->st);
	HIPCHK(hipGetLastError());
	HIPCHK(hipStreamSynchronize(w->st));
	w->host_valid = false;
	return RIC_OK;
}

int ric_band_clear(ric_wavelet* w, int index)
{
	int rc = band_begin(w, index);
	if (rc) return rc;
	const Band& B = w->P.band(index);
	HIPCHK(hipMemsetAsync(w->d_arena + B.off, 0, B.bytes(), w->st));
	HIPCHK(hipStreamSynchronize(w->st));
	w->host_valid = false;
	return RIC_OK;
}

int ric_band_count(ric_wavelet* w) { return w ? w->P.nbands() : RIC_E_ARG; }

int ric_band_info(ric_wavelet* w, int index, int* dimx, int* dimy, int* is_int, float* weight)
{
	if (!w || index < 0 || index >= w->P.nbands()) return RIC_E_ARG;
	const Band& B = w->P.band(index);
	if (dimx) *dimx = B.dx;
	if (dimy) *dimy = B.dy;
	if (is_int) *is_int = B.is_int;
	if (weight) *weight = B.weight;
	return RIC_OK;
}

int ric_band_read(ric_wavelet* w, int index, int32_t* out)
{
	if (!w || !out || index < 0 || index >= w->P.nbands()) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	if (flush_pending(w)) return RIC_E_HIP;
	const Band& B = w->P.band(index);
	if (!w->host_valid) {
		HIPCHK(hipMemcpyAsync(w->h_arena + B.off, w->d_arena + B.off, B.bytes(), hipMemcpyDeviceToHost, w->st));
		HIPCHK(hipStreamSynchronize(w->st));
	} else {
		ref_copy(w, true);
	}
	for (int y = 0; y < B.dy; y++)
		for (int x = 0; x < B.dx; x++) {
			size_t i = (size_t)y * B.pitch + x;
			out[(size_t)y * B.dx + x] = B.is_int ? ((int32_t*)(w->h_arena + B.off))[i] : ((int16_t*)(w->h_arena + B.off))[i];
		}
	return RIC_OK;
}

int ric_band_host(ric_wavelet* w, int index, void** ptr, int* pitch)
{
	if (!w || !ptr || index < 0 || index >= w->P.nbands()) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	if (flush_pending(w)) return RIC_E_HIP;
	if (!w->host_valid) {
		int rc = to_host(w, false);
		if (rc) return rc;
		w->host_valid = true;   // the mirror is authoritative until the next GPU stage
		ref_copy(w, false);
	} else {
		ref_copy(w, true);
	}
	const Band& B = w->P.band(index);
	*ptr = w->h_arena + B.off;
	if (pitch) *pitch = B.pitch;
	return RIC_OK;
}

int ric_band_host_ref(ric_wavelet* w, int index, void** ptr, int* stride)
{
	if (!w || !ptr || index < 0 || index >= w->P.nbands()) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	if (flush_pending(w)) return RIC_E_HIP;
	if ((int)w->ref_buf.size() < w->P.nbands()) {
		w->ref_buf.resize(w->P.nbands());
		w->ref_active.resize(w->P.nbands(), 0);
	}
	if (!w->host_valid) {
		int rc = to_host(w, false);
		if (rc) return rc;
		w->host_valid = true;
	} else {
		ref_copy(w, true);              // other views' writes first
	}
	const Band& B = w->P.band(index);
	const int rs = ref_stride(B);
	auto& buf = w->ref_buf[index];
	if (buf.empty()) buf.assign((size_t)rs * B.dy * (B.is_int ? 4 : 2) + 32, 0);
	w->ref_active[index] = 1;
	ref_copy(w, false);
	*ptr = buf.data();
	if (stride) *stride = rs;
	return RIC_OK;
}

int ric_band_write(ric_wavelet* w, int index, const int32_t* in)
{
	if (!w || !in || index < 0 || index >= w->P.nbands()) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	if (flush_pending(w)) return RIC_E_HIP;
	int rc = to_device(w);
	if (rc) return rc;
	const Band& B = w->P.band(index);
	HIPCHK(hipStreamSynchronize(w->st));
	for (int y = 0; y < B.dy; y++)
		for (int x = 0; x < B.dx; x++) {
			size_t i = (size_t)y * B.pitch + x;
			int32_t v = in[(size_t)y * B.dx + x];
			if (B.is_int) ((int32_t*)(w->h_arena + B.off))[i] = v;
			else ((int16_t*)(w->h_arena + B.off))[i] = (int16_t)v;
		}
	HIPCHK(hipMemcpyAsync(w->d_arena + B.off, w->h_arena + B.off, B.bytes(), hipMemcpyHostToDevice, w->st));
	HIPCHK(hipStreamSynchronize(w->st));
	return RIC_OK;
}

int ric_mux_create_encoder(ric_mux** out, uint8_t* buf, size_t cap, uint16_t first_word)
{
	if (!out) return RIC_E_ARG;
	ric_mux* m = new ric_mux;
	m->encoder = true;
	m->buf = buf;
	// CMuxCodec(0, 0) (src/lib/rududucodec.cpp:36): no buffer until initCoder;
	// coding before that is flagged (capacity 0) instead of writing anywhere
	m->m.init_encoder(buf, buf ? cap : 0, first_word);
	*out = m;
	return RIC_OK;
}

int ric_mux_reinit_encoder(ric_mux* m, uint8_t* buf, size_t cap, uint16_t first_word)
{
	if (!m) return RIC_E_ARG;
	m->encoder = true;
	if (buf) m->buf = buf;
	m->m.reinit_encoder(buf, cap, first_word);
	return RIC_OK;
}

int ric_mux_reinit_decoder(ric_mux* m, const uint8_t* buf, size_t len)
{
	if (!m || (buf && len != 0 && len < 4)) return RIC_E_ARG;
	m->encoder = false;
	if (buf) m->buf = const_cast<uint8_t*>(buf);
	m->m.reinit_decoder(buf, len);
	return RIC_OK;
}

int ric_mux_create_decoder(ric_mux** out, const uint8_t* buf, size_t len)
{
	if (!out || !buf || len < 4) return RIC_E_ARG;
	ric_mux* m = new ric_mux;
	m->encoder = false;
	m->m.init_decoder(buf, len);
	*out = m;
	return RIC_OK;
}

int ric_mux_create_decoder_inplace(ric_mux** out, const uint8_t* buf)
{
	if (!out || !buf) return RIC_E_ARG;
	ric_mux* m = new ric_mux;
	m->encoder = false;
	m->m.init_decoder_inplace(buf);
	*out = m;
	return RIC_OK;
}

int ric_mux_end(ric_mux* m, size_t* len_out)
{
	if (!m || !m->encoder) return RIC_E_ARG;
	if (!m->buf) return RIC_E_ARG;                 // CMuxCodec(0, 0) never given a buffer
	uint8_t* e = m->m.end_coding();
	if (len_out) *len_out = (size_t)(e - m->buf);
	return m->m.overflow() ? RIC_E_CAPACITY : RIC_OK;
}

size_t ric_mux_size(ric_mux* m) { return m ? m->m.size() : 0; }

void ric_mux_destroy(ric_mux* m) { delete m; }

int ric_quants(int idx)
{
	static const unsigned short Q[5] = {0x8000, 0x9000, 0xA800, 0xC000, 0xE000};
	if (idx <= 0) return 0;
	idx--;
	int r = 14 - idx / 5;
	return (short)((Q[idx % 5] + (1 << (r - 1))) >> r);
}

int ric_read_header(const uint8_t* ric, size_t len, int* w, int* h, int* channels, int* q, int* trans)
{
	if (!ric || len < 9) return RIC_E_ARG;
	if (memcmp(ric, "RUD2", 4) != 0) return RIC_E_FORMAT;
	if (w) *w = ric[4] | (ric[5] << 8);
	if (h) *h = ric[6] | (ric[7] << 8);
	if (q) *q = ric[8] & 31;
	if (channels) *channels = ((ric[8] >> 5) & 1) ? 3 : 1;
	if (trans) *trans = (ric[8] >> 6) & 3;
	return RIC_OK;
}

int ric_codec_create(ric_codec** out, int w, int h, int channels, int device)
{
	if (!out || (channels != 1 && channels != 3)) return RIC_E_ARG;
	*out = nullptr;
	ric_codec* c = new ric_codec;
	c->device = device; c->w = w; c->h = h; c->channels = channels;
	int rc = ric_wavelet_create(&c->wav, w, h, 5, 1, device);   // WAV_LEVELS 5, level_chg 1 (ric.cpp:159)
	if (rc) { delete c; return rc; }
	c->pitch = ((long)w + 63) / 64 * 64;
	if (hip_fail(hipMalloc(&c->d_planes, (size_t)c->pitch * h * channels * 2), "hipMalloc planes") ||
	    hip_fail(hipMalloc(&c->d_pix, (size_t)w * h * channels), "hipMalloc pix") ||
	    hip_fail(hipMalloc(&c->d_out, (size_t)w * h * channels * 2), "hipMalloc out")) {
		ric_codec_destroy(c);
		return RIC_E_HIP;
	}
	c->stream.resize((size_t)w * h * channels * 2 + 65536);
	c->dstream.resize((size_t)w * h * channels + 2 + 16);
	*out = c;
	return RIC_OK;
}

void ric_codec_destroy(ric_codec* c)
{
	if (!c) return;
	(void)hipSetDevice(c->device);
	if (c->wav) ric_wavelet_destroy(c->wav);
	if (c->d_planes) (void)dev_free(c->d_planes);
	if (c->d_pix) (void)dev_free(c->d_pix);
	if (c->d_out) (void)dev_free(c->d_out);
	delete c;
}

int ric_codec_set_stream(ric_codec* c, void* s) { return c ? ric_wavelet_set_stream(c->wav, s) : RIC_E_ARG; }

int ric_wavelet_set_host_threads(ric_wavelet* w, int n)
{
	if (!w || n < 1 || n > 64) return RIC_E_ARG;
	w->pool.reset();
	w->host_threads = n;
	if (n > 1) w->pool.reset(new Pool(n - 1));
	return RIC_OK;
}

int ric_codec_set_host_threads(ric_codec* c, int n) { return c ? ric_wavelet_set_host_threads(c->wav, n) : RIC_E_ARG; }

// CompressImage, src/ric/ric.cpp:123-180
int ric_codec_encode(ric_codec* c, const uint8_t* pix, int on_device, int q, int trans,
                     uint8_t* out, size_t cap, size_t* len_out)
{
	if (!c || !pix || !out || q < 0 || q > 31 || trans < 0 || trans > 2) return RIC_E_ARG;
	if (set_dev(c->device)) return RIC_E_HIP;
	ric_wavelet* w = c->wav;
	const size_t npix = (size_t)c->w * c->h * c->channels;
	const uint8_t* dpix = pix;
	if (!on_device) {
		HIPCHK(hipMemcpyAsync(c->d_pix, pix, npix, hipMemcpyHostToDevice, w->st));
		dpix = c->d_pix;
	}
	Mux m;
	m.init_encoder(c->stream.data(), c->stream.size(), 0);
	w->P.set_weight(trans);
	const long plane = c->pitch * c->h;
	for (int p = 0; p < c->channels; p++) {
		const int boost = p ? 8 : 0;                // C_Q_BOOST for chroma (ric.cpp:164-168)
		{
			GpuSection gs(c->device);
			if (p == 0) {
				w->prof.begin(S_PIXIN, w->st);
				launch_pix_in(dpix, c->d_planes, c->w, c->h, c->pitch, c->channels, q, w->st);
				w->prof.end(S_PIXIN, w->st);
				HIPCHK(hipGetLastError());
			}
			int rc = encode_gpu(w, c->d_planes + p * plane, c->pitch, trans,
			                    q ? ric_quants(q + 20 + boost) : 0, q ? ric_quants(q + 13 + boost) : 0, true);
			if (rc) return rc;
			// the copy runs inside the section too: its blit kernels would
			// otherwise share the CUs with another codec's level kernels
			rc = to_host(w, true);
			if (rc) return rc;
		}
		int rc = code_band_host(w, m, false);
		if (rc) return rc;
	}
	uint8_t* e = m.end_coding();
	if (m.overflow()) return RIC_E_CAPACITY;
	const size_t len = (size_t)(e - c->stream.data());
	const size_t total = 9 + len - 2;
	if (len_out) *len_out = total;
	if (total > cap) return RIC_E_CAPACITY;
	memcpy(out, "RUD2", 4);
	out[4] = c->w & 255; out[5] = (c->w >> 8) & 255; out[6] = c->h & 255; out[7] = (c->h >> 8) & 255;
	out[8] = (uint8_t)((q & 31) | ((c->channels == 3) << 5) | ((trans & 3) << 6));
	memcpy(out + 9, c->stream.data() + 2, len - 2);
	return RIC_OK;
}

// DecompressImage, src/ric/ric.cpp:182-251
int ric_codec_decode(ric_codec* c, const uint8_t* ric, size_t len, int dither,
                     uint8_t* pix_out, int16_t* planes_out, int on_device)
{
	if (!c || !ric) return RIC_E_ARG;
	int w_, h_, ch, q, trans;
	int rc = ric_read_header(ric, len, &w_, &h_, &ch, &q, &trans);
	if (rc) return rc;
	if (w_ != c->w || h_ != c->h || ch != c->channels || trans > 2) return RIC_E_ARG;
	if (set_dev(c->device)) return RIC_E_HIP;
	ric_wavelet* w = c->wav;
	// the reference reads W*H*C payload bytes at buf + 2 (ric.cpp:203-205)
	const size_t npix = (size_t)c->w * c->h * c->channels;
	const size_t pay = std::min(len - 9, npix);
	// (the decoder's look-ahead past the end reads zeros: 16 zeroed tail bytes)
	if (c->dstream.size() < pay + 2 + 16) c->dstream.resize(pay + 2 + 16);
	uint8_t* buf = c->dstream.data();
	buf[0] = buf[1] = 0;
	memcpy(buf + 2, ric + 9, pay);
	memset(buf + 2 + pay, 0, 16);
	Mux m;
	m.init_decoder(buf, pay + 2);
	w->P.set_weight(trans);
	const long plane = c->pitch * c->h;
	int stream_rc = RIC_OK;
	for (int p = 0; p < c->channels; p++) {
		const int boost = p ? 8 : 0;
		rc = decode_inverse_pipelined(w, m, c->d_planes + p * plane, c->pitch, trans, q ? ric_quants(q + 20 + boost) : 0);
		if (rc && rc != RIC_E_STREAM) return rc;
		if (rc) stream_rc = rc;
	}
	(void)stream_rc;
	if (dither && q && c->channels == 1) {
		// dither() is a serial error diffusion (src/ric/ric.cpp:51-74): host side
		std::vector<int16_t> img((size_t)c->w * c->h);
		HIPCHK(hipMemcpy2DAsync(img.data(), (size_t)c->w * 2, c->d_planes, (size_t)c->pitch * 2, (size_t)c->w * 2,
		                        c->h, hipMemcpyDeviceToHost, w->st));
		HIPCHK(hipStreamSynchronize(w->st));
		auto clip = [](int v) { return (int16_t)(v < 0 ? 0 : v > 255 ? 255 : v); };
		int16_t* pi = img.data();
		const int W = c->w, H = c->h;
		for (int j = 0; j < H - 1; j++) {
			pi[0] = clip(128 + ((pi[0] + 8) >> 4));
			for (int i = 1; i < W - 1; i++) {
				int16_t tmp = (int16_t)(pi[i] + 8);
				pi[i] = (int16_t)(tmp >> 4);
				tmp = (int16_t)(tmp - (pi[i] << 4));
				pi[i + 1] += (int16_t)((tmp >> 1) - (tmp >> 4));
				pi[i + W - 1] += (int16_t)((tmp >> 3) + (tmp >> 4));
				pi[i + W] += (int16_t)((tmp >> 2) + (tmp >> 4));
				pi[i + W + 1] += (int16_t)(tmp >> 4);
				pi[i] = clip(pi[i] + 128);
			}
			pi += W;
			pi[-1] = clip(128 + ((pi[-1] + 8) >> 4));
		}
		for (int i = 0; i < W; i++) pi[i] = clip(128 + ((pi[i] + 8) >> 4));
		std::vector<uint8_t> px(img.size());
		for (size_t i = 0; i < img.size(); i++) px[i] = (uint8_t)img[i];
		if (on_device) {
			if (pix_out) HIPCHK(hipMemcpyAsync(pix_out, px.data(), px.size(), hipMemcpyHostToDevice, w->st));
			if (planes_out) HIPCHK(hipMemcpyAsync(planes_out, img.data(), img.size() * 2, hipMemcpyHostToDevice, w->st));
			HIPCHK(hipStreamSynchronize(w->st));
		} else {
			if (pix_out) memcpy(pix_out, px.data(), px.size());
			if (planes_out) memcpy(planes_out, img.data(), img.size() * 2);
		}
		return m.overflow() ? RIC_E_STREAM : RIC_OK;
	}
	uint8_t* dpix = on_device ? pix_out : (pix_out ? c->d_pix : nullptr);
	int16_t* dpl = on_device ? planes_out : (planes_out ? c->d_out : nullptr);
	{
		GpuSection gs(c->device);
		w->prof.begin(S_PIXOUT, w->st);
		launch_pix_out(c->d_planes, c->pitch, c->w, c->h, c->channels, q, dpix, dpl, w->st);
		w->prof.end(S_PIXOUT, w->st);
		HIPCHK(hipGetLastError());
		HIPCHK(hipStreamSynchronize(w->st));
	}
	if (!on_device) {
		if (pix_out) HIPCHK(hipMemcpyAsync(pix_out, c->d_pix, npix, hipMemcpyDeviceToHost, w->st));
		if (planes_out) HIPCHK(hipMemcpyAsync(planes_out, c->d_out, npix * 2, hipMemcpyDeviceToHost, w->st));
	}
	HIPCHK(hipStreamSynchronize(w->st));
	w->prof.harvest();
	return m.overflow() ? RIC_E_STREAM : RIC_OK;
}

int ric_prof_enable(ric_wavelet* w, int on)
{
	if (!w) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	w->prof.enable(on != 0);
	w->prof.reset();
	return RIC_OK;
}

int ric_prof_read(ric_wavelet* w, double* ms, long* counts, int n)
{
	if (!w || !ms || !counts) return RIC_E_ARG;
	if (set_dev(w->device)) return RIC_E_HIP;
	HIPCHK(hipStreamSynchronize(w->st));
	w->prof.harvest();
	for (int i = 0; i < n && i < S_COUNT; i++) { ms[i] = w->prof.ms[i]; counts[i] = w->prof.n[i]; }
	return S_COUNT;
}

ric_wavelet* ric_codec_wavelet(ric_codec* c) { return c ? c->wav : nullptr; }

int ric_diag_wgtrace(int device, uint64_t* out, int n)
{
	if (!out || n < 0) return RIC_E_ARG;
	const int r = diag_wgtrace(device, out, n);
	return r < 0 ? RIC_E_HIP : r;
}

long ric_diag_deferred_frees(void) { return deferred_frees(); }

int ric_diag_fault(int on)
{
	diag_set_fault(on);
	return RIC_OK;
}

// SURVEY.md §8(d) synthetic generator (integer-only, bit-reproducible)
void ric_synth_image(int w, int h, int channels, int frame, uint8_t* out)
{
	for (int c = 0; c < channels; c++) {
		uint32_t s = 0x9E3779B9u + 0x1000u * (uint32_t)frame + (uint32_t)c;
		const int phase = 32 * c;
		uint8_t* o = out + (size_t)c * w * h;
		for (int y = 0; y < h; y++) {
			const int gy = (y * 255) / (h - 1);
			for (int x = 0; x < w; x++) {
				s ^= s << 13; s ^= s >> 17; s ^= s << 5;
				const int noise = (int)(s >> 28) - 8;
				const int grad = ((x * 255) / (w - 1) + gy) >> 2;
				int t = (x + 2 * y + phase) & 127;
				t = t < 64 ? t : 127 - t;
				const int v = grad + t + noise + 32;
				*o++ = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
			}
		}
	}
}

}  // extern "C"
