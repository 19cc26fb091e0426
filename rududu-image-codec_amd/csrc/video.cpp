// video.cpp -- the reference video codec, CRududuCodec (src/lib/rududucodec.cpp),
// over HBM: the C-ABI ric_video_* (include/ric_gpu.h).
//
// The data-parallel stages are HIP kernels (motion.hip): pixel input, the
// quarter-pel planes (CImageBuffer::calc_sub), the EPZS motion search, OBMC and
// the frame add / subtract; the wavelet closed loop runs on the .ric path's
// kernels (capi.cpp wapi).  The serial stages stay on the host: the
// motion-vector coder (COBMC::encode / decode with the adaptive CHuffCodec,
// entropy.cpp mv_encode / mv_decode) and the band coder, both into the one
// CMuxCodec stream of the frame.
//
// Behaviour kept from the reference on purpose:
//   * the image pool: CImageBuffer's stack of free images, its allocation
//     order and reuse (imagebuffer.cpp:27-121) -- the quarter-pel pass reads a
//     sample past each edge of images whose borders hold whatever their last
//     use left there, so which buffer serves which image is part of the output;
//   * CImage's memory layout (image.cpp:56-68) and TransformI's samples left in
//     the border (motion.h);
//   * the encoder's reconstruction: TSUQi after CodeBand acts on the bands in
//     CodeBand's sign-magnitude state (rududucodec.cpp:71-73), so encoder and
//     decoder reconstructions differ, frame after frame, as in the reference;
//   * the ILP32 meaning of the reference's unsigned "negative" indices (the
//     row above in the vector field, the column left of the image).
// One change: TransformI is given each plane's END pointer (its contract
// since ric_0.2); rududucodec.cpp:74,83 pass the start and crash.
#include <hip/hip_runtime.h>

#include <array>
#include <cstring>
#include <string>
#include <vector>

#include "ric_gpu.h"
#include "entropy.h"
#include "codec_params.h"
#include "motion.h"
#include "wavelet_api.h"

using namespace ric;

namespace {

constexpr int kVidLevels = 3;                 // WAV_LEVELS (rududucodec.cpp:26)
constexpr int kVidTrans = RIC_CDF97;          // TRANSFORM (:27)
constexpr int kBufferSize = 16 + 1;           // BUFFER_SIZE = SUB_IMAGE_CNT + 1 (:28)

// CRududuCodec::quants (rududucodec.cpp:58-65)
int vquants(int idx)
{
	static const unsigned short Q[5] = {32768, 37641, 43238, 49667, 57052};
	if (idx == 0) return 0;
	idx--;
	const int r = 10 - idx / 5;
	return (short)((Q[idx % 5] + (1 << (r - 1))) >> r);
}

bool vfail(hipError_t e, const char* what)
{
	if (e == hipSuccess) return false;
	set_last_error(std::string(what) + ": " + hipGetErrorString(e));
	return true;
}
#define VCHK(x) do { if (vfail((x), #x)) return RIC_E_HIP; } while (0)

}  // namespace

struct ric_video {
	int device = 0;
	bool encoder = true;
	int quant = 0;
	VidGeom g;
	ric_wavelet* wav = nullptr;
	hipStream_t st = nullptr;
	Mux mux;                                   // the codec's one CMuxCodec (rududucodec.cpp:36)
	// CImageBuffer (imagebuffer.h:36-53): images by id
	std::vector<int16_t*> bufs;                // allocation starts
	std::vector<std::array<int, 16>> list;     // image_list: sub-image ids, -1 = none
	std::vector<int> free_stack;
	int images_left = kBufferSize - 1;
	int16_t* pred = nullptr;                   // predImage (its allocation start)
	uint32_t* d_mv = nullptr;                  // the motion field (COBMC::pMV), persistent
	uint16_t* d_dist = nullptr;
	uint64_t* d_gran = nullptr;                // EPZS hand-off granules (motion.h)
	uint32_t epoch = 0;                        // the last EPZS search's tag
	uint32_t* d_status = nullptr;
	uint8_t* d_rgb = nullptr;
	size_t rgb_cap = 0;
	std::vector<uint32_t> mv;                  // host copy of the field
	int key_count = 0;
	int out_id = -1;                           // *outImage of the last call
	bool has_mv = false;

	int16_t* img(int id) const { return bufs[id] + g.origin(); }
	int16_t* pred_img() const { return pred + g.origin(); }

	// kImgSlack samples of allocated slack before and after every image: the
	// OBMC kernel stages window rows with aligned 16-byte loads that reach up
	// to 16 bytes past a row clamped to the image's first or last sample
	static constexpr size_t kImgSlack = 128;
	int alloc_image(int16_t** out)
	{
		const size_t bytes = (g.image_samples() + 2 * kImgSlack) * sizeof(int16_t);
		int16_t* raw = nullptr;
		VCHK(hipMalloc(&raw, bytes));
		*out = raw + kImgSlack;
		VCHK(hipMemsetAsync(raw, 0, bytes, st));      // a fresh CImage reads as zeros (see oracle/ref_video.cpp)
		return RIC_OK;
	}
	static void free_image(int16_t* p) { if (p) (void)dev_free(p - kImgSlack); }
	// CImageBuffer::getFree (imagebuffer.cpp:44-61)
	int get_free(int* id)
	{
		if (!free_stack.empty()) {
			*id = free_stack.back();
			free_stack.pop_back();
			return RIC_OK;
		}
		if (images_left > 0) {
			int16_t* p = nullptr;
			int rc = alloc_image(&p);
			if (rc) return rc;
			images_left--;
			bufs.push_back(p);
			*id = (int)bufs.size() - 1;
			return RIC_OK;
		}
		set_last_error("video image pool exhausted");
		return RIC_E_ARG;
	}
	// insert(0) (imagebuffer.cpp:68-78)
	int insert0()
	{
		int id = -1;
		int rc = get_free(&id);
		if (rc) return rc;
		std::array<int, 16> e;
		e.fill(-1);
		e[0] = id;
		list.insert(list.begin(), e);
		return RIC_OK;
	}
	// remove(index) (imagebuffer.cpp:80-88)
	void remove(size_t index)
	{
		if (index >= list.size()) return;
		for (int k = 0; k < 16; k++)
			if (list[index][k] >= 0) free_stack.push_back(list[index][k]);
		list.erase(list.begin() + index);
	}
	// calc_sub(index) (imagebuffer.cpp:90-121): the sub-images are taken in
	// the reference's order, then interpolated and extended on the GPU
	int calc_sub(size_t index)
	{
		static const int order[15] = {4, 8, 12, 1, 2, 3, 5, 6, 7, 9, 10, 11, 13, 14, 15};
		for (int k : order)
			if (list[index][k] < 0) {
				int id = -1;
				int rc = get_free(&id);
				if (rc) return rc;
				list[index][k] = id;
			}
		VidSubs s;
		for (int k = 0; k < 16; k++) s.p[k] = img(list[index][k]);
		if (launch_vid_interp(g, s, st) || launch_vid_extend(g, s, 16, st)) return vfail(hipGetLastError(), "calc_sub"), RIC_E_HIP;
		return RIC_OK;
	}
	VidSubs subs(size_t index) const
	{
		VidSubs s;
		for (int k = 0; k < 16; k++) s.p[k] = list[index][k] >= 0 ? img(list[index][k]) : nullptr;
		return s;
	}
	// TransformI's level-1 output left around the plane (motion.h)
	int tinv_side(int16_t* plane)
	{
		const int16_t* p = nullptr;
		long pitch = 0;
		int dx = 0, dy = 0;
		if (!wapi::ll1(wav, &p, &pitch, &dx, &dy)) return RIC_OK;
		return launch_vid_tinv_side(g, plane, p, pitch, dx, dy, st) ? RIC_E_HIP : RIC_OK;
	}
	// encodeImage (rududucodec.cpp:67-76)
	int encode_image(int id)
	{
		for (int c = 0; c < 3; c++) {
			int16_t* plane = img(id) + c * g.P;
			int rc = wapi::encode_plane(wav, mux, plane, g.S, kVidTrans, vquants(quant + 20), vquants(quant + 12),
			                            vquants(quant + 20));
			if (!rc) rc = tinv_side(plane);
			if (rc) return rc;
		}
		return RIC_OK;
	}
	// decodeImage (rududucodec.cpp:78-85)
	int decode_image(int id)
	{
		int result = RIC_OK;
		for (int c = 0; c < 3; c++) {
			int16_t* plane = img(id) + c * g.P;
			int rc = wapi::decode_plane(wav, mux, plane, g.S, kVidTrans, vquants(quant + 20));
			if (rc == RIC_E_STREAM) result = RIC_E_STREAM;
			else if (rc) return rc;
			rc = tinv_side(plane);
			if (rc) return rc;
		}
		return result;
	}
	int sync_status()
	{
		uint32_t s = 0;
		VCHK(hipMemcpyAsync(&s, d_status, sizeof(s), hipMemcpyDeviceToHost, st));
		VCHK(hipStreamSynchronize(st));
		if (s) {
			VCHK(hipMemsetAsync(d_status, 0, sizeof(uint32_t), st));
			set_last_error("EPZS wavefront: a block row waited too long for the row above (device status set)");
			return RIC_E_HIP;
		}
		return RIC_OK;
	}
};

extern "C" {

int ric_video_create(ric_video** out, int encoder, int w, int h, int component, int device)
{
	if (!out || w < 16 || h < 16 || w > 32767 || h > 32767 || component != 3) return RIC_E_ARG;
	*out = nullptr;
	if (vfail(hipSetDevice(device), "hipSetDevice")) return RIC_E_HIP;
	ric_video* v = new ric_video;
	v->device = device;
	v->encoder = encoder != 0;
	v->g.init(w, h);
	// CWavelet2D(width, height, WAV_LEVELS), SetWeight(TRANSFORM) (rududucodec.cpp:39-40)
	int rc = ric_wavelet_create(&v->wav, w, h, kVidLevels, 0, device);
	if (!rc) rc = ric_set_weight(v->wav, kVidTrans, 1.f);
	if (rc) { ric_video_destroy(v); return rc; }
	v->st = wapi::stream(v->wav);
	v->mux.init_encoder(nullptr, 0, 0);                    // CMuxCodec codec(0, 0)
	const size_t nb = (size_t)v->g.bx * v->g.by;
	v->mv.assign(nb, 0);
	int16_t* first = nullptr;
	if (v->alloc_image(&first) || v->alloc_image(&v->pred) ||
	    vfail(hipMalloc(&v->d_mv, sizeof(uint32_t) * (nb + 1)), "hipMalloc") ||
	    vfail(hipMalloc(&v->d_dist, sizeof(uint16_t) * (nb + 1)), "hipMalloc") ||
	    vfail(hipMalloc(&v->d_gran, sizeof(uint64_t) * (nb + 1)), "hipMalloc") ||
	    vfail(hipMemsetAsync(v->d_gran, 0, sizeof(uint64_t) * (nb + 1), v->st), "hipMemset") ||
	    vfail(hipMalloc(&v->d_status, sizeof(uint32_t)), "hipMalloc") ||
	    vfail(hipMemsetAsync(v->d_mv, 0, sizeof(uint32_t) * (nb + 1), v->st), "hipMemset") ||   // COBMC: memset 0 (obmc.cpp:44-45)
	    vfail(hipMemsetAsync(v->d_status, 0, sizeof(uint32_t), v->st), "hipMemset") ||
	    vfail(hipStreamSynchronize(v->st), "hipStreamSynchronize")) {
		ric_video_destroy(v);
		return RIC_E_HIP;
	}
	// CImageBuffer's constructor: one image on the free stack (imagebuffer.cpp:27-32)
	v->bufs.push_back(first);
	v->free_stack.push_back(0);
	*out = v;
	return RIC_OK;
}

void ric_video_destroy(ric_video* v)
{
	if (!v) return;
	(void)hipSetDevice(v->device);
	if (v->st) (void)hipStreamSynchronize(v->st);
	for (int16_t* p : v->bufs) ric_video::free_image(p);
	ric_video::free_image(v->pred);
	if (v->d_mv) (void)dev_free(v->d_mv);
	if (v->d_dist) (void)dev_free(v->d_dist);
	if (v->d_gran) (void)dev_free(v->d_gran);
	if (v->d_status) (void)dev_free(v->d_status);
	if (v->d_rgb) (void)dev_free(v->d_rgb);
	if (v->wav) ric_wavelet_destroy(v->wav);
	delete v;
}

int ric_video_set_host_threads(ric_video* v, int n) { return v ? ric_wavelet_set_host_threads(v->wav, n) : RIC_E_ARG; }

int ric_video_set_quant(ric_video* v, int quant)
{
	// quants(quant + 12) .. quants(quant + 20) must stay inside the table's
	// defined range (rududucodec.cpp:58-65: idx >= 0, shift r >= 1)
	if (!v || quant < -12 || quant > 30) return RIC_E_ARG;
	v->quant = quant;
	return RIC_OK;
}

int ric_video_encode(ric_video* v, const uint8_t* pix, int stride, int pix_on_device, uint8_t* buf, size_t cap, int* size)
{
	if (!v || !pix || !buf || !size || !v->encoder || stride < v->g.w || cap < 16) return RIC_E_ARG;
	if (vfail(hipSetDevice(v->device), "hipSetDevice")) return RIC_E_HIP;
	const VidGeom& g = v->g;
	v->mux.reinit_encoder(buf, cap, 0);                    // codec.initCoder(0, pBuffer) (:89)
	int rc = v->insert0();                                 // images.insert(0) (:91)
	if (rc) return rc;
	const int cur = v->list[0][0];
	// images[0][0]->inputSGI(pImage, stride, -128) (:92)
	const uint8_t* src = pix;
	if (!pix_on_device) {
		const size_t n = (size_t)stride * g.h * 3;
		if (v->rgb_cap < n) {
			if (v->d_rgb) VCHK(dev_free(v->d_rgb));
			VCHK(hipMalloc(&v->d_rgb, n));
			v->rgb_cap = n;
		}
		VCHK(hipMemcpyAsync(v->d_rgb, pix, n, hipMemcpyHostToDevice, v->st));
		src = v->d_rgb;
	}
	if (launch_vid_input(g, src, stride, v->img(cur), v->st)) return vfail(hipGetLastError(), "k_vid_input"), RIC_E_HIP;
	if (v->key_count != 0) {                               // an inter frame (:94-105)
		rc = v->calc_sub(1);
		if (rc) return rc;
		const VidSubs ref = v->subs(1);
		if (++v->epoch == 0) {                             // tags wrapped: clear the granules
			VCHK(hipMemsetAsync(v->d_gran, 0, sizeof(uint64_t) * v->mv.size(), v->st));
			v->epoch = 1;
		}
		if (launch_vid_epzs(g, v->img(cur), ref, v->d_mv, v->d_dist, v->d_gran, v->epoch, v->d_status, v->st))
			return vfail(hipGetLastError(), "k_vid_epzs"), RIC_E_HIP;
		VCHK(hipMemcpyAsync(v->mv.data(), v->d_mv, sizeof(uint32_t) * v->mv.size(), hipMemcpyDeviceToHost, v->st));
		rc = v->sync_status();
		if (rc) return rc;
		mv_encode(v->mux, v->mv.data(), g.bx, g.by);       // obme->encode(&codec)
		if (launch_vid_obmc(g, v->d_mv, ref, v->pred_img(), v->img(cur), v->st))   // apply_mv, then *im -= *pred
			return vfail(hipGetLastError(), "k_vid_obmc"), RIC_E_HIP;
		rc = v->encode_image(cur);
		if (rc) return rc;
		if (launch_vid_addsub(g, v->img(cur), v->pred_img(), +1, v->st)) return vfail(hipGetLastError(), "k_vid_addsub"), RIC_E_HIP;
		buf[0] |= 0x80;
		v->has_mv = true;
	} else {
		rc = v->encode_image(cur);
		if (rc) return rc;
	}
	if (++v->key_count == 10) v->key_count = 0;            // (:110-112)
	v->out_id = cur;
	v->remove(1);
	VCHK(hipStreamSynchronize(v->st));
	uint8_t* end = v->mux.end_coding();
	if (v->mux.overflow()) {
		set_last_error("ric_video_encode: stream larger than the buffer");
		return RIC_E_CAPACITY;
	}
	*size = (int)(end - buf - 2);                          // codec.endCoding() - pBuffer - 2 (:118)
	return RIC_OK;
}

int ric_video_decode(ric_video* v, const uint8_t* buf, size_t len, int* size)
{
	if (!v || !buf || !size || (len != 0 && len < 4)) return RIC_E_ARG;
	if (vfail(hipSetDevice(v->device), "hipSetDevice")) return RIC_E_HIP;
	const VidGeom& g = v->g;
	v->mux.reinit_decoder(buf, len);                       // codec.initDecoder(pBuffer) (:123)
	int rc = v->insert0();
	if (rc) return rc;
	const int cur = v->list[0][0];
	int result = RIC_OK;
	if (buf[0] & 0x80) {                                   // (:127-133)
		rc = v->calc_sub(1);
		if (rc) return rc;
		mv_decode(v->mux, v->mv.data(), g.bx, g.by);       // obmc->decode(&codec)
		VCHK(hipMemcpyAsync(v->d_mv, v->mv.data(), sizeof(uint32_t) * v->mv.size(), hipMemcpyHostToDevice, v->st));
		if (launch_vid_obmc(g, v->d_mv, v->subs(1), v->pred_img(), nullptr, v->st)) return vfail(hipGetLastError(), "k_vid_obmc"), RIC_E_HIP;
		result = v->decode_image(cur);
		if (result && result != RIC_E_STREAM) return result;
		if (launch_vid_addsub(g, v->img(cur), v->pred_img(), +1, v->st)) return vfail(hipGetLastError(), "k_vid_addsub"), RIC_E_HIP;
		v->has_mv = true;
	} else {
		result = v->decode_image(cur);
		if (result && result != RIC_E_STREAM) return result;
	}
	v->out_id = cur;
	v->remove(1);
	VCHK(hipStreamSynchronize(v->st));
	*size = (int)v->mux.size();                            // codec.getSize() (:140)
	return v->mux.overflow() ? RIC_E_STREAM : result;
}

int ric_video_output(ric_video* v, int16_t* planes, int border, int on_device)
{
	if (!v || !planes) return RIC_E_ARG;
	if (v->out_id < 0 && border != 2) return RIC_E_ARG;
	if (vfail(hipSetDevice(v->device), "hipSetDevice")) return RIC_E_HIP;
	const VidGeom& g = v->g;
	const int b = border ? kVidBorder : 0;
	const int ow = g.w + 2 * b, oh = g.h + 2 * b;
	const int16_t* base = border == 2 ? v->pred_img() : v->img(v->out_id);
	for (int c = 0; c < 3; c++) {
		const int16_t* src = base + c * g.P - (long)b * g.S - b;
		VCHK(hipMemcpy2DAsync(planes + (size_t)c * ow * oh, (size_t)ow * 2, src, (size_t)g.S * 2, (size_t)ow * 2, oh,
		                      on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, v->st));
	}
	VCHK(hipStreamSynchronize(v->st));
	return RIC_OK;
}

int ric_video_motion(ric_video* v, uint32_t* mv)
{
	if (!v || !mv) return RIC_E_ARG;
	if (vfail(hipSetDevice(v->device), "hipSetDevice")) return RIC_E_HIP;
	VCHK(hipMemcpyAsync(mv, v->d_mv, sizeof(uint32_t) * v->mv.size(), hipMemcpyDeviceToHost, v->st));
	VCHK(hipStreamSynchronize(v->st));
	return RIC_OK;
}

}  // extern "C"
