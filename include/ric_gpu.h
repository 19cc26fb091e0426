/* ric_gpu.h -- C-ABI of the MI355X-native rududu .ric encode/decode path.
 *
 * Drop-in boundary for the reference's src/lib codec API (the reference has no
 * C binding; these entry points are what an FFI over its C++ classes would
 * bind).  Each function names the reference interface it replaces
 * (paths relative to the reference repository root).  Plain pointers and
 * sizes only; every call returns RIC_OK (0) or a negative RIC_E_* status.
 *
 * Objects:
 *   ric_wavelet -- CWavelet2D (src/lib/wavelet2d.h:27-88): the band pyramid,
 *                  resident in HBM of one GPU; DWT / quantiser / dequantiser /
 *                  inverse DWT are HIP kernels.
 *   ric_mux     -- CMuxCodec (src/lib/muxcodec.h:66-277): the serial range
 *                  coder / raw-bit multiplexer, on the host, with an explicit
 *                  capacity (the reference has none).
 *   ric_codec   -- CompressImage / DecompressImage (src/ric/ric.cpp:123-251)
 *                  as a reusable object for one image geometry.
 */
#ifndef RIC_GPU_H
#define RIC_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RIC_OK          0
#define RIC_E_ARG      -1   /* invalid argument / geometry */
#define RIC_E_HIP      -2   /* HIP runtime error (no GPU, OOM, launch failure) */
#define RIC_E_CAPACITY -3   /* output buffer too small */
#define RIC_E_FORMAT   -4   /* bad .ric magic (the reference throws BAD_MAGIC = 2) */
#define RIC_E_STREAM   -5   /* decoder ran past the end of the stream */

/* transforms: enum trans, src/lib/utils.h:28 */
#define RIC_CDF97 0
#define RIC_CDF53 1
#define RIC_HAAR  2

typedef struct ric_wavelet ric_wavelet;
typedef struct ric_mux ric_mux;
typedef struct ric_codec ric_codec;

/* ------------------------------------------------------------- library */
const char* ric_version(void);
/* number of visible HIP devices (0 when none) */
int ric_device_count(void);
/* last HIP error string of this thread (for diagnostics) */
const char* ric_last_error(void);

/* --------------------------------------------------------- ric_wavelet */
/* CWavelet2D::CWavelet2D(int x, int y, int level, int level_chg, int Align)
 * (src/lib/wavelet2d.h:29, wavelet2d.cpp:38-81).  Align is implicit. */
int ric_wavelet_create(ric_wavelet** out, int x, int y, int level, int level_chg, int device);
/* CWavelet2D::~CWavelet2D (src/lib/wavelet2d.cpp:64-67) */
void ric_wavelet_destroy(ric_wavelet* w);
/* run this object's kernels on an existing hipStream_t (NULL: own stream) */
int ric_wavelet_set_host_threads(ric_wavelet* w, int n);
int ric_wavelet_set_stream(ric_wavelet* w, void* hip_stream);
/* block until this object's queued GPU work is done */
int ric_wavelet_sync(ric_wavelet* w);
/* CWavelet2D::SetWeight(trans t, float baseWeight) (src/lib/wavelet2d.h:36) */
int ric_set_weight(ric_wavelet* w, int trans, float base_weight);
/* CWavelet2D::Transform<short>(short* pImage, int Stride, trans t)
 * (src/lib/wavelet2d.h:33).  image_on_device: pImage is a device pointer.
 * The caller's image is only read (the reference uses it as scratch).
 * A host image is copied to the device at once and its transform deferred to
 * the next call on this object, so that Transform followed by CodeBand runs
 * as one fused forward+quantiser pass; any other call runs it first. */
int ric_transform(ric_wavelet* w, const int16_t* image, int stride, int trans, int image_on_device);
/* CWavelet2D::TransformI<short>(short* pImageEnd, int Stride, trans t)
 * (src/lib/wavelet2d.h:34).  Takes the image START (the reference takes the
 * end pointer, src/lib/wavelet2d.cpp:960-990). */
int ric_transform_inv(ric_wavelet* w, int16_t* image, int stride, int trans, int image_on_device);
/* CWavelet2D::CodeBand(CMuxCodec*, int Quant, int lambda) (src/lib/wavelet2d.h:39) */
int ric_code_band(ric_wavelet* w, ric_mux* m, int quant, int lambda);
/* The device half of CodeBand alone: buildTree (src/lib/bandcodec.cpp:239-319)
 * on every level, the coarsest LL TSUQ and the zerotree block records, left in
 * HBM (no copy, no coding).  Returns after the work completes. */
int ric_quantize(ric_wavelet* w, int quant, int lambda);
/* Transform followed by the device half of CodeBand, as one fused pass over
 * the pyramid (the 9/7 short levels transform and quantise in one kernel, the
 * unquantised bands never reach HBM).  Synchronous. */
int ric_transform_quantize(ric_wavelet* w, const int16_t* image, int stride, int trans, int image_on_device,
                           int quant, int lambda);
/* CWavelet2D::DecodeBand(CMuxCodec*) (src/lib/wavelet2d.h:38) */
int ric_decode_band(ric_wavelet* w, ric_mux* m);
/* CWavelet2D::TSUQ(int Quant, float Thres) (src/lib/wavelet2d.h:41): dead-zone
 * quantiser on every band (the LL with Thres 0.5); *count = non-zeros. */
int ric_tsuq(ric_wavelet* w, int quant, float thres, unsigned int* count);
/* CWavelet2D::TSUQi(int Quant) (src/lib/wavelet2d.h:42) */
int ric_tsuqi(ric_wavelet* w, int quant);
/* band pyramid introspection, canonical order: levels finest->coarsest
 * D, H, V, then the coarsest LL.  Replaces reads of the public
 * DBand/HBand/VBand/LBand/pLow members (src/lib/wavelet2d.h:46-51) and
 * CBand::DimX/DimY/type/Weight/pBand (src/lib/band.h:43-59). */
int ric_band_count(ric_wavelet* w);
int ric_band_info(ric_wavelet* w, int index, int* dimx, int* dimy, int* is_int, float* weight);
int ric_band_read(ric_wavelet* w, int index, int32_t* host_out);
int ric_band_write(ric_wavelet* w, int index, const int32_t* host_in);
/* CBand::pBand (src/lib/band.h:58): a pointer to band `index` in this
 * object's host mirror (row pitch *pitch samples, the band's C type), synced
 * from the device; the mirror stays authoritative -- what the caller writes
 * there is what the next GPU stage reads -- until a stage rewrites the bands. */
int ric_band_host(ric_wavelet* w, int index, void** ptr, int* pitch);
/* CBand::pBand in the reference's own layout: a stable host buffer holding
 * band `index` with row stride *stride samples = DimXAlign of CBand::Init
 * (DimX * sample size rounded up to 32 bytes, src/lib/band.cpp:57), synced
 * from the mirror on this call and whenever the mirror is rewritten
 * (CodeBand's host half, DecodeBand); what the caller writes there goes to the
 * device with the mirror at the next GPU stage, as through ric_band_host. */
int ric_band_host_ref(ric_wavelet* w, int index, void** ptr, int* stride);
/* CBand's operations on one band (band index as ric_band_info), run on the
 * device (bands written through ric_band_host go to the device first; the host
 * mirror is stale afterwards):
 *   ric_band_tsuq   CBand::TSUQ<C>(Quant, Thres) (src/lib/band.h:65-92), the
 *                   non-zero count and the Max / Min of the quantised values;
 *   ric_band_tsuqi  CBand::TSUQi<C>(Quant) (band.h:94-107);
 *   ric_band_sums   CBand::Mean's Sum and SSum (band.h:116-132: int products,
 *                   int64 sums); Mean and Var follow from them on the host;
 *   ric_band_add    CBand::Add<C>(val) (band.h:135-141), padding included;
 *   ric_band_clear  CBand::Clear (band.cpp). */
int ric_band_tsuq(ric_wavelet* w, int index, int quant, float thres, unsigned int* count, int* max, int* min);
int ric_band_tsuqi(ric_wavelet* w, int index, int quant);
int ric_band_sums(ric_wavelet* w, int index, int64_t* sum, int64_t* ssum);
int ric_band_add(ric_wavelet* w, int index, int val);
int ric_band_clear(ric_wavelet* w, int index);

/* ------------------------------------------------------------- ric_mux */
/* CMuxCodec(unsigned char* pStream, unsigned short firstWord)
 * (src/lib/muxcodec.h:102): encoder writing at most cap bytes into buf
 * (cap SIZE_MAX: no bound, the reference's contract).  buf NULL is the
 * reference's CMuxCodec(0, 0) (src/lib/rududucodec.cpp:36): no output until
 * ric_mux_reinit_encoder gives it a buffer. */
int ric_mux_create_encoder(ric_mux** out, uint8_t* buf, size_t cap, uint16_t first_word);
/* CMuxCodec::initCoder(unsigned short firstWord, unsigned char* pStream)
 * (src/lib/muxcodec.h:104, muxcodec.cpp:36-49): restart the coder (low =
 * firstWord << 16, full range, empty bit buffer).  buf non-NULL: the output
 * restarts at buf (cap bytes; SIZE_MAX: no bound); NULL keeps the output
 * position, as in the reference.  Turns a decoder object into an encoder
 * (the reference's one CMuxCodec serves both, src/lib/rududucodec.cpp:89,123). */
int ric_mux_reinit_encoder(ric_mux* m, uint8_t* buf, size_t cap, uint16_t first_word);
/* CMuxCodec::initDecoder(unsigned char* pStream) (src/lib/muxcodec.h:105,
 * muxcodec.cpp:51-61): restart the decoder on buf (payload at buf + 2): len
 * bytes copied and zero padded, or len 0 to read buf in place with no end
 * (the reference's form; UNSAFE on untrusted input, see below).  buf NULL
 * only resets the range and bit buffer, as in the reference. */
int ric_mux_reinit_decoder(ric_mux* m, const uint8_t* buf, size_t len);
/* CMuxCodec(unsigned char* pStream) (src/lib/muxcodec.h:103): decoder over
 * len bytes of buf (the reference reads its payload from buf + 2). */
int ric_mux_create_decoder(ric_mux** out, const uint8_t* buf, size_t len);
/* CMuxCodec(unsigned char* pStream) exactly (src/lib/muxcodec.h:103,
 * muxcodec.cpp:31-34): reads buf + 2 in place with no end, like the
 * reference (the caller's buffer must hold the stream).
 * UNSAFE on untrusted input: a corrupt or truncated stream makes the decoder
 * read past the caller's buffer, as the reference's does.  Kept for source
 * compatibility only; untrusted streams go through ric_mux_create_decoder
 * (bounded) -- every product path does. */
int ric_mux_create_decoder_inplace(ric_mux** out, const uint8_t* buf);
/* CMuxCodec::endCoding() (src/lib/muxcodec.h:106): *len_out = end - buf. */
int ric_mux_end(ric_mux* m, size_t* len_out);
/* CMuxCodec::getSize() (src/lib/muxcodec.h:107) */
size_t ric_mux_size(ric_mux* m);
void ric_mux_destroy(ric_mux* m);

/* ----------------------------------------------------------- ric_codec */
/* One reusable encoder/decoder for w x h images with 1 (gray) or 3 (RGB)
 * channels (src/ric/ric.cpp:123-251: 5 levels, level_chg 1, YCoCg, Quants). */
int ric_codec_create(ric_codec** out, int w, int h, int channels, int device);
void ric_codec_destroy(ric_codec* c);
int ric_codec_set_stream(ric_codec* c, void* hip_stream);
/* Host threads of one encode's serial stage (default 1).  n > 1: each band of
 * a plane is modelled on its own task of an (n - 1)-thread pool owned by the
 * object while the calling thread writes the stream in coding order from the
 * finished bands' event lists (the models are per band, bandcodec.cpp:
 * 487-507; only the range coder crosses bands, muxcodec.cpp:63-74): lower
 * latency per frame, byte-identical output.  ric_wavelet_set_host_threads is
 * the same for CWavelet2D::CodeBand. */
int ric_codec_set_host_threads(ric_codec* c, int n);
/* CompressImage: pix = channels planes of w*h bytes (R,G,B planar), on the
 * device if pix_on_device.  Writes the whole .ric file (9-byte header +
 * payload) to out (host), *len_out = its size. */
int ric_codec_encode(ric_codec* c, const uint8_t* pix, int pix_on_device, int q, int trans,
                     uint8_t* out, size_t cap, size_t* len_out);
/* DecompressImage: decodes a whole .ric file (host bytes) of this geometry.
 * pix_out: channels planes of w*h bytes (device if pix_on_device, may be
 * NULL); planes_out: the int16 planes before the 8-bit clip (device if
 * pix_on_device, may be NULL). */
int ric_codec_decode(ric_codec* c, const uint8_t* ric, size_t len, int dither,
                     uint8_t* pix_out, int16_t* planes_out, int pix_on_device);
/* ----------------------------------------------------------- ric_batch */
/* CompressImage / DecompressImage (src/ric/ric.cpp:123-251) over batches of
 * frames of one geometry -- the serving form of ric_codec, byte-identical to
 * it.  The frames of a group (at most `slots`) are coded together: every GPU
 * stage is one launch per level over the whole group (the small coarse levels
 * of one frame leave the chip mostly idle; a group fills it), and a native
 * pool of `threads` host threads runs the serial coder of different frames in
 * parallel.  Two sets of slots: ric_batch_roundtrip overlaps the GPU stages of
 * one group with the host coding of the previous one.  One call at a time per
 * object. */
typedef struct ric_batch ric_batch;
int ric_batch_create(ric_batch** out, int w, int h, int channels, int slots, int threads, int device);
void ric_batch_destroy(ric_batch* b);
/* n <= slots frames: pix[i] = channels planes of w*h bytes (device pointers
 * if pix_on_device); the .ric file of frame i is written to out[i] (cap[i]
 * bytes, host), its size to len[i]. */
int ric_batch_encode(ric_batch* b, const uint8_t* const* pix, int n, int pix_on_device, int q, int trans,
                     uint8_t* const* out, const size_t* cap, size_t* len);
/* n <= slots .ric files (host bytes) of this geometry and one transform;
 * frame i's pixels to pix_out[i] (device if pix_on_device).  RIC_E_STREAM
 * when a stream ran past its end (the frames are still written). */
int ric_batch_decode(ric_batch* b, const uint8_t* const* ric, const size_t* len, int n, uint8_t* const* pix_out,
                     int pix_on_device);
/* encode then decode n frames (any n, device pixels in and out; .ric files
 * to host out[i]), in groups of `slots` frames, pipelined. */
int ric_batch_roundtrip(ric_batch* b, const uint8_t* const* pix, int n, int q, int trans, uint8_t* const* out,
                        const size_t* cap, size_t* len, uint8_t* const* pix_out);
/* The whole CompressImage of n <= slots frames on the GPU, the serial coder
 * included (one wave per frame's stream; colour: the three planes into one
 * stream on one wave, as ric.cpp:157-176, with 3 n <= 2 slots: a frame's
 * plane pyramids take three arenas): pix[i] device pixels; the
 * .ric file of frame i to out + i * ostride (DEVICE memory, cap <= ostride
 * bytes each; cap and ostride multiples of 16, else RIC_E_ARG), its size to
 * len[i] (host).  Byte-identical to ric_batch_encode.
 * No reference counterpart (the reference's CompressImage is one stream on
 * one host thread). */
int ric_batch_encode_gpu(ric_batch* b, const uint8_t* const* pix, int n, int q, int trans, uint8_t* out, size_t ostride,
                         size_t cap, size_t* len);
/* The whole DecompressImage of n <= slots frames on the GPU (colour as for
 * ric_batch_encode_gpu: 3 n <= 2 slots), the serial
 * decoder included (one wave per stream): the .ric files at in + i * istride
 * (DEVICE memory, istride a multiple of 16), their sizes len[i]; pixels to
 * device pix_out[i].  RIC_E_STREAM as ric_batch_decode. */
int ric_batch_decode_gpu(ric_batch* b, const uint8_t* in, size_t istride, const size_t* len, int n, uint8_t* const* pix_out);
/* Diagnostics (no reference counterpart), process-wide: while dev_buf is set,
 * every ric_batch_decode_gpu call of n frames writes into it (u32 words):
 *   frame f, words [f*2048, f*2048 + 512): 8 words of coder state (range, low,
 *     code, nbits, buffer, read position, overflow flags, 0xC0DE) after the LL
 *     and after each band, 64 slots;
 *   frame f, words [f*2048 + 1024, f*2048 + 2048): the first 1024 values of
 *     the decoded LL, row-major;
 *   frame 0's whole decoded pyramid from word n*2048 on (finest first, D H V,
 *     then the LL; dimx*dimy words per band).
 * Size dev_buf for n*2048 words plus the pyramid's sample count.  NULL: off.
 * One caller at a time (the pointer is a process global). */
int ric_diag_gdec_dbg(void* dev_buf);
/* Hybrid round trip: the serial encoder runs on the GPU (one wave per
 * stream, launches of `pool_frames` frames, each stream up to stream_cap
 * bytes: a multiple of 16; a longer stream fails the call with
 * RIC_E_CAPACITY), the serial decoder on the GPU or the host pool.  Gray or
 * colour (a colour frame's Y, Co, Cg plane pyramids sit side by side in the
 * pool and one wave codes them into the frame's one stream, ric.cpp:157-176).
 * Configure once.
 * A pool that does not fit in device memory returns RIC_E_CAPACITY with
 * nothing allocated (the batch stays usable: retry with fewer frames). */
int ric_batch_hybrid_config(ric_batch* b, int pool_frames, size_t stream_cap);
/* The same, with the pool's level-0 value capacity.  value_cap > 0: the pool
 * holds each frame's (each colour plane's) three finest bands compacted --
 * only their non-zero values, at most value_cap of them, and a mask per 4x4
 * block -- instead of dense (at C3 about 25 MB instead of 50 MB per frame, so
 * more frames fit); a frame with more non-zero values than that is coded on
 * the host instead (same bytes, slower), never an error.  value_cap < 0: the
 * default, 9 / 16 of the finest bands' coefficients
 * (ric_batch_hybrid_config); 0: dense bands (no compaction). */
int ric_batch_hybrid_config_ex(ric_batch* b, int pool_frames, size_t stream_cap, long value_cap);
/* Output digests (no reference counterpart; for verifying a serving step
 * whose output buffers are reused): while set, the decode / round-trip calls
 * write, for frame i of the call (i < n), the 64-bit digest of its decoded
 * pixels, sum over byte k of pix[k] * (k * 0x9E3779B97F4A7C15 + 1) mod 2^64,
 * to dev_digests[i] (device memory), in stream order right after the pixels.
 * n = 0 turns it off.  The library keeps the pointer across calls: the buffer
 * must stay allocated until the digests are turned off (or the batch is
 * destroyed). */
int ric_batch_set_digests(ric_batch* b, unsigned long long* dev_digests, long n);
/* Stream-ready words (no reference counterpart; they let a caller ship the
 * .ric files while the call still runs, e.g. the multi-GPU gather): while set,
 * ric_batch_roundtrip and ric_batch_roundtrip_hybrid store, for frame i of
 * the call (i < n), the file's length into host_words[i] (release order) as
 * soon as out[i] holds the complete file; the caller zeroes the words before
 * each call and polls them.  The words must stay allocated until turned off
 * (n = 0). */
int ric_batch_set_ready(ric_batch* b, uint32_t* host_words, long n);
/* As ric_batch_roundtrip (device pixels in and out, .ric files to host
 * out[i]): frames [0, n_host) encoded and decoded on the host; frames
 * [n_host, n) encoded by the GPU stream coder and decoded by the GPU stream
 * decoder (gpu_decode 1), on the host pool (0), or per coder launch by
 * whichever is free (2: the host pool while its backlog is shorter than a
 * launch, the GPU for the rest).  Byte-identical streams either way.  Colour
 * frames coded or decoded on the host take three slots each (one per plane),
 * so their groups are slots / 3 frames: with host frames or gpu_decode != 1
 * a colour batch needs slots >= 3 (else RIC_E_ARG). */
int ric_batch_roundtrip_hybrid(ric_batch* b, const uint8_t* const* pix, int n, int n_host, int gpu_decode, int q,
                               int trans, uint8_t* const* out, const size_t* cap, size_t* len, uint8_t* const* pix_out);
/* When each side of the last ric_batch_roundtrip_hybrid finished, in ms from
 * its entry: the last host round-trip group, the last stream-coder batch (0
 * for a side with no work).  For splitting frames between the two (no
 * reference counterpart). */
int ric_batch_hybrid_times(ric_batch* b, double* host_ms, double* gpu_ms);
/* Frames of the last ric_batch_roundtrip_hybrid that the stream coder left
 * to a host round trip because they hold more level-0 values than the
 * compacted pool's capacity (no reference counterpart). */
int ric_batch_hybrid_fallbacks(ric_batch* b, int* frames);
/* Stage timers of the batch (no reference counterpart): 0 pixel conversion
 * in, 1..8 forward level 0..7 (fused DWT + quantiser + records), 9 D2H of
 * bands + records, 10 host encode, 11 host decode, 12 H2D of the bands,
 * 13..20 inverse level 0..7 (fused TSUQi), 21 pixel conversion out, 22 / 23 the
 * GPU stream encoder / decoder launches (ms = kernel time, frames = streams), 24
 * the compacted payload values of host-coded frames to the host (a kernel
 * writing the device-mapped mirrors; stage 9 then covers only the dense rest:
 * int bands, LL, records).  ms are
 * sums; frames = frames covered; launches = GPU launches (host: frames). */
#define RIC_BATCH_STAGES 25
/* Diagnostics: the batch's GPU stages alone, iters times over n <= slots
 * device frames (forward levels + D2H, H2D + inverse levels of the bands just
 * quantised, pixel output to pix_out if given); no host coding. */
int ric_batch_diag_gpu(ric_batch* b, const uint8_t* const* pix, int n, int q, int trans, int iters,
                       uint8_t* const* pix_out);
/* The forward levels alone, iters times back to back over n <= slots device
 * frames (what the serving step's front runs before a coder launch; the
 * bench's roofline_isolated). */
int ric_batch_diag_gpu_encode(ric_batch* b, const uint8_t* const* pix, int n, int q, int trans, int iters);
int ric_batch_prof_enable(ric_batch* b, int on);
int ric_batch_prof_read(ric_batch* b, double* ms, long* frames, long* launches, int n);

/* ----------------------------------------------------------- ric_video */
/* The reference video codec, CRududuCodec (src/lib/rududucodec.{h,cpp}):
 * key frames every 10 frames, the others predicted by EPZS motion search
 * (COBME, src/lib/obme.cpp) and OBMC (COBMC, src/lib/obmc.cpp) from the
 * previous reconstruction at quarter pel (CImageBuffer::calc_sub), the
 * residual through a 3-level 9/7 wavelet closed loop, motion vectors and
 * bands in one CMuxCodec stream per frame.  Frames stay in HBM; the search,
 * interpolation, OBMC and wavelet stages are HIP kernels, the two serial
 * coders run on the host.  One change from the reference: TransformI gets
 * each plane's end pointer (rududucodec.cpp:74,83 pass the start, which
 * writes outside the image: DESIGN.md §9). */
typedef struct ric_video ric_video;
/* CRududuCodec(cmode mode, int width, int height, int component)
 * (src/lib/rududucodec.h:35, rududucodec.cpp:32-48); encoder 1 = encode,
 * 0 = decode; component must be 3 (CImage::inputSGI writes Y, Co, Cg). */
int ric_video_create(ric_video** out, int encoder, int w, int h, int component, int device);
/* CRududuCodec::~CRududuCodec (rududucodec.cpp:51-56) */
void ric_video_destroy(ric_video* v);
/* the public member CRududuCodec::quant (rududucodec.h:33): the quantiser is
 * quants(quant + 20), the RD lambda quants(quant + 12) (rududucodec.cpp:58-71);
 * -12 <= quant <= 30 (the table's defined range) */
int ric_video_set_quant(ric_video* v, int quant);
/* the encoder's serial stage over n host threads (ric_codec_set_host_threads) */
int ric_video_set_host_threads(ric_video* v, int n);
/* CRududuCodec::encode(unsigned char* pImage, int stride, unsigned char*
 * pBuffer, CImage** outImage) (rududucodec.cpp:87-119).  pix: 3 planes R, G,
 * B of h rows x stride bytes, bottom row first (CImage::inputSGI), on the host
 * or the device (pix_on_device).  The stream goes to the host buffer buf (cap
 * bytes; the reference has no bound); *size = the reference's return value,
 * endCoding() - pBuffer - 2 (the stream is *size + 2 bytes). */
int ric_video_encode(ric_video* v, const uint8_t* pix, int stride, int pix_on_device, uint8_t* buf, size_t cap,
                     int* size);
/* CRududuCodec::decode(unsigned char* pBuffer, CImage** outImage)
 * (rududucodec.cpp:121-141): buf holds the len bytes of one frame's stream;
 * *size = codec.getSize().  RIC_E_STREAM when the decoder ran past len.
 * len 0 reads buf in place with no end, as the reference does (UNSAFE on
 * untrusted input, see ric_mux_create_decoder_inplace). */
int ric_video_decode(ric_video* v, const uint8_t* buf, size_t len, int* size);
/* *outImage of the last encode / decode: its planes Y, Co, Cg as int16,
 * 3 x h x w (border 0), or with the 15-sample border, 3 x (h + 30) x (w + 30)
 * (border 1), to host or device memory (on_device).  Diagnostics: border 2
 * copies the OBMC prediction (predImage) instead, with its border. */
int ric_video_output(ric_video* v, int16_t* planes, int border, int on_device);
/* the motion field after the last encode / decode: (w >> 3) x (h >> 3)
 * vectors in quarter pel, x in the low 16 bits, y in the high 16, MV_INTRA =
 * 0x80008000 (COBMC::pMV, obmc.h:29-57) */
int ric_video_motion(ric_video* v, uint32_t* mv);

/* ------------------------------------------------------- device memory */
/* HBM buffers from this library's own HIP runtime (no reference counterpart:
 * the reference is host-only).  Callers that have no HIP runtime of their own
 * (the ctypes binding, the tests, the benchmark) use these, so only this
 * library's runtime is ever mapped into the process.  Copies, memsets and
 * digests are synchronous to the caller and run on a per-device side stream
 * of their own: they never wait for the library's kernels in flight (e.g. the
 * stream coder's launch), and never synchronise the device.  ric_device_free
 * (hipFree) does synchronise the device: keep it out of a running step. */
#define RIC_COPY_H2D 1
#define RIC_COPY_D2H 2
#define RIC_COPY_D2D 3
int ric_device_alloc(int device, size_t bytes, void** out);   /* RIC_E_CAPACITY when HBM is exhausted */
/* ric_device_free / ric_host_free never wait for a GPU stream coder launch:
 * hipFree / hipHostFree synchronise the whole device, so while a call with a
 * coder launch in flight runs (ric_batch_encode_gpu, _decode_gpu,
 * _roundtrip_hybrid, on any thread) the pointer is parked and freed when the
 * last such call returns; otherwise it is freed at once.  The same holds for
 * the buffers of any ric_* object destroyed meanwhile. */
int ric_device_free(void* p);
int ric_device_copy(int device, void* dst, const void* src, size_t bytes, int kind);
int ric_device_memset(int device, void* p, int value, size_t bytes);
int ric_device_sync(int device);
/* pinned (page-locked) host memory */
int ric_host_alloc(size_t bytes, void** out);
int ric_host_free(void* p);
/* the 64-bit digest of ric_batch_set_digests over n device byte runs
 * base + off[i], len[i] bytes each (position 0 = the run's first byte), to
 * host_out[i] */
int ric_device_digests(int device, const uint8_t* base, int n, const size_t* off, const size_t* len,
                       unsigned long long* host_out);
/* the same digest over n host byte runs base + off[i], len[i] bytes each */
int ric_host_digests(const uint8_t* base, int n, const size_t* off, const size_t* len, unsigned long long* out);
/* n host byte runs src[i] (len[i] bytes) packed at dst + off[i] on the device
 * (the gaps between runs zeroed, up to the last run's end): one copy through a
 * pinned staging buffer of the library's (sized once, >= 64 MiB); dig_out
 * (optional): each run's digest, taken from its source on the way */
int ric_device_pack_h2d(int device, uint8_t* dst, int n, const uint8_t* const* src, const size_t* len, const size_t* off,
                        unsigned long long* dig_out);

/* ------------------------------------------------------------ ric_comm */
/* The path's one exchange across GPUs: the .ric streams
 * of every rank gathered to rank 0, over RCCL (xGMI).  One communicator per
 * process (one process per GPU).  No reference counterpart: the reference
 * writes one file per image (src/ric/ric.cpp:174-176).  The chunked gather
 * protocol runs on the host (shard.py StreamGather) over these primitives. */
typedef struct ric_comm ric_comm;
#define RIC_COMM_ID_BYTES 128
#define RIC_RED_SUM 0
#define RIC_RED_MAX 1
#define RIC_RED_MIN 2
/* rank 0 makes the id; every rank passes the same bytes to ric_comm_create */
int ric_comm_unique_id(uint8_t* id, size_t len);
int ric_comm_create(ric_comm** out, const uint8_t* id, int nranks, int rank, int device);
void ric_comm_destroy(ric_comm* c);
/* all-reduce of n host doubles in place (op RIC_RED_*); also the barrier */
int ric_comm_allreduce_f64(ric_comm* c, double* vals, int n, int op);
/* one group of point-to-point operations, completed before return: op i sends
 * (is_send[i]) or receives bytes[i] bytes of DEVICE buffer buf[i] to / from
 * rank peer[i]; sends and receives between two ranks match in issue order */
int ric_comm_sendrecv(ric_comm* c, int nops, const int* peer, const int* is_send, void* const* buf, const size_t* bytes);

/* .ric header fields (src/ric/ric.cpp:114-121, 187-200) */
int ric_read_header(const uint8_t* ric, size_t len, int* w, int* h, int* channels, int* q, int* trans);
/* src/ric/ric.cpp:42-49 */
int ric_quants(int idx);

/* ------------------------------------------------------ instrumentation */
/* Stage timers (no reference counterpart).  Stage order: 0 forward level 0,
 * 1 forward all levels, 2 quantiser, 3 bands D2H, 4 host entropy encode,
 * 5 host entropy decode, 6 bands H2D, 7 dequantiser, 8 inverse all levels,
 * 9 pixel conversion in, 10 pixel conversion out.  GPU stages are HIP events
 * on the object's stream; ms are sums, counts the number of samples. */
#define RIC_PROF_STAGES 11
int ric_prof_enable(ric_wavelet* w, int on);
int ric_prof_read(ric_wavelet* w, double* ms, long* counts, int n);
ric_wavelet* ric_codec_wavelet(ric_codec* c);
/* Diagnostics: with RIC_FQ_PC bit 128 set, every level-0 launch of the fused
 * level kernel records 168 u64 per workgroup: start realtime, start shader
 * clock, end realtime of waves 0-3, producer HW_ID << 32 | end clock,
 * XCC_ID << 32 | workgroup index, then per role (producer, D, H, V) 20
 * (barrier arrival, departure) realtime pairs; copies up to n u64. */
int ric_diag_wgtrace(int device, uint64_t* out, int n);
/* Fault injection (tests): while on, the consumer waves of the fused level
 * kernels' LDS ring hand-off wait for a block row that never comes; the wait
 * gives up, raises the device status word, and the call that syncs next
 * (CodeBand, Quantize, TransformQuantize, the codec's encode) returns
 * RIC_E_HIP instead of a corrupt result. */
int ric_diag_fault(int on);
/* the number of frees parked so far (ric_device_free above) */
long ric_diag_deferred_frees(void);
/* SURVEY.md §8(d) synthetic image: channels planes of w*h bytes */
void ric_synth_image(int w, int h, int channels, int frame, uint8_t* out);

#ifdef __cplusplus
}
#endif

#endif /* RIC_GPU_H */
