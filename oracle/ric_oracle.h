/* oracle/ric_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement of the rududu .ric encode/decode path (the
 * reference's src/lib + the caller side of src/ric/ric.cpp).  It is the parity
 * checker for the HIP product path and the "port" CPU baseline; the product
 * never links or calls it.  The API mirrors oracle/ref_driver.cpp one for one
 * (ricor_* here, ricref_* there) so tests compare the two directly.
 *
 * Canonical band order: for each level finest->coarsest: D, H, V; then LL.
 * Bands are DimX*DimY int32, row-major, no padding.
 */
#ifndef RIC_ORACLE_H
#define RIC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int  ricor_layout(int w, int h, int levels, int lc, int32_t* out);
long ricor_bands(const int16_t* img, int w, int h, int levels, int lc, int trans,
                 int stage, int quant, int lambda, int32_t* out);
long ricor_encode_planes(const int16_t* planes, int nplanes, int w, int h, int levels,
                         int lc, int trans, const int* quant, const int* lambda,
                         uint8_t* out, long cap);
long ricor_decode_planes(const uint8_t* in, long len, int nplanes, int w, int h, int levels,
                         int lc, int trans, const int* quant, int16_t* planes_out,
                         int32_t* bands_out);
long ricor_encode_ric(const uint8_t* pix, int w, int h, int channels, int q, int trans,
                      uint8_t* out, long cap);
long ricor_decode_ric(const uint8_t* ric, long len, int dither_on, int16_t* planes_out,
                      uint8_t* pix_out, int32_t* dims);
/* inverse transform only: bands (canonical order, already dequantised) -> plane */
long ricor_inverse(const int32_t* bands, int w, int h, int levels, int lc, int trans,
                   int16_t* plane_out);
/* Transform -> CodeBand -> TSUQi(dq) -> TransformI on one plane
 * (src/lib/rududucodec.cpp:67-74); bands_out (optional) after TSUQi */
long ricor_closed_loop(const int16_t* img, int w, int h, int levels, int lc, int trans, int quant, int lambda,
                       int dq, int16_t* plane_out, int32_t* bands_out);
/* SURVEY.md §8(d) synthetic generator: channels planes of w*h bytes */
void ricor_synth(int w, int h, int channels, int frame, uint8_t* out);
short ricor_quants(int idx);

#ifdef __cplusplus
}
#endif
#endif
