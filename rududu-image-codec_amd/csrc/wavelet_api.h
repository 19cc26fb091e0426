// wavelet_api.h -- the CWavelet2D plane operations the video codec
// (video.cpp) drives, on device planes, implemented in capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "ric_gpu.h"
#include "entropy.h"

namespace ric {
namespace wapi {

// the stream every GPU stage of this pyramid runs on
hipStream_t stream(ric_wavelet* w);
// Transform(plane) -> CodeBand(m, quant, lambda) -> TSUQi(dq) -> TransformI,
// the reference's encodeImage body for one component
// (src/lib/rududucodec.cpp:70-74): the plane is rewritten with the
// reconstruction the encoder keeps
int encode_plane(ric_wavelet* w, Mux& m, int16_t* plane, long stride, int trans, int quant, int lambda, int dq);
// DecodeBand(m) -> TSUQi(dq) -> TransformI (rududucodec.cpp:81-83)
int decode_plane(ric_wavelet* w, Mux& m, int16_t* plane, long stride, int trans, int dq);
// the output of the level-1 inverse (the finest level's LL band, int16) in
// HBM after a TransformI; false for a one-level pyramid
bool ll1(ric_wavelet* w, const int16_t** p, long* pitch, int* dx, int* dy);

}  // namespace wapi
}  // namespace ric
