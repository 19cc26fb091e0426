// ric_image.h -- launchers of the pixel conversion kernels (image.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ric {
// u8 planes (R,G,B planar or gray) -> int16 coding planes (Y,Cg,Co or gray), pitch po
void launch_pix_in(const uint8_t* pix, int16_t* planes, int w, int h, long po, int channels, int q, hipStream_t st);
// int16 decoded planes (Y,Cg,Co or gray, pitch pi) -> u8 pixels and/or int16 output planes (w*h)
void launch_pix_out(const int16_t* planes_in, long pi, int w, int h, int channels, int q,
                    uint8_t* pix, int16_t* planes_out, hipStream_t st);
}  // namespace ric
