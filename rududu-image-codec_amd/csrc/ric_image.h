// ric_image.h -- launchers of the pixel conversion kernels (image.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ric {
// u8 planes (R,G,B planar or gray) -> int16 coding planes (Y,Cg,Co or gray), pitch po
void launch_pix_in(const uint8_t* pix, int16_t* planes, int w, int h, long po, int channels, int q, hipStream_t st);
// int16 decoded planes (Y,Cg,Co or gray, pitch pi) -> u8 pixels and/or int16 output planes (w*h);
// dig (with pix): the pixels' digest (launch_digest's) added into *dig, fused into
// the conversion where the 8-pixel gray form runs
void launch_pix_out(const int16_t* planes_in, long pi, int w, int h, int channels, int q,
                    uint8_t* pix, int16_t* planes_out, hipStream_t st, unsigned long long* dig = nullptr);
// 64-bit digest of n bytes: sum over i of p[i] * (i * 0x9E3779B97F4A7C15 + 1),
// mod 2^64, added into *out (zero it first): an order-free checksum of a
// decoded frame (ric_batch_set_digests)
void launch_digest(const uint8_t* p, size_t n, unsigned long long* out, hipStream_t st);
// the same over up to kDigestRuns runs base + off[i] (len[i] bytes each) in one
// launch, run i's digest to out[i] (written, not added)
constexpr int kDigestRuns = 64;
void launch_digests(const uint8_t* base, const size_t* off, const size_t* len, int n, unsigned long long* out, hipStream_t st);
// out[i] = the sum of part[16 i .. 16 i + 15] for i < n (the fused pixel
// output's 16 partial digest words per frame: launch_inv_level_z)
void launch_digest_fold(const unsigned long long* part, unsigned long long* out, int n, hipStream_t st);
}  // namespace ric
