// video_intra.cpp -- the reference video codec's intra coding loop, written
// against the reference's src/lib API, built twice:
//   * with -DRIC_SHIM on include/rududu_gpu.hpp (the GPU drop-in):
//     tests/native/video_intra;
//   * against the reference's own headers and src/lib sources compiled where
//     they lie (oracle/Makefile): oracle/_ref/video_intra_ref -- TEST
//     INFRASTRUCTURE, the checker.
//
// It restates CRududuCodec::encodeImage / decodeImage
// (src/lib/rududucodec.cpp:67-85) with the reference's call forms: ONE
// CMuxCodec constructed as CMuxCodec(0, 0) (:36) and re-initialised per frame
// with initCoder(0, pBuffer) (:89) / initDecoder(pBuffer) (:123), reused as
// encoder and decoder; CWavelet2D(w, h, 3) with SetWeight(cdf97) (:39-40);
// per component Transform -> CodeBand(quants(q + 20), quants(q + 12)) ->
// TSUQi(quants(q + 20)) -> TransformI on a CImage-style bordered plane
// (dimXAlign stride, BORDER 15: src/lib/image.cpp:56-68), and the video
// quantiser table quants() (:58-65).
//
// One deliberate difference from rududucodec.cpp:74,83: TransformI gets the
// plane's END pointer, the form CWavelet2D::TransformI takes since ric_0.2
// (src/lib/wavelet2d.cpp:507 starts its output DimY rows before the pointer;
// ric.cpp:216-225 passes the end).  rududucodec.cpp passes the plane START,
// which writes the reconstruction DimY rows above the plane -- outside the
// allocation for plane 0 (the reference video codec crashes).
//
//   video_intra W H Q NFRAMES in.i16 out.bin
//     in.i16:  NFRAMES x 3 planes x H x W int16 (the planes' samples)
//     out.bin: per frame: u32 size (endCoding() - pBuffer - 2), the stream's
//              size + 2 bytes, the encoder's reconstruction (3 x H x W int16),
//              the decoder's planes (3 x H x W int16), u32 decoder getSize()
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#ifdef RIC_SHIM
#include "rududu_gpu.hpp"
#else
#include "muxcodec.h"
#include "wavelet2d.h"
#endif

using namespace rududu;

namespace {

const int kLevels = 3;          // WAV_LEVELS (rududucodec.cpp:26)
const int kBorder = 15;         // BORDER (src/lib/image.h:27)
const int kComp = 3;

// CRududuCodec::quants (src/lib/rududucodec.cpp:58-65)
short quants(int idx)
{
	static const unsigned short Q[5] = {32768, 37641, 43238, 49667, 57052};
	if (idx == 0) return 0;
	idx--;
	int r = 10 - idx / 5;
	return (short)((Q[idx % 5] + (1 << (r - 1))) >> r);
}

// a CImage's planes (src/lib/image.cpp:56-68): dimXAlign = (x + 2 BORDER +
// 31) & -32 samples, BORDER rows above and below, planes back to back
struct Planes {
	int w, h, stride;
	std::vector<short> data;
	short* plane[kComp];
	Planes(int w_, int h_) : w(w_), h(h_)
	{
		stride = (w + 2 * kBorder + 31) & -32;
		const size_t per = (size_t)stride * (h + 2 * kBorder);
		data.assign(per * kComp + 64, 0);
		for (int c = 0; c < kComp; c++) plane[c] = data.data() + 32 + c * per + kBorder * stride + kBorder;
	}
};

}  // namespace

int main(int argc, char** argv)
{
	if (argc != 7) {
		fprintf(stderr, "usage: %s W H Q NFRAMES in.i16 out.bin\n", argv[0]);
		return 2;
	}
	const int W = atoi(argv[1]), H = atoi(argv[2]), q = atoi(argv[3]), nf = atoi(argv[4]);
	FILE* fi = fopen(argv[5], "rb");
	FILE* fo = fopen(argv[6], "wb");
	if (!fi || !fo) return 2;

	std::vector<unsigned char> buf((size_t)W * H * kComp * 4 + 4096, 0);
	CMuxCodec codec(0, 0);                            // rududucodec.cpp:36
	CWavelet2D* wavelet = new CWavelet2D(W, H, kLevels);
	wavelet->SetWeight(cdf97);
	Planes enc(W, H), dec(W, H);
	std::vector<short> in((size_t)W * H);

	for (int f = 0; f < nf; f++) {
		for (int c = 0; c < kComp; c++) {
			if (fread(in.data(), 2, in.size(), fi) != in.size()) return 3;
			for (int y = 0; y < H; y++) memcpy(enc.plane[c] + (size_t)y * enc.stride, in.data() + (size_t)y * W, 2 * W);
		}
		// CRududuCodec::encode (rududucodec.cpp:89) + encodeImage (:67-76)
		std::fill(buf.begin(), buf.end(), 0);
		codec.initCoder(0, buf.data());
		for (int c = 0; c < kComp; c++) {
			wavelet->Transform(enc.plane[c], enc.stride, cdf97);
			wavelet->CodeBand(&codec, quants(q + 20), quants(q + 12));
			wavelet->TSUQi(quants(q + 20));
			wavelet->TransformI(enc.plane[c] + (size_t)H * enc.stride, enc.stride, cdf97);
		}
		const uint32_t size = (uint32_t)(codec.endCoding() - buf.data() - 2);
		fwrite(&size, 4, 1, fo);
		fwrite(buf.data(), 1, size + 2, fo);
		for (int c = 0; c < kComp; c++)
			for (int y = 0; y < H; y++) fwrite(enc.plane[c] + (size_t)y * enc.stride, 2, W, fo);

		// CRududuCodec::decode (rududucodec.cpp:123) + decodeImage (:78-85):
		// the same CMuxCodec object, now a decoder
		codec.initDecoder(buf.data());
		for (int c = 0; c < kComp; c++) {
			wavelet->DecodeBand(&codec);
			wavelet->TSUQi(quants(q + 20));
			wavelet->TransformI(dec.plane[c] + (size_t)H * dec.stride, dec.stride, cdf97);
		}
		for (int c = 0; c < kComp; c++)
			for (int y = 0; y < H; y++) fwrite(dec.plane[c] + (size_t)y * dec.stride, 2, W, fo);
		const uint32_t dsize = codec.getSize();
		fwrite(&dsize, 4, 1, fo);
	}
	delete wavelet;
	fclose(fo);
	fclose(fi);
	return 0;
}
