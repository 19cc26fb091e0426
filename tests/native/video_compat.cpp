// video_compat.cpp -- a testmotion.cpp-style caller (src/utils/testmotion.cpp:
// 30-69) of the video codec, written against the reference's API and built on
// include/rududu_gpu.hpp: CRududuCodec encoder / decoder objects, the public
// `quant`, encode() / decode() with their return values and CImage**
// outputs, CImage::psnr and CImage::outputYV12<char, false>.
//
//   video_compat W H Q NFRAMES in.rgb out.bin
//     in.rgb : NFRAMES frames of 3 planes R, G, B, bottom row first (W bytes a row)
//     out.bin: per frame: u32 encode() return, the size + 2 stream bytes,
//              u32 decode() return, the encoder's output image as
//              outputYV12<char, false>(out, W, -128) (W * H * 3 / 2 bytes),
//              3 float psnr(origin, encoder image), 3 float psnr(origin, decoder image)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rududu_gpu.hpp"

using namespace rududu;

int main(int argc, char** argv)
{
	if (argc != 7) {
		fprintf(stderr, "usage: %s W H Q NFRAMES in.rgb out.bin\n", argv[0]);
		return 2;
	}
	const int W = atoi(argv[1]), H = atoi(argv[2]), Q = atoi(argv[3]), N = atoi(argv[4]);
	const int CMPNT = 3;
	FILE* fi = fopen(argv[5], "rb");
	FILE* fo = fopen(argv[6], "wb");
	if (!fi || !fo) return 2;
	std::vector<unsigned char> tmp((size_t)W * H * CMPNT), pStream((size_t)W * H * CMPNT * 4 + 4096, 0);
	CImage origin(W, H, CMPNT, ALIGN);
	CRududuCodec encoder(rududu::encode, W, H, CMPNT);
	CRududuCodec decoder(rududu::decode, W, H, CMPNT);
	encoder.quant = Q;
	decoder.quant = Q;
	std::vector<char> yv((size_t)W * H * 3 / 2 + 16);
	for (int k = 0; k < N; k++) {
		if (fread(tmp.data(), 1, tmp.size(), fi) != tmp.size()) return 3;
		origin.inputSGI(tmp.data(), W, -128);
		CImage* encOutImage = 0;
		const int size_enc = encoder.encode(tmp.data(), W, pStream.data(), &encOutImage);
		const uint32_t se = (uint32_t)size_enc;
		fwrite(&se, 4, 1, fo);
		fwrite(pStream.data(), 1, se + 2, fo);
		CImage* outImage = 0;
		const uint32_t sd = (uint32_t)decoder.decode(pStream.data(), &outImage);
		fwrite(&sd, 4, 1, fo);
		float psnr[2][CMPNT];
		origin.psnr(*encOutImage, psnr[0]);
		origin.psnr(*outImage, psnr[1]);
		encOutImage->outputYV12<char, false>(yv.data(), W, -128);
		fwrite(yv.data(), 1, (size_t)W * H * 3 / 2, fo);
		fwrite(psnr, sizeof(float), 2 * CMPNT, fo);
		fprintf(stderr, "%d\t%d\t%.3f\t%.3f\t%.3f\t%.3f\t%.3f\t%.3f\n", size_enc, (int)sd, psnr[0][0], psnr[0][1], psnr[0][2],
		        psnr[1][0], psnr[1][1], psnr[1][2]);
	}
	fclose(fo);
	fclose(fi);
	return 0;
}
