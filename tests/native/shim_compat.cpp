// shim_compat.cpp -- a caller written against the reference's src/lib API,
// built on include/rududu_gpu.hpp (the GPU drop-in).  It uses the reference's
// own call forms: CMuxCodec(pStream, 0) / CMuxCodec(pStream) without sizes
// (src/ric/ric.cpp:157, 207), Transform on the plane start and TransformI on
// the plane END (ric.cpp:163-171, 216-225), the public band members
// DBand/HBand/VBand/LBand and the pLow chain (src/lib/wavelet2d.h:46-51), and
// CBand's fields and `(C*) pBand` (src/lib/band.h:43-59).
//
//   shim_compat enc W H Q TRANS in.raw out.ric    8-bit gray raw in, .ric out
//   shim_compat dec in.ric out.raw                 .ric in, 8-bit gray raw out
//   shim_compat bands W H Q TRANS in.raw out.i32   Transform, then every band
//                                                  read through (C*) pBand,
//                                                  canonical order, int32
//   shim_compat stats W H TRANS in.raw              Transform, then Stats()
//   shim_compat poke W H TRANS in.raw               writes through pBand reach the device
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "rududu_gpu.hpp"

using namespace rududu;

namespace {

const int kLevels = 5, kShift = 4;   // WAV_LEVELS, SHIFT (src/ric/ric.cpp:36-39)

int Quants(int idx) { return ric_quants(idx); }

std::vector<unsigned char> slurp(const char* path)
{
	std::ifstream f(path, std::ios::binary);
	return std::vector<unsigned char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

std::vector<short> gray_plane(const std::vector<unsigned char>& px, int Quant)
{
	std::vector<short> img(px.size());
	for (size_t i = 0; i < px.size(); i++) img[i] = Quant ? (short)((px[i] - 128) << kShift) : (short)(px[i] - 128);
	return img;
}

int enc(int W, int H, int Quant, trans Trans, const char* in, const char* out)
{
	std::vector<short> img = gray_plane(slurp(in), Quant);
	const unsigned int imSize = W * H;
	std::vector<unsigned char> buf(imSize * 2 + 65536);
	unsigned char* pStream = buf.data();
	unsigned char* pEnd = pStream;
	CMuxCodec Codec(pEnd, 0);
	CWavelet2D Wavelet(W, H, kLevels, kLevels - 4);
	Wavelet.SetWeight(Trans);
	Wavelet.Transform(img.data(), W, Trans);
	Wavelet.CodeBand(&Codec, Quant ? Quants(Quant + kShift * 5) : 0, Quant ? Quants(Quant + kShift * 5 - 7) : 0);
	pEnd = Codec.endCoding();
	std::ofstream o(out, std::ios::binary);
	o << "RUD2";
	unsigned short tmp = W;
	o.write((char*)&tmp, 2);
	tmp = H;
	o.write((char*)&tmp, 2);
	const unsigned char head = (unsigned char)(Quant | ((int)Trans << 6));
	o.write((const char*)&head, 1);
	o.write((char*)pStream + 2, pEnd - pStream - 2);
	return 0;
}

int dec(const char* in, const char* out)
{
	std::vector<unsigned char> file = slurp(in);
	unsigned short W, H;
	memcpy(&W, &file[4], 2);
	memcpy(&H, &file[6], 2);
	const int Quant = file[8] & 31;
	const trans Trans = (trans)(file[8] >> 6);
	std::vector<unsigned char> buf((size_t)W * H + 2 + 16, 0);
	unsigned char* pStream = buf.data();
	memcpy(pStream + 2, file.data() + 9, std::min(file.size() - 9, (size_t)W * H));
	CMuxCodec Codec(pStream);
	CWavelet2D Wavelet(W, H, kLevels, kLevels - 4);
	Wavelet.SetWeight(Trans);
	Wavelet.DecodeBand(&Codec);
	if (Quant != 0) Wavelet.TSUQi(Quants(Quant + kShift * 5));
	std::vector<short> img((size_t)W * H, 0);
	Wavelet.TransformI(img.data() + W * H, W, Trans);
	std::vector<unsigned char> px(img.size());
	for (size_t i = 0; i < img.size(); i++) {
		int v = Quant == 0 ? img[i] + 128 : 128 + ((img[i] + (1 << (kShift - 1))) >> kShift);
		px[i] = (unsigned char)(v < 0 ? 0 : v > 255 ? 255 : v);
	}
	std::ofstream(out, std::ios::binary).write((const char*)px.data(), px.size());
	return 0;
}

// the caller recomputes the row stride the reference's way (CBand::Init,
// src/lib/band.cpp:57: DimX * sizeof(C) rounded up to ALIGN = 32 bytes) and
// walks pBand with it
template <class C>
unsigned int ref_stride(const CBand& b)
{
	return (unsigned int)(((b.DimX * sizeof(C) + 31) & ~(size_t)31) / sizeof(C));
}

template <class C>
void dump_band(CBand& b, std::vector<int32_t>& out)
{
	if (b.DimXAlign != ref_stride<C>(b)) throw RicError(RIC_E_ARG, "DimXAlign is not the reference's");
	const C* p = (C*)b.pBand;
	const unsigned int stride = ref_stride<C>(b);
	for (unsigned int j = 0; j < b.DimY; j++)
		for (unsigned int i = 0; i < b.DimX; i++) out.push_back(p[j * stride + i]);
}

// writes through pBand (the reference's stride), then a device operation on
// the band (CBand::Add(0): the write must reach the device first) and the band
// read back through pBand: every written sample, in place
template <class C>
int poke_band(CBand& b)
{
	C* p = (C*)b.pBand;
	const unsigned int stride = ref_stride<C>(b);
	for (unsigned int j = 0; j < b.DimY; j++)
		for (unsigned int i = 0; i < b.DimX; i++) p[j * stride + i] = (C)((int)i * 3 - (int)j * 5 + 7);
	b.Add<C>(0);
	const C* q = (C*)b.pBand;
	for (unsigned int j = 0; j < b.DimY; j++)
		for (unsigned int i = 0; i < b.DimX; i++)
			if (q[j * stride + i] != (C)((int)i * 3 - (int)j * 5 + 7)) return 4;
	return 0;
}

void dump_any(CBand& b, std::vector<int32_t>& out)
{
	if (b.type == sshort) dump_band<short>(b, out); else dump_band<int>(b, out);
}

int bands(int W, int H, int Quant, trans Trans, const char* in, const char* out)
{
	std::vector<short> img = gray_plane(slurp(in), Quant);
	CWavelet2D Wavelet(W, H, kLevels, kLevels - 4);
	Wavelet.SetWeight(Trans);
	Wavelet.Transform(img.data(), W, Trans);
	std::vector<int32_t> v;
	CWavelet2D* c = &Wavelet;
	for (;;) {
		// the parent links of the pyramid (src/lib/wavelet2d.cpp:53-59)
		if (c->pLow && c->DBand.pParent != &c->pLow->DBand) return 3;
		dump_any(c->DBand, v);
		dump_any(c->HBand, v);
		dump_any(c->VBand, v);
		if (!c->pLow) break;
		c = c->pLow;
	}
	dump_any(c->LBand, v);
	std::ofstream(out, std::ios::binary).write((const char*)v.data(), v.size() * 4);
	return 0;
}

int poke(int W, int H, trans Trans, const char* in)
{
	std::vector<short> img = gray_plane(slurp(in), 9);
	CWavelet2D Wavelet(W, H, kLevels, kLevels - 4);
	Wavelet.SetWeight(Trans);
	Wavelet.Transform(img.data(), W, Trans);
	CWavelet2D* c = &Wavelet;
	while (c->pLow) c = c->pLow;
	if (int r = poke_band<short>(Wavelet.HBand)) return r;      // finest level: short
	return poke_band<int>(c->VBand);                             // coarsest: int (level_chg)
}

int stats(int W, int H, trans Trans, const char* in)
{
	std::vector<short> img = gray_plane(slurp(in), 9);
	CWavelet2D Wavelet(W, H, kLevels, kLevels - 4);
	Wavelet.SetWeight(Trans);
	Wavelet.Transform(img.data(), W, Trans);
	Wavelet.Stats();
	return 0;
}

}  // namespace

int main(int argc, char** argv)
{
	try {
		const std::string mode = argc > 1 ? argv[1] : "";
		if (mode == "enc" && argc == 8) return enc(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), (trans)atoi(argv[5]), argv[6], argv[7]);
		if (mode == "dec" && argc == 4) return dec(argv[2], argv[3]);
		if (mode == "bands" && argc == 8) return bands(atoi(argv[2]), atoi(argv[3]), atoi(argv[4]), (trans)atoi(argv[5]), argv[6], argv[7]);
		if (mode == "stats" && argc == 6) return stats(atoi(argv[2]), atoi(argv[3]), (trans)atoi(argv[4]), argv[5]);
		if (mode == "poke" && argc == 6) return poke(atoi(argv[2]), atoi(argv[3]), (trans)atoi(argv[4]), argv[5]);
	} catch (const RicError& e) {
		fprintf(stderr, "%s\n", e.what());
		return 2;
	}
	fprintf(stderr, "usage: see the header of shim_compat.cpp\n");
	return 1;
}
