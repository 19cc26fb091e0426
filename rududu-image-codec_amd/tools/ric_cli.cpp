// ric_cli.cpp -- command-line counterpart of the reference's src/ric/ric.cpp
// (Rududu Image Codec v0.2.2 options and .ric format), written against the
// drop-in C++ classes of include/rududu_gpu.hpp: CompressImage and
// DecompressImage below follow src/ric/ric.cpp:123-251 call for call.  CImg
// is replaced by 8-bit PGM/PPM I/O (P5/P6).
//
//   ric -i <input file> [-o <output file>] [-q 0..31] [-t 0|1|2] [-d] [-h]
//   (input ending in .ric => decode to .pnm, else encode to .ric)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "rududu_gpu.hpp"

using namespace rududu;

namespace {

const int kShift = 4, kQBoost = 8, kLevels = 5;   // src/ric/ric.cpp:36-39

short Quants(int idx) { return (short)ric_quants(idx); }

struct Image {                      // planar 8-bit image
	int w = 0, h = 0, c = 0;
	std::vector<short> px;          // c planes of w*h
};

bool read_pnm(const std::string& f, Image& im)
{
	std::ifstream in(f, std::ios::binary);
	if (!in) return false;
	std::string magic;
	in >> magic;
	if (magic != "P5" && magic != "P6") return false;
	auto next = [&](int& v) {
		in >> std::ws;
		while (in.peek() == '#') { std::string line; std::getline(in, line); in >> std::ws; }
		in >> v;
	};
	int maxv;
	next(im.w); next(im.h); next(maxv);
	in.get();
	if (maxv != 255) return false;
	im.c = magic == "P6" ? 3 : 1;
	std::vector<unsigned char> raw((size_t)im.w * im.h * im.c);
	in.read((char*)raw.data(), raw.size());
	if (!in) return false;
	const size_t n = (size_t)im.w * im.h;
	im.px.resize(n * im.c);
	for (size_t i = 0; i < n; i++)
		for (int k = 0; k < im.c; k++) im.px[k * n + i] = raw[i * im.c + k];
	return true;
}

bool write_pnm(const std::string& f, const Image& im)
{
	std::ofstream out(f, std::ios::binary);
	if (!out) return false;
	out << (im.c == 3 ? "P6" : "P5") << "\n" << im.w << " " << im.h << "\n255\n";
	const size_t n = (size_t)im.w * im.h;
	std::vector<unsigned char> raw(n * im.c);
	for (size_t i = 0; i < n; i++)
		for (int k = 0; k < im.c; k++) {
			const int v = im.px[k * n + i];
			raw[i * im.c + k] = (unsigned char)(v < 0 ? 0 : v > 255 ? 255 : v);
		}
	out.write((const char*)raw.data(), raw.size());
	return (bool)out;
}

// src/ric/ric.cpp:51-74
void dither(short* pIn, int width, int heigth)
{
	auto clip = [](int v) { return (short)(v < 0 ? 0 : v > 255 ? 255 : v); };
	for (int j = 0; j < heigth - 1; j++) {
		pIn[0] = clip(128 + ((pIn[0] + (1 << (kShift - 1))) >> kShift));
		for (int i = 1; i < width - 1; i++) {
			short tmp = pIn[i] + (1 << (kShift - 1));
			pIn[i] = tmp >> kShift;
			tmp -= pIn[i] << kShift;
			pIn[i + 1] += (tmp >> 1) - (tmp >> 4);
			pIn[i + width - 1] += (tmp >> 3) + (tmp >> 4);
			pIn[i + width] += (tmp >> 2) + (tmp >> 4);
			pIn[i + width + 1] += tmp >> 4;
			pIn[i] = clip(pIn[i] + 128);
		}
		pIn += width;
		pIn[-1] = clip(128 + ((pIn[-1] + (1 << (kShift - 1))) >> kShift));
	}
	for (int i = 0; i < width; i++) pIn[i] = clip(128 + ((pIn[i] + (1 << (kShift - 1))) >> kShift));
}

// src/ric/ric.cpp:123-180
void CompressImage(const std::string& infile, const std::string& outfile, int Quant, trans Trans)
{
	Image img;
	if (!read_pnm(infile, img)) throw std::runtime_error("cannot read 8-bit PGM/PPM " + infile);
	const size_t n = (size_t)img.w * img.h;
	const int color = img.c == 3;
	if (color) {                     // RGBtoYCoCg (:76-91); planes 0=Co, 1=Cg, 2=Y
		for (size_t i = 0; i < n; i++) {
			short &R = img.px[i], &G = img.px[n + i], &B = img.px[2 * n + i];
			R -= B; B += R >> 1; G -= B; B += (G >> 1) - 128;
			if (Quant) { R <<= kShift - 1; G <<= kShift - 1; B <<= kShift; }
		}
	} else {
		for (size_t i = 0; i < n; i++) img.px[i] = Quant ? (short)((img.px[i] - 128) << kShift) : (short)(img.px[i] - 128);
	}
	std::vector<unsigned char> stream(n * img.c * 2 + 65536);
	unsigned char* pStream = stream.data();
	CMuxCodec Codec(pStream, 0);                                // the reference's form (ric.cpp:157)
	CWavelet2D Wavelet(img.w, img.h, kLevels, kLevels - 4);
	Wavelet.SetWeight(Trans);
	const int planes[3] = {2, 1, 0};
	for (int k = 0; k < img.c; k++) {
		const int p = color ? planes[k] : 0, boost = k ? kQBoost : 0;
		Wavelet.Transform(img.px.data() + p * n, img.w, Trans);
		Wavelet.CodeBand(&Codec, Quant ? Quants(Quant + kShift * 5 + boost) : 0,
		                 Quant ? Quants(Quant + kShift * 5 - 7 + boost) : 0);
	}
	unsigned char* pEnd = Codec.endCoding();
	std::ofstream o(outfile, std::ios::binary);
	const unsigned char head[9] = {'R', 'U', 'D', '2', (unsigned char)(img.w & 255), (unsigned char)(img.w >> 8),
	                               (unsigned char)(img.h & 255), (unsigned char)(img.h >> 8),
	                               (unsigned char)((Quant & 31) | (color << 5) | ((int)Trans << 6))};
	o.write((const char*)head, 9);
	o.write((const char*)stream.data() + 2, pEnd - stream.data() - 2);
}

// src/ric/ric.cpp:182-251
void DecompressImage(const std::string& infile, const std::string& outfile, bool Dither)
{
	std::ifstream in(infile, std::ios::binary);
	std::vector<unsigned char> file((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
	int w, h, c, q, t;
	const int rc = ric_read_header(file.data(), file.size(), &w, &h, &c, &q, &t);
	if (rc == RIC_E_FORMAT) throw 2;                            // BAD_MAGIC
	ric_check(rc, "read header");
	const size_t n = (size_t)w * h;
	std::vector<unsigned char> stream(n * c + 2 + 16, 0);       // payload at buf + 2 (:203-205), look-ahead pad
	memcpy(stream.data() + 2, file.data() + 9, std::min(file.size() - 9, n * c));
	unsigned char* pStream = stream.data();
	CMuxCodec Codec(pStream);                                   // the reference's form (ric.cpp:207)
	CWavelet2D Wavelet(w, h, kLevels, kLevels - 4);
	Wavelet.SetWeight((trans)t);
	Image img;
	img.w = w; img.h = h; img.c = c;
	img.px.assign(n * c, 0);
	const int planes[3] = {2, 1, 0};
	for (int k = 0; k < c; k++) {
		const int p = c == 3 ? planes[k] : 0, boost = k ? kQBoost : 0;
		Wavelet.DecodeBand(&Codec);
		if (q != 0) Wavelet.TSUQi(Quants(q + kShift * 5 + boost));
		Wavelet.TransformI(img.px.data() + (p + 1) * n, w, (trans)t);
	}
	if (c == 1) {
		if (q == 0) for (auto& v : img.px) v += 128;
		else if (Dither) dither(img.px.data(), w, h);
		else for (auto& v : img.px) { v = 128 + ((v + (1 << (kShift - 1))) >> kShift); v = v < 0 ? 0 : v > 255 ? 255 : v; }
	} else {                         // YCoCgtoRGB (:93-112)
		for (size_t i = 0; i < n; i++) {
			short &R = img.px[i], &G = img.px[n + i], &B = img.px[2 * n + i];
			if (q) {
				R = (R + (1 << (kShift - 2))) >> (kShift - 1);
				G = (G + (1 << (kShift - 2))) >> (kShift - 1);
				B = (B + (1 << (kShift - 1))) >> kShift;
			}
			B -= (G >> 1) - 128; G += B; B -= R >> 1; R += B;
			if (q) { R = R < 0 ? 0 : R > 255 ? 255 : R; G = G < 0 ? 0 : G > 255 ? 255 : G; B = B < 0 ? 0 : B > 255 ? 255 : B; }
		}
	}
	if (!write_pnm(outfile, img)) throw std::runtime_error("cannot write " + outfile);
}

}  // namespace

int main(int argc, char* argv[])
{
	std::string infile, outfile;
	int Quant = 9, Trans = -1;
	bool dith = false, help = false;
	for (int i = 1; i < argc; i++) {
		std::string a = argv[i];
		if (a == "-i" && i + 1 < argc) infile = argv[++i];
		else if (a == "-o" && i + 1 < argc) outfile = argv[++i];
		else if (a == "-q" && i + 1 < argc) Quant = atoi(argv[++i]);
		else if (a == "-t" && i + 1 < argc) Trans = atoi(argv[++i]);
		else if (a == "-d") dith = true;
		else if (a == "-h" || a == "-help" || a == "--help") help = true;
	}
	if (Trans < 0) Trans = Quant == 0 ? 1 : 0;                 // :313
	if (Trans > 2) Trans = 0;
	if (Quant < 0) Quant = 0;
	if (Quant > 31) Quant = 31;
	if (infile.empty() || help) {
		std::cerr << "ric (MI355X) -- Rududu Image Codec .ric files\n"
		             "Usage: ric -i <input file> [-o <output file>] [-q 0..31] [-t 0|1|2] [-d]\n";
		return 1;
	}
	const bool decoding = infile.size() > 4 && infile.compare(infile.size() - 4, 4, ".ric") == 0;
	if (outfile.empty()) {
		outfile = infile;
		if (decoding) outfile += ".pnm";
		else {
			size_t dot = outfile.find_last_of('.'), slash = outfile.find_last_of('/');
			if (dot != std::string::npos && (slash == std::string::npos || slash < dot)) outfile.resize(dot);
			outfile += ".ric";
		}
	}
	try {
		if (decoding) DecompressImage(infile, outfile, dith);
		else CompressImage(infile, outfile, Quant, (trans)Trans);
	} catch (int e) {
		std::cerr << "bad magic\n";
		return e;
	} catch (std::exception& e) {
		std::cerr << e.what() << "\n";
		return 1;
	}
	return 0;
}
