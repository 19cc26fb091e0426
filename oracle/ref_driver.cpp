// oracle/ref_driver.cpp -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
//
// Thin extern "C" driver around the *unmodified* reference library
// (/root/reference/src/lib/*.cpp, compiled in place by oracle/Makefile into
// oracle/_ref/libricref.so).  It restates the caller side of the reference CLI
// (src/ric/ric.cpp:123-251, CompressImage/DecompressImage) without CImg, and
// exposes band dumps so kernels can be checked stage by stage.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// the resulting library.
//
// Canonical band order used by every dump in this repo:
//   for each level from finest to coarsest: D, H, V; then the coarsest LL.
//   Each band is DimX*DimY int32 values, row-major, no padding.

#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>

#include "wavelet2d.h"

using namespace rududu;

namespace {

const int kShift = 4;     // src/ric/ric.cpp:39
const int kQBoost = 8;    // src/ric/ric.cpp:38
const int kLevels = 5;    // src/ric/ric.cpp:36

short quants(int idx)     // src/ric/ric.cpp:42-49
{
	static const unsigned short Q[5] = {0x8000, 0x9000, 0xA800, 0xC000, 0xE000};
	if (idx <= 0) return 0;
	idx--;
	int r = 14 - idx / 5;
	return (short)((Q[idx % 5] + (1 << (r - 1))) >> r);
}

template <class C>
void dump_band(const CBand& b, int32_t*& out)
{
	const C* p = (const C*)b.pBand;
	for (unsigned j = 0; j < b.DimY; j++)
		for (unsigned i = 0; i < b.DimX; i++)
			*out++ = (int32_t)p[j * b.DimXAlign + i];
}

void dump_any(const CBand& b, int32_t*& out)
{
	if (b.type == sshort) dump_band<short>(b, out); else dump_band<int>(b, out);
}

long dump_all(CWavelet2D& w, int32_t* out)
{
	int32_t* o = out;
	CWavelet2D* c = &w;
	while (true) {
		dump_any(c->DBand, o);
		dump_any(c->HBand, o);
		dump_any(c->VBand, o);
		if (!c->pLow) break;
		c = c->pLow;
	}
	dump_any(c->LBand, o);
	return (long)(o - out);
}

// Mirrors the first half of CWavelet2D::CodeBand (src/lib/wavelet2d.cpp:110-126):
// buildTree on the finest D/H/V (recursing to parents) and TSUQ on the LL.
void build_tree_only(CWavelet2D& w, int quant, int lambda)
{
	if (w.DBand.type == sshort) {
		w.DBand.buildTree<true, short>(quant, lambda);
		w.HBand.buildTree<true, short>(quant, lambda);
		w.VBand.buildTree<true, short>(quant, lambda);
	} else {
		w.DBand.buildTree<true, int>(quant, lambda);
		w.HBand.buildTree<true, int>(quant, lambda);
		w.VBand.buildTree<true, int>(quant, lambda);
	}
	CWavelet2D* c = &w;
	while (c->pLow) c = c->pLow;
	if (c->LBand.type == sshort) c->LBand.TSUQ<short>(quant, 0.5f);
	else c->LBand.TSUQ<int>(quant, 0.5f);
}

}  // namespace

extern "C" {

// Band geometry: writes (dimx, dimy, is_int) triples in canonical order.
// Returns the number of bands.
int ricref_layout(int w, int h, int levels, int lc, int32_t* out)
{
	CWavelet2D wav(w, h, levels, lc);
	CWavelet2D* c = &wav;
	int n = 0;
	auto put = [&](const CBand& b) {
		if (out) { out[3*n] = b.DimX; out[3*n+1] = b.DimY; out[3*n+2] = b.type == sint; }
		n++;
	};
	while (true) {
		put(c->DBand); put(c->HBand); put(c->VBand);
		if (!c->pLow) break;
		c = c->pLow;
	}
	put(c->LBand);
	return n;
}

// Forward transform of one int16 plane; dumps all bands.  stage: 0 = after
// Transform, 1 = after buildTree + LL TSUQ, 2 = after the whole CodeBand.
long ricref_bands(const int16_t* img, int w, int h, int levels, int lc, int trans,
                  int stage, int quant, int lambda, int32_t* out)
{
	std::vector<short> buf(img, img + (size_t)w * h);
	CWavelet2D wav(w, h, levels, lc);
	wav.SetWeight((rududu::trans)trans);
	wav.Transform(buf.data(), w, (rududu::trans)trans);
	if (stage == 1) build_tree_only(wav, quant, lambda);
	if (stage == 2) {
		std::vector<unsigned char> s((size_t)w * h * 4 + 4096);
		CMuxCodec codec(s.data(), 0);
		wav.CodeBand(&codec, quant, lambda);
	}
	return dump_all(wav, out);
}

// The video driver's closed loop on one plane (src/lib/rududucodec.cpp:67-74):
// Transform, CodeBand, TSUQi on the bands CodeBand left, TransformI.  Dumps
// the bands after TSUQi (bands_out, optional) and the reconstructed plane.
long ricref_closed_loop(const int16_t* img, int w, int h, int levels, int lc, int trans, int quant, int lambda,
                        int dq, int16_t* plane_out, int32_t* bands_out)
{
	const size_t n = (size_t)w * h;
	std::vector<short> buf(img, img + n);
	CWavelet2D wav(w, h, levels, lc);
	wav.SetWeight((rududu::trans)trans);
	wav.Transform(buf.data(), w, (rududu::trans)trans);
	std::vector<unsigned char> s(n * 4 + 4096);
	CMuxCodec codec(s.data(), 0);
	wav.CodeBand(&codec, quant, lambda);
	wav.TSUQi(dq);
	long nb = bands_out ? dump_all(wav, bands_out) : 0;
	std::fill(buf.begin(), buf.end(), 0);
	wav.TransformI(buf.data() + n, w, (rududu::trans)trans);
	std::copy(buf.begin(), buf.end(), plane_out);
	return nb;
}

// CWavelet2D::Stats' numbers (src/lib/wavelet2d.cpp:270-303): CBand::Mean's
// variance of every band after Transform (SetWeight(trans) weights),
// canonical order.  Returns the number of bands.
long ricref_stats(const int16_t* img, int w, int h, int levels, int lc, int trans, float* var_out)
{
	std::vector<short> buf(img, img + (size_t)w * h);
	CWavelet2D wav(w, h, levels, lc);
	wav.SetWeight((rududu::trans)trans);
	wav.Transform(buf.data(), w, (rududu::trans)trans);
	long n = 0;
	auto one = [&](CBand& b) {
		float mean = 0, var = 0;
		if (b.type == sshort) b.Mean<short>(mean, var); else b.Mean<int>(mean, var);
		var_out[n++] = var;
	};
	CWavelet2D* c = &wav;
	while (true) {
		one(c->DBand); one(c->HBand); one(c->VBand);
		if (!c->pLow) break;
		c = c->pLow;
	}
	one(c->LBand);
	return n;
}

// Encodes nplanes int16 planes (coded in the given order) into one stream.
// Returns the full coder buffer length (endCoding() - buf, including the two
// leading bytes that the .ric file drops), or -needed if cap is too small.
long ricref_encode_planes(const int16_t* planes, int nplanes, int w, int h, int levels,
                          int lc, int trans, const int* quant, const int* lambda,
                          uint8_t* out, long cap)
{
	size_t n = (size_t)w * h;
	std::vector<unsigned char> s(n * nplanes * 4 + 4096, 0);
	CMuxCodec codec(s.data(), 0);
	CWavelet2D wav(w, h, levels, lc);
	wav.SetWeight((rududu::trans)trans);
	std::vector<short> buf(n);
	for (int p = 0; p < nplanes; p++) {
		std::copy(planes + p * n, planes + (p + 1) * n, buf.begin());
		wav.Transform(buf.data(), w, (rududu::trans)trans);
		wav.CodeBand(&codec, quant[p], lambda[p]);
	}
	unsigned char* end = codec.endCoding();
	long len = (long)(end - s.data());
	if (len > cap) return -len;
	memcpy(out, s.data(), len);
	return len;
}

// Decodes nplanes planes from a full coder buffer (as produced by
// ricref_encode_planes).  quant[p] == 0 skips TSUQi (lossless), as
// src/ric/ric.cpp:213 does.  Optional band dump of the last plane after
// DecodeBand (before TSUQi).
long ricref_decode_planes(const uint8_t* in, long len, int nplanes, int w, int h, int levels,
                          int lc, int trans, const int* quant, int16_t* planes_out,
                          int32_t* bands_out)
{
	size_t n = (size_t)w * h;
	std::vector<unsigned char> s(std::max<size_t>(len, 0) + n * nplanes + 4096, 0);
	memcpy(s.data(), in, len);
	CMuxCodec codec(s.data());
	CWavelet2D wav(w, h, levels, lc);
	wav.SetWeight((rududu::trans)trans);
	std::vector<short> buf(n);
	for (int p = 0; p < nplanes; p++) {
		wav.DecodeBand(&codec);
		if (bands_out && p == nplanes - 1) dump_all(wav, bands_out);
		if (quant[p] != 0) wav.TSUQi(quant[p]);
		std::fill(buf.begin(), buf.end(), 0);
		wav.TransformI(buf.data() + n, w, (rududu::trans)trans);
		std::copy(buf.begin(), buf.end(), planes_out + p * n);
	}
	return 0;
}

// Whole-file encode, restating CompressImage (src/ric/ric.cpp:123-180).
// pix: channels planes of w*h bytes (R,G,B planar for colour).
long ricref_encode_ric(const uint8_t* pix, int w, int h, int channels, int q, int trans,
                       uint8_t* out, long cap)
{
	size_t n = (size_t)w * h;
	std::vector<short> img(n * channels);
	for (size_t i = 0; i < n * channels; i++) img[i] = pix[i];
	int color = channels == 3;
	if (color) {  // RGBtoYCoCg, src/ric/ric.cpp:76-91
		for (size_t i = 0; i < n; i++) {
			short& R = img[i]; short& G = img[n + i]; short& B = img[2 * n + i];
			R -= B; B += R >> 1; G -= B; B += (G >> 1) - 128;
			if (q != 0) { R <<= kShift - 1; G <<= kShift - 1; B <<= kShift; }
		}
	} else {
		for (size_t i = 0; i < n; i++)
			img[i] = q == 0 ? (short)(img[i] - 128) : (short)((img[i] - 128) << kShift);
	}
	std::vector<int16_t> planes;
	std::vector<int> qs, ls;
	if (color) {
		const int order[3] = {2, 1, 0};
		for (int k = 0; k < 3; k++) {
			int p = order[k];
			planes.insert(planes.end(), img.begin() + p * n, img.begin() + (p + 1) * n);
			int boost = k ? kQBoost : 0;
			qs.push_back(q ? quants(q + kShift * 5 + boost) : 0);
			ls.push_back(q ? quants(q + kShift * 5 - 7 + boost) : 0);
		}
	} else {
		planes = std::vector<int16_t>(img.begin(), img.end());
		qs.push_back(q ? quants(q + kShift * 5) : 0);
		ls.push_back(q ? quants(q + kShift * 5 - 7) : 0);
	}
	std::vector<uint8_t> s(n * channels * 4 + 4096);
	long len = ricref_encode_planes(planes.data(), channels, w, h, kLevels, kLevels - 4, trans,
	                                qs.data(), ls.data(), s.data(), (long)s.size());
	long total = 9 + len - 2;
	if (total > cap) return -total;
	memcpy(out, "RUD2", 4);
	out[4] = w & 255; out[5] = w >> 8; out[6] = h & 255; out[7] = h >> 8;
	out[8] = (uint8_t)((q & 31) | (color << 5) | ((trans & 3) << 6));
	memcpy(out + 9, s.data() + 2, len - 2);
	return total;
}

// Whole-file decode, restating DecompressImage (src/ric/ric.cpp:182-251).
// Writes the int16 planes before the final 8-bit conversion (planes_out, may be
// null) and the 8-bit planes clipped to [0,255] (pix_out).  Returns 0, or -2
// on a bad magic (the reference throws BAD_MAGIC = 2).
long ricref_decode_ric(const uint8_t* ric, long len, int dither_on, int16_t* planes_out,
                       uint8_t* pix_out, int32_t* dims)
{
	if (len < 9 || memcmp(ric, "RUD2", 4) != 0) return -2;
	int w = ric[4] | (ric[5] << 8), h = ric[6] | (ric[7] << 8);
	int q = ric[8] & 31, color = (ric[8] >> 5) & 1, trans = (ric[8] >> 6) & 3;
	int channels = color ? 3 : 1;
	if (dims) { dims[0] = w; dims[1] = h; dims[2] = channels; dims[3] = q; dims[4] = trans; }
	if (!pix_out && !planes_out) return 0;
	size_t n = (size_t)w * h;
	// the reference reads W*H*C bytes at buf+2 (src/ric/ric.cpp:203-205)
	std::vector<uint8_t> s(n * channels + 4096, 0);
	long pay = std::min<long>(len - 9, (long)(n * channels));
	memcpy(s.data() + 2, ric + 9, pay);
	std::vector<int16_t> dec(n * channels);
	std::vector<int> qs;
	if (color) {
		qs.push_back(q ? quants(q + kShift * 5) : 0);
		qs.push_back(q ? quants(q + kShift * 5 + kQBoost) : 0);
		qs.push_back(q ? quants(q + kShift * 5 + kQBoost) : 0);
	} else {
		qs.push_back(q ? quants(q + kShift * 5) : 0);
	}
	ricref_decode_planes(s.data(), (long)s.size(), channels, w, h, kLevels, kLevels - 4, trans,
	                     qs.data(), dec.data(), nullptr);
	// decoded stream order is Y, Cg, Co -> planar index 2, 1, 0
	std::vector<short> img(n * channels);
	if (color) {
		for (int k = 0; k < 3; k++)
			std::copy(dec.begin() + k * n, dec.begin() + (k + 1) * n, img.begin() + (2 - k) * n);
	} else {
		std::copy(dec.begin(), dec.end(), img.begin());
	}
	if (!color) {
		if (q == 0) {
			for (size_t i = 0; i < n; i++) img[i] += 128;
		} else if (dither_on) {  // dither(), src/ric/ric.cpp:51-74
			short* pIn = img.data();
			int width = w, heigth = h;
			for (int j = 0; j < heigth - 1; j++) {
				pIn[0] = 128 + ((pIn[0] + (1 << (kShift - 1))) >> kShift);
				pIn[0] = std::min<short>(std::max<short>(pIn[0], 0), 255);
				for (int i = 1; i < width - 1; i++) {
					short tmp = pIn[i] + (1 << (kShift - 1));
					pIn[i] = tmp >> kShift;
					tmp -= pIn[i] << kShift;
					pIn[i + 1] += (tmp >> 1) - (tmp >> 4);
					pIn[i + width - 1] += (tmp >> 3) + (tmp >> 4);
					pIn[i + width] += (tmp >> 2) + (tmp >> 4);
					pIn[i + width + 1] += tmp >> 4;
					pIn[i] = std::min(std::max(pIn[i] + 128, 0), 255);
				}
				pIn += width;
				pIn[-1] = 128 + ((pIn[-1] + (1 << (kShift - 1))) >> kShift);
				pIn[-1] = std::min<short>(std::max<short>(pIn[-1], 0), 255);
			}
			for (int i = 0; i < width; i++) {
				pIn[i] = 128 + ((pIn[i] + (1 << (kShift - 1))) >> kShift);
				pIn[i] = std::min<short>(std::max<short>(pIn[i], 0), 255);
			}
		} else {
			for (size_t i = 0; i < n; i++) {
				short v = 128 + ((img[i] + (1 << (kShift - 1))) >> kShift);
				img[i] = std::min<short>(std::max<short>(v, 0), 255);
			}
		}
	} else {  // YCoCgtoRGB, src/ric/ric.cpp:93-112
		for (size_t i = 0; i < n; i++) {
			short& R = img[i]; short& G = img[n + i]; short& B = img[2 * n + i];
			if (q != 0) {
				R = (R + (1 << (kShift - 2))) >> (kShift - 1);
				G = (G + (1 << (kShift - 2))) >> (kShift - 1);
				B = (B + (1 << (kShift - 1))) >> kShift;
			}
			B -= (G >> 1) - 128; G += B; B -= R >> 1; R += B;
			if (q != 0) {
				R = std::min<short>(std::max<short>(R, 0), 255);
				G = std::min<short>(std::max<short>(G, 0), 255);
				B = std::min<short>(std::max<short>(B, 0), 255);
			}
		}
	}
	if (planes_out) std::copy(img.begin(), img.end(), planes_out);
	if (pix_out)
		for (size_t i = 0; i < n * channels; i++)
			pix_out[i] = (uint8_t)std::min(std::max((int)img[i], 0), 255);
	return 0;
}

}  // extern "C"
