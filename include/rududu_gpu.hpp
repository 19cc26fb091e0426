// rududu_gpu.hpp -- header-only C++ drop-in for the reference's src/lib codec
// classes on the .ric hot path, implemented over the C-ABI in ric_gpu.h.
//
// Callers written against the reference (src/ric/ric.cpp:123-251,
// src/lib/rududucodec.cpp:67-85) keep their code: same namespace, class and
// method names, argument meaning and defaults:
//
//   rududu::CMuxCodec   (src/lib/muxcodec.h:66-130)
//   rududu::CWavelet2D  (src/lib/wavelet2d.h:27-51)
//   rududu::trans / cmode / band_t  (src/lib/utils.h:27-28, band.h:35)
//
// Differences, all explicit:
//   * the band pyramid lives in GPU memory; DBand/HBand/VBand/LBand expose
//     DimX/DimY/DimXAlign/type/Weight and read() instead of a raw pBand;
//   * CMuxCodec takes an explicit capacity (the reference has none) and throws
//     rududu::RicError on overflow or on any HIP failure -- there is no CPU
//     fallback;
//   * after CodeBand the bands hold the reference's post-CodeBand state
//     (quantised sign-magnitude, the markers the zerotree scan consumes
//     cleared), so TSUQi / TransformI after CodeBand match the reference.
#pragma once

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "ric_gpu.h"

namespace rududu {

typedef enum { encode, decode } cmode;
typedef enum { cdf97 = 0, cdf53 = 1, haar = 2 } trans;
typedef enum { sshort, sint } band_t;

struct RicError : std::runtime_error {
	int status;
	RicError(int rc, const std::string& what)
		: std::runtime_error(what + " failed (status " + std::to_string(rc) + "): " + ric_last_error()), status(rc) {}
};

inline void ric_check(int rc, const char* what)
{
	if (rc != RIC_OK) throw RicError(rc, what);
}

class CMuxCodec {
public:
	// encoder: CMuxCodec(unsigned char* pStream, unsigned short firstWord)
	CMuxCodec(unsigned char* pStream, unsigned short firstWord, size_t capacity) : buf_(pStream)
	{
		ric_check(ric_mux_create_encoder(&m_, pStream, capacity, firstWord), "CMuxCodec(encoder)");
	}
	// decoder: CMuxCodec(unsigned char* pStream) -- reads from pStream + 2
	CMuxCodec(const unsigned char* pStream, size_t length) : buf_(const_cast<unsigned char*>(pStream))
	{
		ric_check(ric_mux_create_decoder(&m_, pStream, length), "CMuxCodec(decoder)");
	}
	~CMuxCodec() { ric_mux_destroy(m_); }
	CMuxCodec(const CMuxCodec&) = delete;
	CMuxCodec& operator=(const CMuxCodec&) = delete;

	unsigned char* endCoding()
	{
		size_t n = 0;
		ric_check(ric_mux_end(m_, &n), "endCoding");
		return buf_ + n;
	}
	unsigned int getSize() { return (unsigned int)ric_mux_size(m_); }
	ric_mux* handle() { return m_; }

private:
	ric_mux* m_ = nullptr;
	unsigned char* buf_;
};

class CWavelet2D;

// Read-only view of one band of the GPU-resident pyramid (CBand's public
// geometry fields, src/lib/band.h:43-59).
class CBandView {
public:
	unsigned int DimX = 0, DimY = 0, DimXAlign = 0;
	band_t type = sshort;
	float Weight = 1.f;
	// the band's values as int32, row-major DimX * DimY (copied from HBM)
	std::vector<int32_t> read() const
	{
		std::vector<int32_t> v((size_t)DimX * DimY);
		ric_check(ric_band_read(w_, index_, v.data()), "band read");
		return v;
	}
	void write(const std::vector<int32_t>& v)
	{
		ric_check(ric_band_write(w_, index_, v.data()), "band write");
	}

private:
	friend class CWavelet2D;
	ric_wavelet* w_ = nullptr;
	int index_ = 0;
};

class CWavelet2D {
public:
	// CWavelet2D(int x, int y, int level, int level_chg = 0, int Align = ALIGN)
	CWavelet2D(int x, int y, int level, int level_chg = 0, int /*Align*/ = 32, int device = 0)
		: DimX(x), DimY(y), levels_(level)
	{
		ric_check(ric_wavelet_create(&w_, x, y, level, level_chg, device), "CWavelet2D");
		nbands_ = ric_band_count(w_);
		nlev_ = (nbands_ - 1) / 3;
	}
	~CWavelet2D() { ric_wavelet_destroy(w_); }
	CWavelet2D(const CWavelet2D&) = delete;
	CWavelet2D& operator=(const CWavelet2D&) = delete;

	// Transform<short>(short* pImage, int Stride, trans t): pImage on the host
	void Transform(short* pImage, int Stride, trans t)
	{
		ric_check(ric_transform(w_, pImage, Stride, (int)t, 0), "Transform");
	}
	// TransformI<short>(short* pImageEnd, int Stride, trans t): like the
	// reference, the END pointer (image + DimY * Stride) of the host image
	void TransformI(short* pImageEnd, int Stride, trans t)
	{
		ric_check(ric_transform_inv(w_, pImageEnd - (long)DimY * Stride, Stride, (int)t, 0), "TransformI");
	}
	// device-pointer variants (images already resident in HBM)
	void TransformDevice(const short* dImage, int Stride, trans t)
	{
		ric_check(ric_transform(w_, dImage, Stride, (int)t, 1), "Transform");
	}
	void TransformIDevice(short* dImage, int Stride, trans t)
	{
		ric_check(ric_transform_inv(w_, dImage, Stride, (int)t, 1), "TransformI");
	}
	void SetWeight(trans t, float baseWeight = 1.f) { ric_check(ric_set_weight(w_, (int)t, baseWeight), "SetWeight"); }
	void CodeBand(CMuxCodec* pCodec, int Quant, int lambda)
	{
		ric_check(ric_code_band(w_, pCodec->handle(), Quant, lambda), "CodeBand");
	}
	void DecodeBand(CMuxCodec* pCodec)
	{
		const int rc = ric_decode_band(w_, pCodec->handle());
		if (rc != RIC_OK && rc != RIC_E_STREAM) ric_check(rc, "DecodeBand");
	}
	unsigned int TSUQ(int Quant, float Thres)
	{
		unsigned int n = 0;
		ric_check(ric_tsuq(w_, Quant, Thres, &n), "TSUQ");
		return n;
	}
	void TSUQi(int Quant) { ric_check(ric_tsuqi(w_, Quant), "TSUQi"); }

	// CWavelet2D::Stats (src/lib/wavelet2d.cpp:270-303): weighted band variances
	void Stats()
	{
		static const char* nm[3] = {"D", "H", "V"};
		for (int i = 0; i < nbands_; i++) {
			CBandView b = band(i);
			std::vector<int32_t> v = b.read();
			int64_t sum = 0, ssum = 0;
			for (int32_t x : v) { sum += x; ssum += (int64_t)x * x; }
			const float n = (float)b.DimX * b.DimY;
			const float var = ((float)(ssum - sum * sum)) * b.Weight * b.Weight / (n * n);
			std::printf("%s :\t%g\n", i == nbands_ - 1 ? "L" : nm[i % 3], var);
		}
	}

	// band i in canonical order: levels finest->coarsest D, H, V, then the LL
	CBandView band(int i) const
	{
		CBandView v;
		int dx, dy, isint;
		float wt;
		ric_check(ric_band_info(w_, i, &dx, &dy, &isint, &wt), "band_info");
		v.DimX = dx; v.DimY = dy; v.type = isint ? sint : sshort; v.Weight = wt;
		v.DimXAlign = ((dx * (isint ? 4 : 2) + 31) & -32) / (isint ? 4 : 2);
		v.w_ = w_; v.index_ = i;
		return v;
	}
	// the finest level's bands (DBand/HBand/VBand) and the coarsest LBand
	CBandView DBand() const { return band(0); }
	CBandView HBand() const { return band(1); }
	CBandView VBand() const { return band(2); }
	CBandView LBand() const { return band(nbands_ - 1); }
	int levels() const { return nlev_; }
	ric_wavelet* handle() { return w_; }

	const int DimX, DimY;

private:
	ric_wavelet* w_ = nullptr;
	int levels_ = 0, nbands_ = 0, nlev_ = 0;
};

}  // namespace rududu
