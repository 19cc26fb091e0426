// rududu_gpu.hpp -- header-only C++ drop-in for the reference's src/lib codec
// classes on the .ric hot path, implemented over the C-ABI in ric_gpu.h.
//
// Callers written against the reference (src/ric/ric.cpp:123-251,
// src/lib/rududucodec.cpp:67-85) keep their code: same namespace, class and
// member names, constructor forms, argument meaning and defaults:
//
//   rududu::CMuxCodec   (src/lib/muxcodec.h:66-130)
//   rududu::CWavelet2D  (src/lib/wavelet2d.h:27-51): DBand/HBand/VBand/LBand,
//                       pLow/pHigh, Transform/TransformI/CodeBand/DecodeBand/
//                       TSUQ/TSUQi/SetWeight/Stats
//   rududu::CBand / CBandCodec (src/lib/band.h:37-161): the public fields
//                       DimX..type, pParent/pChild, pBand, Mean/TSUQ/TSUQi/
//                       Add/Clear/GetBand
//   rududu::trans / cmode / band_t  (src/lib/utils.h:27-28, band.h:35)
//   rududu::CRududuCodec (src/lib/rududucodec.h:31-55) and the CImage caller
//                       container (src/lib/image.h:30-66): the video codec
//
// What differs, and why:
//   * the pyramid lives in GPU memory.  CBand::pBand converts (C-style cast,
//     `(short*) band.pBand`) to a pointer into a host copy of the band in the
//     reference's layout -- row stride DimXAlign = DimX rounded up to 32 bytes
//     (CBand::Init, src/lib/band.cpp:57) -- synced from the device on that
//     conversion (ric_band_host_ref); writes through it are what the next GPU
//     operation on the pyramid reads.  The pointer stays the band's (stable);
//     its contents are current after the conversion and after CodeBand /
//     DecodeBand, not after a device-side band operation (convert again).
//   * every failure (HIP error, no GPU, stream capacity) throws
//     rududu::RicError: there is no CPU fallback.
//   * the sub-level CWavelet2D objects of the pLow chain are views of the one
//     pyramid: their bands and Stats are theirs, the transform / coding
//     methods act on the whole pyramid and are called on the top object, as
//     every reference caller does.
//   * after CodeBand the bands hold the reference's post-CodeBand state
//     (quantised sign-magnitude, the markers the zerotree scan consumes
//     cleared), so TSUQi / TransformI after CodeBand match the reference.
#pragma once

#include <cstdint>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <utility>
#include <iostream>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "ric_gpu.h"

namespace rududu {

typedef enum { encode, decode } cmode;
typedef enum { cdf97 = 0, cdf53 = 1, haar = 2 } trans;
typedef enum { sshort, sint } band_t;

#ifndef ALIGN
#define ALIGN 32
#endif

struct RicError : std::runtime_error {
	int status;
	RicError(int rc, const std::string& what)
		: std::runtime_error(what + " failed (status " + std::to_string(rc) + "): " + ric_last_error()), status(rc) {}
};

inline void ric_check(int rc, const char* what)
{
	if (rc != RIC_OK) throw RicError(rc, what);
}

// tag of the bounded decoder constructor
struct bounded_t {};
constexpr bounded_t bounded{};

class CMuxCodec {
public:
	// CMuxCodec(unsigned char* pStream, unsigned short firstWord): encoder
	// (src/lib/muxcodec.h:102).  Like the reference it takes no capacity and
	// writes pStream in place -- the caller's buffer must hold the stream, as
	// with the reference.  CMuxCodec(0, 0) (src/lib/rududucodec.cpp:36) is a
	// coder without a buffer until initCoder / initDecoder give it one.
	CMuxCodec(unsigned char* pStream, unsigned short firstWord) : buf_(pStream)
	{
		ric_check(ric_mux_create_encoder(&m_, pStream, pStream ? SIZE_MAX : 0, firstWord), "CMuxCodec(encoder)");
	}
	// the bounded encoder: writes pStream directly, at most capacity bytes
	CMuxCodec(unsigned char* pStream, unsigned short firstWord, size_t capacity) : buf_(pStream)
	{
		ric_check(ric_mux_create_encoder(&m_, pStream, capacity, firstWord), "CMuxCodec(encoder)");
	}
	// CMuxCodec(unsigned char* pStream): decoder reading from pStream + 2 in
	// place, with no end, like the reference (src/lib/muxcodec.h:103)
	explicit CMuxCodec(const unsigned char* pStream) : buf_(const_cast<unsigned char*>(pStream))
	{
		ric_check(ric_mux_create_decoder_inplace(&m_, pStream), "CMuxCodec(decoder)");
	}
	// the bounded decoder: `length` bytes of pStream (payload at pStream + 2)
	CMuxCodec(const unsigned char* pStream, size_t length, bounded_t) : buf_(const_cast<unsigned char*>(pStream))
	{
		ric_check(ric_mux_create_decoder(&m_, pStream, length), "CMuxCodec(decoder)");
	}
	~CMuxCodec() { ric_mux_destroy(m_); }
	CMuxCodec(const CMuxCodec&) = delete;
	CMuxCodec& operator=(const CMuxCodec&) = delete;

	// CMuxCodec::initCoder(unsigned short firstWord, unsigned char* pStream)
	// (src/lib/muxcodec.h:104): restart as an encoder; pStream 0 keeps the
	// output position, as in the reference
	void initCoder(unsigned short firstWord, unsigned char* pStream)
	{
		ric_check(ric_mux_reinit_encoder(m_, pStream, SIZE_MAX, firstWord), "initCoder");
		if (pStream) buf_ = pStream;
	}
	// the bounded form: at most capacity bytes at pStream
	void initCoder(unsigned short firstWord, unsigned char* pStream, size_t capacity)
	{
		ric_check(ric_mux_reinit_encoder(m_, pStream, capacity, firstWord), "initCoder");
		if (pStream) buf_ = pStream;
	}
	// CMuxCodec::initDecoder(unsigned char* pStream) (src/lib/muxcodec.h:105):
	// restart as a decoder reading pStream + 2 in place, like the reference
	void initDecoder(const unsigned char* pStream)
	{
		ric_check(ric_mux_reinit_decoder(m_, pStream, 0), "initDecoder");
		if (pStream) buf_ = const_cast<unsigned char*>(pStream);
	}
	// the bounded form: `length` bytes of pStream
	void initDecoder(const unsigned char* pStream, size_t length, bounded_t)
	{
		ric_check(ric_mux_reinit_decoder(m_, pStream, length), "initDecoder");
		if (pStream) buf_ = const_cast<unsigned char*>(pStream);
	}

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

// CBand::pBand: converts to a typed pointer into the band's host mirror
// (synced from the device on conversion; see the header comment)
class BandData {
public:
	template <class T> operator T*() const
	{
		if (!w_) return nullptr;
		void* p = nullptr;
		int stride = 0;
		ric_check(ric_band_host_ref(w_, index_, &p, &stride), "CBand::pBand");
		return (T*)p;
	}
	explicit operator bool() const { return w_ != nullptr; }

private:
	friend class CWavelet2D;
	friend class CBand;
	ric_wavelet* w_ = nullptr;
	int index_ = 0;
};

// CBand, src/lib/band.h:37-161: one band of the GPU-resident pyramid
class CBand {
public:
	unsigned int DimX = 0;       // width of the band
	unsigned int DimY = 0;       // height
	unsigned int DimXAlign = 0;  // row stride of pBand (samples)
	unsigned int BandSize = 0;   // DimXAlign * DimY
	int Max = 0, Min = 0;        // set by TSUQ (band level)
	unsigned int Dist = 0;
	unsigned int Count = 0;      // set by TSUQ (band level)
	float Weight = 1.f;
	CBand* pParent = nullptr;    // the same band one level coarser
	CBand* pChild = nullptr;     // the same band one level finer
	CBand* pNeighbor[3] = {nullptr, nullptr, nullptr};
	BandData pBand;
	band_t type = sshort;

	// src/lib/band.h:65-92, on the device (ric_band_tsuq)
	template <class C> unsigned int TSUQ(int Quant, float Thres)
	{
		unsigned int n = 0;
		int mx = 0, mn = 0;
		ric_check(ric_band_tsuq(pBand.w_, pBand.index_, Quant, Thres, &n, &mx, &mn), "CBand::TSUQ");
		Count = n;
		Max = mx;
		Min = mn;
		return Count;
	}
	// src/lib/band.h:94-107, on the device
	template <class C> void TSUQi(C Quant) { ric_check(ric_band_tsuqi(pBand.w_, pBand.index_, (int)Quant), "CBand::TSUQi"); }
	// src/lib/band.h:116-132: the sums on the device (the reference's
	// arithmetic: int products, int64 sums), then its float formula with the
	// sample-count square in unsigned (both wrap on big bands)
	template <class C> void Mean(float& Mean, float& Var)
	{
		int64_t Sum = 0, SSum = 0;
		ric_check(ric_band_sums(pBand.w_, pBand.index_, &Sum, &SSum), "CBand::Mean");
		const unsigned int n = DimX * DimY;
		Mean = (float)Sum * Weight / n;
		Var = ((float)(SSum - Sum * Sum)) * Weight * Weight / (n * n);
	}
	// src/lib/band.h:135-141, on the device (every sample of the rows)
	template <class C> void Add(C val) { ric_check(ric_band_add(pBand.w_, pBand.index_, (int)val), "CBand::Add"); }
	// src/lib/band.cpp:162-167 (recurse: the finer bands too), on the device
	void Clear(bool recurse = false)
	{
		if (!pBand) return;
		ric_check(ric_band_clear(pBand.w_, pBand.index_), "CBand::Clear");
		if (recurse && pChild) pChild->Clear(true);
	}
	// src/lib/band.h:145-155
	template <class C, class T> void GetBand(T* pOut)
	{
		const C* pIn = (const C*)pBand;
		const int add = 1 << (sizeof(T) * 8 - 1);
		for (unsigned int j = 0; j < DimY; j++, pOut += DimX, pIn += DimXAlign)
			for (unsigned int i = 0; i < DimX; i++) pOut[i] = (T)(pIn[i] + add);
	}

	// the band's values as int32, row-major DimX * DimY
	std::vector<int32_t> read() const
	{
		std::vector<int32_t> v((size_t)DimX * DimY);
		ric_check(ric_band_read(pBand.w_, pBand.index_, v.data()), "band read");
		return v;
	}
	void write(const std::vector<int32_t>& v)
	{
		ric_check(ric_band_write(pBand.w_, pBand.index_, v.data()), "band write");
	}
};

// the reference's CBandCodec adds the band coder to CBand; here the coder
// runs inside CodeBand / DecodeBand and the band's public face is CBand's
typedef CBand CBandCodec;

class CWavelet2D {
public:
	// CWavelet2D(int x, int y, int level, int level_chg = 0, int Align = ALIGN)
	CWavelet2D(int x, int y, int level, int level_chg = 0, int /*Align*/ = ALIGN, int device = 0)
		: DimX(x), DimY(y)
	{
		ric_check(ric_wavelet_create(&w_, x, y, level, level_chg, device), "CWavelet2D");
		const int nb = ric_band_count(w_);
		const int nlev = (nb - 1) / 3;
		// the pLow chain: one view per level (src/lib/wavelet2d.cpp:47-81)
		CWavelet2D* cur = this;
		for (int l = 0; l < nlev; l++) {
			cur->w_ = w_;
			cur->level_ = l;
			cur->bind(cur->DBand, 3 * l + 0);
			cur->bind(cur->HBand, 3 * l + 1);
			cur->bind(cur->VBand, 3 * l + 2);
			if (l + 1 < nlev) {
				CWavelet2D* low = new CWavelet2D(cur);
				cur->pLow = low;
				cur = low;
			}
		}
		cur->bind(cur->LBand, nb - 1);
		// parents: the same band one level coarser (src/lib/wavelet2d.cpp:53-59)
		for (CWavelet2D* c = this; c->pLow; c = c->pLow) {
			c->DBand.pParent = &c->pLow->DBand; c->pLow->DBand.pChild = &c->DBand;
			c->HBand.pParent = &c->pLow->HBand; c->pLow->HBand.pChild = &c->HBand;
			c->VBand.pParent = &c->pLow->VBand; c->pLow->VBand.pChild = &c->VBand;
		}
	}
	~CWavelet2D()
	{
		delete pLow;
		if (!pHigh) ric_wavelet_destroy(w_);
	}
	CWavelet2D(const CWavelet2D&) = delete;
	CWavelet2D& operator=(const CWavelet2D&) = delete;

	// Transform<short>(short* pImage, int Stride, trans t): pImage on the host
	void Transform(short* pImage, int Stride, trans t)
	{
		ric_check(ric_transform(top(), pImage, Stride, (int)t, 0), "Transform");
	}
	// TransformI<short>(short* pImageEnd, int Stride, trans t): like the
	// reference, the END pointer (image + DimY * Stride) of the host image
	void TransformI(short* pImageEnd, int Stride, trans t)
	{
		ric_check(ric_transform_inv(top(), pImageEnd - (long)DimY * Stride, Stride, (int)t, 0), "TransformI");
	}
	// device-pointer variants (images already resident in HBM)
	void TransformDevice(const short* dImage, int Stride, trans t)
	{
		ric_check(ric_transform(top(), dImage, Stride, (int)t, 1), "Transform");
	}
	void TransformIDevice(short* dImage, int Stride, trans t)
	{
		ric_check(ric_transform_inv(top(), dImage, Stride, (int)t, 1), "TransformI");
	}
	void SetWeight(trans t, float baseWeight = 1.f)
	{
		ric_check(ric_set_weight(top(), (int)t, baseWeight), "SetWeight");
		refresh_weights();
	}
	void CodeBand(CMuxCodec* pCodec, int Quant, int lambda)
	{
		ric_check(ric_code_band(top(), pCodec->handle(), Quant, lambda), "CodeBand");
	}
	void DecodeBand(CMuxCodec* pCodec)
	{
		const int rc = ric_decode_band(top(), pCodec->handle());
		if (rc != RIC_OK && rc != RIC_E_STREAM) ric_check(rc, "DecodeBand");
	}
	unsigned int TSUQ(int Quant, float Thres)
	{
		unsigned int n = 0;
		ric_check(ric_tsuq(top(), Quant, Thres, &n), "TSUQ");
		return n;
	}
	void TSUQi(int Quant) { ric_check(ric_tsuqi(top(), Quant), "TSUQi"); }

	// CWavelet2D::Stats (src/lib/wavelet2d.cpp:270-303): band variances, D H V
	// per level from this one down, then the coarsest L (CBand::Mean arithmetic)
	void Stats()
	{
		float Mean = 0, Var = 0;
		const char* nm[3] = {"D", "H", "V"};
		CBand* b[3] = {&DBand, &HBand, &VBand};
		for (int k = 0; k < 3; k++) {
			if (b[k]->type == sshort) b[k]->Mean<short>(Mean, Var); else b[k]->Mean<int>(Mean, Var);
			std::cout << nm[k] << " :\t" << Var << std::endl;
		}
		if (pLow) {
			pLow->Stats();
		} else {
			if (LBand.type == sshort) LBand.Mean<short>(Mean, Var); else LBand.Mean<int>(Mean, Var);
			std::cout << "L" << " :\t" << Var << std::endl;
		}
	}

	CBandCodec DBand;
	CBandCodec HBand;
	CBandCodec VBand;
	CBandCodec LBand;
	CWavelet2D* pLow = nullptr;
	CWavelet2D* pHigh = nullptr;

	int levels() const { int n = 1; for (const CWavelet2D* c = this; c->pLow; c = c->pLow) n++; return n; }
	ric_wavelet* handle() { return w_; }

	const int DimX, DimY;

private:
	explicit CWavelet2D(CWavelet2D* high) : pHigh(high), DimX(0), DimY(0) {}
	ric_wavelet* top()
	{
		if (pHigh) throw RicError(RIC_E_ARG, "CWavelet2D: call on the top of the pLow chain");
		return w_;
	}
	void bind(CBand& b, int index)
	{
		int dx, dy, isint;
		float wt;
		ric_check(ric_band_info(w_, index, &dx, &dy, &isint, &wt), "band_info");
		b.DimX = dx; b.DimY = dy; b.type = isint ? sint : sshort; b.Weight = wt;
		// CBand::Init (src/lib/band.cpp:57): DimX * sample size rounded up to ALIGN (32) bytes
		const int ss = isint ? 4 : 2;
		b.DimXAlign = (unsigned int)(((dx * ss + 31) & -32) / ss);
		b.BandSize = b.DimXAlign * dy;
		b.pBand.w_ = w_;
		b.pBand.index_ = index;
	}
	void refresh_weights()
	{
		for (CWavelet2D* c = this; c; c = c->pLow) {
			CBand* bs[4] = {&c->DBand, &c->HBand, &c->VBand, &c->LBand};
			for (CBand* b : bs) {
				if (!b->pBand) continue;
				int dx, dy, isint;
				float wt;
				ric_check(ric_band_info(w_, b->pBand.index_, &dx, &dy, &isint, &wt), "band_info");
				b->Weight = wt;
			}
		}
	}
	ric_wavelet* w_ = nullptr;
	int level_ = 0;
};

// CImage (src/lib/image.h:30-66): the caller's image container, host planes in
// the reference's layout -- dimXAlign = (x + 2 BORDER + Align - 1) & -Align
// samples per row, BORDER rows and columns of border, planes back to back
// (image.cpp:56-68).  The codec's own images live in HBM (ric_video); the
// CImage a CRududuCodec call hands back is a host copy of its output image,
// border included.  The pixel helpers are the reference's caller-side
// conversions (image.cpp:70-278).
#ifndef BORDER
#define BORDER 15
#endif
class CImage {
public:
	unsigned int dimX = 0, dimY = 0, dimXAlign = 0;
	int component = 0;
	short* pImage[3] = {nullptr, nullptr, nullptr};

	CImage(unsigned int x, unsigned int y, int cmpnt, int Align) : dimX(x), dimY(y), component(cmpnt) { init(Align); }
	CImage(CImage* pImg, int Align) : dimX(pImg->dimX), dimY(pImg->dimY), component(pImg->component) { init(Align); }

	// image.cpp:96-123: planes R, G, B (stride bytes per row, bottom row
	// first) -> Y, Co, Cg; 8-bit input is scaled (Y << 4, Co / Cg << 3)
	template <class input_t> void inputSGI(input_t* pIn, int stride, short offset)
	{
		const long ps = (long)stride * dimY;
		for (unsigned int j = 0; j < dimY; j++) {
			const input_t* R = pIn + (long)(dimY - 1 - j) * stride;
			const input_t* G = R + ps;
			const input_t* B = G + ps;
			short *Y = pImage[0] + (long)j * dimXAlign, *Co = pImage[1] + (long)j * dimXAlign,
			      *Cg = pImage[2] + (long)j * dimXAlign;
			for (unsigned int i = 0; i < dimX; i++) {
				Co[i] = (short)(R[i] - B[i]);
				Y[i] = (short)(B[i] + (Co[i] >> 1));
				Cg[i] = (short)(G[i] - Y[i]);
				Y[i] = (short)(Y[i] + (Cg[i] >> 1) + offset);
				if (sizeof(input_t) == 1) {
					Y[i] = (short)(Y[i] * 16);
					Co[i] = (short)(Co[i] * 8);
					Cg[i] = (short)(Cg[i] * 8);
				}
			}
		}
	}
	// image.cpp:148-185 (reads one sample right of / below odd-sized images)
	template <class output_t, bool i420> void outputYV12(output_t* pOut, int stride, short offset)
	{
		output_t* Yo = pOut;
		output_t* Vo = Yo + (long)stride * dimY;
		output_t* Uo = Vo + (((long)stride * dimY) >> 2);
		const int shift = 12 - (int)sizeof(output_t) * 8;
		if (sizeof(output_t) == 1) offset = (short)(offset * 16);
		else if (sizeof(output_t) == 2) offset = (short)(offset >> 4);
		if (i420) std::swap(Uo, Vo);
		const long S = dimXAlign;
		for (unsigned int j = 0; j < dimY; j += 2) {
			const short *Y = pImage[0] + j * S, *Co = pImage[1] + j * S, *Cg = pImage[2] + j * S;
			for (unsigned int i = 0; i < dimX; i += 2) {
				auto luma = [&](long k) {
					return (output_t)(((440 * (Y[k] - offset) + 82 * Co[k] + 76 * Cg[k] + (1 << (8 + shift))) >> (9 + shift)) + 16);
				};
				Yo[i] = luma(i);
				Yo[i + 1] = luma(i + 1);
				Yo[i + stride] = luma(i + S);
				Yo[i + stride + 1] = luma(i + S + 1);
				const int co = Co[i] + Co[i + 1] + Co[i + S] + Co[i + S + 1];
				const int cg = Cg[i] + Cg[i + 1] + Cg[i + S] + Cg[i + S + 1];
				Uo[i >> 1] = (output_t)(((-150 * co - 148 * cg + (1 << (9 + shift))) >> (10 + shift)) + 128);
				Vo[i >> 1] = (output_t)(((130 * co - 188 * cg + (1 << (9 + shift))) >> (10 + shift)) + 128);
			}
			Yo += stride * 2;
			Vo += stride >> 1;
			Uo += stride >> 1;
		}
	}
	// image.cpp:216-246
	CImage& operator-=(const CImage& In) { return addsub(In, -1); }
	CImage& operator+=(const CImage& In) { return addsub(In, 1); }
	// image.cpp:248-265: per component 10 log10(4096^2 / MSE)
	void psnr(const CImage& In, float* ret)
	{
		for (int c = 0; c < component; c++) {
			long long sum = 0;
			for (unsigned int j = 0; j < dimY; j++)
				for (unsigned int i = 0; i < dimX; i++) {
					const int t = In.pImage[c][(long)j * In.dimXAlign + i] - pImage[c][(long)j * dimXAlign + i];
					sum += t * t;
				}
			ret[c] = (float)(10. * (std::log((double)(1 << 24)) - std::log((double)sum / (dimX * dimY))) / std::log(10.));
		}
	}
	// image.cpp:267-278
	void copy(const CImage& In)
	{
		for (int c = 0; c < component; c++)
			for (unsigned int j = 0; j < dimY; j++)
				std::memcpy(pImage[c] + (long)j * dimXAlign, In.pImage[c] + (long)j * In.dimXAlign, sizeof(short) * dimX);
	}
	// this image's planes with their border from `bordered` (3 x (dimY + 30)
	// x (dimX + 30) int16, ric_video_output with border)
	void load_bordered(const int16_t* bordered)
	{
		const unsigned int bw = dimX + 2 * BORDER, bh = dimY + 2 * BORDER;
		for (int c = 0; c < component; c++)
			for (unsigned int r = 0; r < bh; r++)
				std::memcpy(pImage[c] + ((long)r - BORDER) * dimXAlign - BORDER, bordered + ((size_t)c * bh + r) * bw,
				            sizeof(short) * bw);
	}

private:
	std::vector<short> data_;
	void init(int Align)
	{
		dimXAlign = (dimX + 2 * BORDER + Align - 1) & -Align;
		const size_t plane = (size_t)dimXAlign * (dimY + 2 * BORDER);
		data_.assign(plane * component + Align, 0);
		for (int c = 0; c < component && c < 3; c++) pImage[c] = data_.data() + c * plane + BORDER * dimXAlign + BORDER;
	}
	CImage& addsub(const CImage& In, int sign)
	{
		for (int c = 0; c < component; c++)
			for (unsigned int j = 0; j < dimY; j++)
				for (unsigned int i = 0; i < dimX; i++) {
					short& o = pImage[c][(long)j * dimXAlign + i];
					o = (short)(o + sign * In.pImage[c][(long)j * In.dimXAlign + i]);
				}
		return *this;
	}
};

// CRududuCodec (src/lib/rududucodec.h:31-55): the video codec over ric_video.
// encode / decode keep the reference's signatures and return values; the
// CImage* handed back is a host copy of the codec's output image (valid until
// the next call).  Like the reference, encode writes pBuffer with no bound and
// decode reads it in place.
class CRududuCodec {
public:
	int quant = 0;
	CRududuCodec(cmode mode, int width, int height, int component, int device = 0)
		: out_(width, height, component, ALIGN), bordered_((size_t)3 * (width + 2 * BORDER) * (height + 2 * BORDER))
	{
		ric_check(ric_video_create(&v_, mode == rududu::encode ? 1 : 0, width, height, component, device), "CRududuCodec");
	}
	~CRududuCodec() { ric_video_destroy(v_); }
	CRududuCodec(const CRududuCodec&) = delete;
	CRududuCodec& operator=(const CRududuCodec&) = delete;

	int encode(unsigned char* pImage, int stride, unsigned char* pBuffer, CImage** outImage)
	{
		ric_check(ric_video_set_quant(v_, quant), "CRududuCodec::quant");
		int size = 0;
		ric_check(ric_video_encode(v_, pImage, stride, 0, pBuffer, SIZE_MAX, &size), "CRududuCodec::encode");
		if (outImage) *outImage = sync_out();
		return size;
	}
	int decode(unsigned char* pBuffer, CImage** outImage)
	{
		ric_check(ric_video_set_quant(v_, quant), "CRududuCodec::quant");
		int size = 0;
		const int rc = ric_video_decode(v_, pBuffer, 0, &size);
		if (rc != RIC_OK && rc != RIC_E_STREAM) ric_check(rc, "CRududuCodec::decode");
		if (outImage) *outImage = sync_out();
		// a stream that ran past its end (the reference has no error channel and
		// returns garbage silently): the frame is still decoded and *outImage set,
		// then the caller is told
		if (rc == RIC_E_STREAM) throw RicError(rc, "CRududuCodec::decode: the decoder ran past the end of the stream");
		return size;
	}
	ric_video* handle() { return v_; }

private:
	ric_video* v_ = nullptr;
	CImage out_;
	std::vector<int16_t> bordered_;
	CImage* sync_out()
	{
		ric_check(ric_video_output(v_, bordered_.data(), 1, 0), "outImage");
		out_.load_bordered(bordered_.data());
		return &out_;
	}
};

}  // namespace rududu
