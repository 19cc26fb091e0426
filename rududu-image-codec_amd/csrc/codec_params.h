// codec_params.h -- host-side per-band parameters of the quantiser and the
// dequantiser, computed in float32 exactly as the reference does (the kernels
// get the resulting integers).  Shared by the single-frame C-ABI (capi.cpp)
// and the batch coder (batch.cpp).
#pragma once
#include <cstdint>
#include <string>
#include "ric_types.h"
#include "ric_kernels.h"

namespace ric {

// this thread's ric_last_error() message (capi.cpp)
void set_last_error(const std::string& msg);

inline int tr_any(bool sh, int v) { return sh ? (int)(int16_t)v : v; }

// CBandCodec::makeThres + clen (src/lib/bandcodec.cpp:129-157)
inline void make_thres(bool sh, int* thres, int quant, int lambda)
{
	static const int blen[17] = {20, 40, 55, 66, 75, 81, 85, 88, 89, 88, 85, 81, 75, 66, 55, 40, 20};
	static const uint8_t kk[] = {0,0,0,0,0,0,0,0,0,0,0,1,1,1,1,2};
	static const uint8_t mps[] = {1,1,2,2,2,5,5,5,5,5,5,5,5,5,5,5};
	for (int i = 0; i < 16; i++) {
		int clen1 = (kk[i] + 1) * 5 + mps[i];
		int t = tr_any(sh, (quant + ((lambda * (blen[i + 1] - blen[i] + clen1) + 8) >> 4)) & 0xFFFE);
		if (t > quant * 2) t = tr_any(sh, quant * 2);
		if (t < (quant & 0xFFFE)) t = tr_any(sh, quant & 0xFFFE);
		thres[i] = t;
	}
}

// buildTree parameters of level l (src/lib/bandcodec.cpp:243-247, float32 as
// the reference); qin carries CodeBand's per-level C-typed Quant.
inline QuantParams level_qp(const Pyramid& P, int l, int& qin, int lambda)
{
	const bool sh = !P.L[l].is_int;
	qin = tr_any(sh, qin);
	QuantParams qp;
	for (int b = 0; b < 3; b++) {
		const Band& B = P.L[l].b[b];
		int lbda = (int)((float)lambda / B.weight);
		int Q = tr_any(sh, (int16_t)(int)((float)qin / B.weight));
		if (Q == 0) Q = 1;
		qp.Q[b] = Q;
		qp.iQ[b] = (1 << 16) / Q;
		make_thres(sh, qp.thres[b], Q, lbda);
	}
	return qp;
}

// CBand::TSUQ on the coarsest LL with Thres 0.5 (src/lib/band.h:65-92)
inline void ll_params(const Pyramid& P, int quant, int& Q, int& iQ, int& T0)
{
	const Band& B = P.L[P.nlev - 1].b[BL];
	Q = (int)((float)quant / B.weight);
	if (Q == 0) Q = 1;
	iQ = (1 << 16) / Q;
	T0 = tr_any(!B.is_int, (int)(0.5f * (float)Q));
}

// CWavelet2D::TSUQi fused into TransformI (the codec's decode path): the
// bands stay quantised in HBM and every inverse level multiplies the band
// values it loads by their TSUQi factor (src/lib/band.h:94-107,
// src/lib/wavelet2d.cpp:248-268); the coarsest level also its LL.
inline int tsuqi_factor(const Band& B, int quant)
{
	const bool sh = !B.is_int;
	int q = tr_any(sh, quant);
	q = tr_any(sh, (int)((float)q / B.weight));
	return q == 0 ? 1 : q;
}

// src/ric/ric.cpp:42-49
inline int quants(int idx)
{
	static const unsigned short Q[5] = {0x8000, 0x9000, 0xA800, 0xC000, 0xE000};
	if (idx <= 0) return 0;
	idx--;
	int r = 14 - idx / 5;
	return (short)((Q[idx % 5] + (1 << (r - 1))) >> r);
}

}  // namespace ric
