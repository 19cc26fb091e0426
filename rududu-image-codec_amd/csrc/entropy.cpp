// entropy.cpp -- host serial coder of the .ric path (see entropy.h).
#include "entropy.h"
#include "coder_tables.h"
#include "symbols.h"

#include <cstdlib>
#include <algorithm>

namespace ric {

#include "huff_tables.inc"

namespace {

using namespace tables;

// Cnk[k][n] = C(n, k + 1) (src/lib/muxcodec.cpp:282-292), built once.
struct CnkTable {
	uint16_t v[8][16];
	CnkTable()
	{
		for (int k = 0; k < 8; k++)
			for (int n = 0; n < 16; n++) {
				int kk = k + 1;
				if (n < kk) { v[k][n] = 0; continue; }
				uint32_t c = 1;
				for (int i = 1; i <= kk; i++) c = c * (n - kk + i) / i;
				v[k][n] = (uint16_t)c;
			}
	}
};
const CnkTable kCnk;

// taboo code tables for n = 2 (initTaboo(2), src/lib/muxcodec.cpp:113-129)
struct TabooTable {
	uint32_t nb[32], sum[32];
	TabooTable()
	{
		const uint32_t k = 2;
		nb[0] = 1;
		for (uint32_t i = 1; i < k; i++) nb[i] = 1u << (i - 1);
		for (uint32_t i = k; i < 32; i++) {
			uint32_t acc = nb[i - k];
			for (uint32_t j = i - k + 1; j < i; j++) acc += nb[j];
			nb[i] = acc;
		}
		sum[0] = nb[0];
		for (int i = 1; i < 32; i++) sum[i] = sum[i - 1] + nb[i];
	}
};
const TabooTable kTaboo;

// 8-bit first-level decode LUTs for the 33 static Huffman tables:
// entry = sym << 8 | len, or 0 when the code is longer than 8 bits.
struct HuffLut {
	uint16_t lut[33][256];
	HuffLut()
	{
		for (int t = 0; t < 33; t++) {
			const uint16_t* tab = t < 17 ? kHuff_LOW[t] : kHuff_HIGH[t - 17];
			int n = t < 17 ? 17 : 16;
			for (int i = 0; i < 256; i++) {
				lut[t][i] = 0;
				for (int s = 0; s < n; s++) {
					int len = tab[s] & 31;
					if (len <= 8 && (i >> (8 - len)) == (tab[s] >> 5)) { lut[t][i] = (uint16_t)((s << 8) | len); break; }
				}
			}
		}
	}
};
const HuffLut kHuffLut;


constexpr size_t kDecPad = 1 << 16;

}  // namespace

// ================================================================= Mux
namespace {
// buf + cap, saturated at the top of the address space (cap SIZE_MAX: no bound)
uint8_t* bound_of(uint8_t* buf, size_t cap)
{
	const uintptr_t b = (uintptr_t)buf;
	return (uint8_t*)(cap > UINTPTR_MAX - b ? UINTPTR_MAX : b + cap);
}
}  // namespace

void Mux::init_encoder(uint8_t* buf, size_t cap, uint16_t first_word)
{
	base_ = buf;
	limit_ = bound_of(buf, cap);
	low_ = (uint32_t)first_word << 16;
	range_ = 1u << 16;
	outcount_ = 0; nbits_ = 0; buffer_ = 0; reserved_ = nullptr; overflow_ = cap < 4;
	ebuf_ = 0; ebits_ = 0;
	p_ = buf + 4; init_ = buf + 2;
	for (int i = 0; i < 4; i++) last_[i] = buf + i;
}

void Mux::init_decoder(const uint8_t* buf, size_t len)
{
	free(owned_);
	owned_cap_ = 0;
	owned_ = (uint8_t*)calloc(len + kDecPad, 1);
	memcpy(owned_, buf, len);
	base_ = owned_;
	limit_ = owned_ + len + kDecPad - 16;
	range_ = 1u << 16;
	nbits_ = 0; buffer_ = 0; overflow_ = false;
	init_ = owned_ + 2; p_ = owned_ + 2;
	code_ = low_ = ((uint32_t)p_[0] << 8) | p_[1];
	p_ += 2;
}

void Mux::init_decoder_payload(const uint8_t* payload, size_t n)
{
	// the reference reads the payload at buf + 2 (src/ric/ric.cpp:203-205):
	// two zero bytes, then the .ric payload, then zero padding.  The buffer
	// is kept across frames (no fresh zeroed pages per frame).
	const size_t need = n + 2 + kDecPad;
	if (owned_cap_ < need) {
		free(owned_);
		owned_ = (uint8_t*)malloc(need);
		owned_cap_ = need;
	}
	owned_[0] = owned_[1] = 0;
	memcpy(owned_ + 2, payload, n);
	memset(owned_ + 2 + n, 0, kDecPad);
	base_ = owned_;
	limit_ = owned_ + n + 2 + kDecPad - 16;
	range_ = 1u << 16;
	nbits_ = 0; buffer_ = 0; overflow_ = false;
	init_ = owned_ + 2; p_ = owned_ + 2;
	code_ = low_ = ((uint32_t)p_[0] << 8) | p_[1];
	p_ += 2;
}

void Mux::init_decoder_inplace(const uint8_t* buf)
{
	// no copy and no end: the reference's CMuxCodec(pStream) contract
	base_ = const_cast<uint8_t*>(buf);
	limit_ = reinterpret_cast<uint8_t*>(UINTPTR_MAX);
	range_ = 1u << 16;
	nbits_ = 0; buffer_ = 0; overflow_ = false;
	init_ = base_ + 2; p_ = base_ + 2;
	code_ = low_ = ((uint32_t)p_[0] << 8) | p_[1];
	p_ += 2;
}

void Mux::reinit_encoder(uint8_t* buf, size_t cap, uint16_t first_word)
{
	if (buf) {
		init_encoder(buf, cap, first_word);
		return;
	}
	// no buffer: the state only (muxcodec.cpp:38-42), the output continues
	low_ = (uint32_t)first_word << 16;
	range_ = 1u << 16;
	outcount_ = 0; nbits_ = 0; reserved_ = nullptr;
	ebuf_ = 0; ebits_ = 0;
}

void Mux::reinit_decoder(const uint8_t* buf, size_t len)
{
	if (!buf) {                           // muxcodec.cpp:53-54
		range_ = 1u << 16;
		nbits_ = 0;
		return;
	}
	if (len == 0) init_decoder_inplace(buf);
	else init_decoder(buf, len);
}

Mux::~Mux() { free(owned_); }

void Mux::normalize_enc()                  // src/lib/muxcodec.cpp:63-74
{
	flush_buffer(false);
	do {
		put(last_[outcount_++ & 3], (uint8_t)(low_ >> 24));
		if (((low_ + range_ - 1) ^ low_) >= 0x01000000u) range_ = (0u - low_) & 4095u;
		last_[(outcount_ + 3) & 3] = p_++;
		range_ <<= 8;
		low_ <<= 8;
	} while (range_ <= 4096u);
}

void Mux::normalize_dec()                  // src/lib/muxcodec.cpp:76-85
{
	do {
		if (((code_ - low_ + range_ - 1) ^ (code_ - low_)) >= 0x01000000u) range_ = (low_ - code_) & 4095u;
		uint8_t b = *p_;
		if (p_ < limit_) p_++; else overflow_ = true;
		low_ = (low_ << 8) | b;
		code_ = (code_ << 8) | b;
		range_ <<= 8;
	} while (range_ <= 4096u);
}

void Mux::empty_buffer()                   // src/lib/muxcodec.cpp:536-548
{
	while (ebits_ >= 8) {
		ebits_ -= 8;
		uint8_t b = (uint8_t)(ebuf_ >> ebits_);
		if (!reserved_) put(p_++, b);
		else { put(reserved_, b); reserved_ = nullptr; }
	}
}

void Mux::flush_buffer(bool end)           // src/lib/muxcodec.cpp:550-570
{
	if (ebits_ >= 8) empty_buffer();
	if (ebits_ > 0) {
		if (end) {
			uint8_t b = (uint8_t)(ebuf_ << (8 - ebits_));
			if (!reserved_) put(p_++, b);
			else { put(reserved_, b); reserved_ = nullptr; }
			ebits_ = 0;
		} else if (!reserved_) {
			reserved_ = p_++;
		}
	}
}

void Mux::fill_buffer(uint32_t len)        // src/lib/muxcodec.cpp:572-579
{
	do {
		nbits_ += 8;
		buffer_ = (buffer_ << 8) | p_[0];
		if (p_ < limit_) p_++; else overflow_ = true;
	} while (nbits_ < len);
}

uint8_t* Mux::end_coding()                 // src/lib/muxcodec.cpp:87-106
{
	flush_buffer(true);
	if (range_ <= 4096u) normalize_enc();
	const uint32_t last_out = 0x200 | 'W';
	if ((low_ & 4095u) > (last_out & 4095u)) low_ += 4096u;
	low_ = (low_ & ~4095u) | (last_out & 4095u);
	put(last_[outcount_ & 3], (uint8_t)(low_ >> 24));
	put(last_[(outcount_ + 1) & 3], (uint8_t)(low_ >> 16));
	put(last_[(outcount_ + 2) & 3], (uint8_t)(low_ >> 8));
	put(last_[(outcount_ + 3) & 3], (uint8_t)low_);
	if (p_ > limit_) overflow_ = true;
	return p_;
}

uint32_t Mux::huff_decode(int high, int idx)
{
	const int t = high ? 17 + idx : idx;
	const uint32_t code = (((buffer_ << 16) | ((uint32_t)p_[0] << 8) | p_[1]) >> nbits_) & 0xFFFF;
	uint32_t e = kHuffLut.lut[t][code >> 8];
	uint32_t sym, len;
	if (e) {
		sym = e >> 8; len = e & 0xFF;
	} else {
		const uint16_t* tab = high ? kHuff_HIGH[idx] : kHuff_LOW[idx];
		const int n = high ? 16 : 17;
		sym = 0; len = tab[0] & 31;
		for (int s = 0; s < n; s++) {
			uint32_t l = tab[s] & 31;
			if ((code >> (16 - l)) == (uint32_t)(tab[s] >> 5)) { sym = s; len = l; break; }
		}
	}
	p_ -= (int)(nbits_ - len) >> 3;
	if (p_ > limit_) { p_ = limit_; overflow_ = true; }
	if (nbits_ < len) buffer_ = p_[-1];
	nbits_ = (nbits_ - len) & 7;
	return sym;
}

uint32_t Mux::huff_decode_table(const HuffSym* t)
{
	const uint32_t code = (((buffer_ << 16) | ((uint32_t)p_[0] << 8) | p_[1]) >> nbits_) & 0xFFFF;
	while (code < t->code) t++;                    // the last entry's code is 0
	if (t->len > 16) { overflow_ = true; return 0; }   // a code the reference cannot read either
	p_ -= (int)(nbits_ - t->len) >> 3;
	if (p_ > limit_) { p_ = limit_; overflow_ = true; }
	if (nbits_ < t->len) buffer_ = p_[-1];
	nbits_ = (nbits_ - t->len) & 7;
	return (t->value - (code >> (16 - t->len))) & 0xFF;
}

void Mux::golomb_lin_code(uint32_t nb, int k, int m)
{
	uint32_t l = 1;
	while (nb >= (1u << (k + m))) {
		l += 1u << m;
		nb -= 1u << (k + m);
		k++;
	}
	l += nb >> k;
	nb &= (1u << k) - 1;
	// l - 1 zeros then a one (the reference shifts them through its 32-bit
	// buffer in pieces, muxcodec.cpp:479-490: only the bit order matters)
	while (l > 32) { bits_code(0, 32); l -= 32; }
	bits_code(1, l);
	bits_code(nb, k);
}

uint32_t Mux::golomb_lin_decode(int k, int m)
{
	uint32_t l = 0;
	// the zero run, one bit at a time: a byte is read exactly when the bit
	// buffer runs dry, as in the reference's scan (muxcodec.cpp:499-506)
	for (;;) {
		if (bits_decode(1)) break;
		if (++l > (1u << 20)) { overflow_ = true; return 0; }   // no valid stream has such a run
	}
	uint32_t nb = ((1u << (l >> m)) - 1) << k;
	k += l >> m;
	l &= (1u << m) - 1;
	if (k > 24) { overflow_ = true; return 0; }
	nb += (l << k) | bits_decode(k);
	return nb;
}

void Mux::taboo_code(uint32_t nb)
{
	const uint32_t nt = 2;
	int i = 0, l;
	uint32_t r = 0;
	while (kTaboo.sum[i] <= nb) i++;
	if (i == 0) { bits_code(0, nt); return; }
	l = i; i--;
	nb -= kTaboo.sum[i];
	while (i > (int)nt) {
		uint32_t k = i - nt + 1, cnt = kTaboo.nb[k], j = 0;
		while (nb >= cnt) cnt += kTaboo.nb[k + ++j];
		nb -= cnt - kTaboo.nb[k + j];
		j = nt - j;
		r = (r << j) | 1;
		i -= j;
	}
	if (i == (int)nt) nb++;
	r = ((((r << i) | (nb & ((1u << i) - 1))) << 1) | 1) << nt;
	bits_code(r, l + nt);
}

uint32_t Mux::taboo_decode()
{
	const uint32_t nt = 2;
	int i, l = nt;
	uint32_t nb = 0;
	if (nbits_ < nt) fill_buffer(nt);
	uint32_t t = ((1u << nt) - 1) << (nbits_ - nt);
	while ((~buffer_ & t) != t) {
		l++;
		if (l > (int)nbits_) { fill_buffer(l); t <<= 8; }
		t >>= 1;
		// the 32-bit raw-bit buffer holds a code of at most 25 bits (fill
		// adds up to 7 bits past the request); the reference's own buffer
		// overflows on a longer, i.e. corrupt, code
		if (l > 25) { overflow_ = true; return 0; }
	}
	nbits_ -= l;
	uint32_t cd = buffer_ >> (nbits_ + nt + 1);
	i = l - nt;
	if (i > 0) { i--; nb += kTaboo.sum[i]; }
	while (i > (int)nt) {
		uint32_t j = 1;
		while (j < (uint32_t)i && ((cd >> (i - j)) & 1) == 0) j++;   // (a valid code has the 1 bit)
		nb += kTaboo.sum[i - j] - kTaboo.sum[i - nt];
		i -= j;
	}
	if (i == (int)nt) nb -= 1;
	nb += cd & ((1u << i) - 1);
	return nb;
}

void Mux::enum_code(uint32_t bits, uint32_t k, uint32_t nmax)
{
	uint32_t code = 0, n = 0, row = 0;
	if (k > ((nmax + 1) >> 1)) { k = nmax - k; bits ^= (1u << nmax) - 1; }
	do {
		if (bits & 1) { code += kCnk.v[row][n]; row++; }
		n++;
		bits >>= 1;
	} while (bits != 0);
	const uint32_t lost = kCnkLost[nmax - 1][k - 1], len = kCnkLen[nmax - 1][k - 1];
	if (code < lost) bits_code(code, len - 1);
	else bits_code(code + lost, len);
}

uint32_t Mux::enum_decode(uint32_t k, uint32_t nmax)
{
	int n = nmax - 1;
	uint32_t bits = 0;
	if (k > ((nmax + 1) >> 1)) { k = nmax - k; bits ^= (1u << nmax) - 1; }
	int row = (int)k - 1;
	const uint32_t lost = kCnkLost[nmax - 1][k - 1];
	uint32_t code = bits_decode(kCnkLen[nmax - 1][k - 1] - 1);
	if (code >= lost) code = ((code << 1) | bits_decode(1)) - lost;
	do {
		if (n >= 0 && code >= kCnk.v[row][n]) { bits ^= 1u << n; code -= kCnk.v[row][n]; row--; }
		n--;
		if (n < -1) break;
	} while (row >= 0);
	return bits;
}

void Mux::max_code(uint32_t value, uint32_t max)
{
	const uint32_t len = bitlen(max), lost = (1u << len) - max - 1;
	if (value < lost) bits_code(value, len - 1);
	else bits_code(value + lost, len);
}

uint32_t Mux::max_decode(uint32_t max)
{
	// maxDecode reads one bit even for max == 0 (src/lib/muxcodec.cpp:526-534),
	// where maxCode wrote none: kept for bit-exactness with the reference.
	uint32_t value = 0;
	const uint32_t len = bitlen(max), lost = (1u << len) - max - 1;
	if (len > 1) value = bits_decode(len - 1);
	if (value >= lost) value = ((value << 1) | bits_decode(1)) - lost;
	return value;
}

// ============================================================== models
void BitModel::init()
{
	for (int i = 0; i < 16; i++) { freq[i] = 2048; shift[i] = 0; mps[i] = 0; }
}

inline void BitModel::adj(int c)           // shift_adj, bitcodec.h:81-92
{
	if (freq[c] > kBitThres[shift[c]]) {
		if (shift[c] == 0) { mps[c] ^= 1; freq[c] = (uint16_t)(4096 - freq[c]); shift[c] = 1; }
		else shift[c]--;
	} else if (shift[c] < 9) shift[c]++;
}

inline void BitModel::code(Mux& m, uint32_t sym, int c)   // bitcodec.h:52-60
{
	const uint32_t s = sym ^ mps[c];
	m.code_bin(freq[c], s ^ 1);
	const int sh = shift[c];
	freq[c] = (uint16_t)(freq[c] + (s << (9 - sh)) - (freq[c] >> (3 + sh)));
	if ((uint16_t)(freq[c] - kBitThres[sh + 1]) > kBitThres[sh] - kBitThres[sh + 1]) adj(c);
}

inline uint32_t BitModel::decode(Mux& m, int c)           // bitcodec.h:62-70
{
	uint32_t sym = m.get_bit(freq[c]) ^ 1;
	const int sh = shift[c];
	freq[c] = (uint16_t)(freq[c] + (sym << (9 - sh)) - (freq[c] >> (3 + sh)));
	sym ^= mps[c];
	if ((uint16_t)(freq[c] - kBitThres[sh + 1]) > kBitThres[sh] - kBitThres[sh + 1]) adj(c);
	return sym;
}

void GeomModel::init(const uint8_t* kinit)                // setCtx, geomcodec.cpp:31-41
{
	for (int c = 0; c < 16; c++) {
		idx[c] = kinit[c];
		freq[c] = idx[c] >= 9 ? 2048 : (uint16_t)((kGeoThres[idx[c] - 1] + kGeoThres[idx[c]]) >> 1);
	}
}

inline void GeomModel::adj(int c)          // shift_adj, geomcodec.h:88-97
{
	const int s = kGeoShift[idx[c]];
	if (freq[c] < kGeoThres[s - 1]) { if (idx[c] < 24) idx[c]++; }
	else if (idx[c] > 0) idx[c]--;
	if (idx[c] >= 9) freq[c] = 2048;
}

inline void GeomModel::code(Mux& m, uint32_t sym, int c)  // geomcodec.h:41-57
{
	const uint32_t k = kGeoK[idx[c]], f = freq[c];
	const int s = kGeoShift[idx[c]];
	for (uint32_t l = sym >> k; l > 0; l--) {
		m.code_bin(f, 1);
		freq[c] -= freq[c] >> (3 + s);
	}
	m.code_bin(f, 0);
	if (k > 0) m.bits_code(sym & ((1u << k) - 1), k);
	freq[c] += (4096 - freq[c]) >> (3 + s);
	if ((uint16_t)(freq[c] - kGeoThres[s - 1]) > kGeoThres[s] - kGeoThres[s - 1]) adj(c);
}

inline void GeomModel::code_signed(Mux& m, uint32_t sym, uint32_t sign, int c)
{
	const uint32_t k = kGeoK[idx[c]], f = freq[c];
	const int s = kGeoShift[idx[c]];
	for (uint32_t l = sym >> k; l > 0; l--) {
		m.code_bin(f, 1);
		freq[c] -= freq[c] >> (3 + s);
	}
	m.code_bin(f, 0);
	m.bits_code(((sym & ((1u << k) - 1)) << 1) | sign, k + 1);
	freq[c] += (4096 - freq[c]) >> (3 + s);
	if ((uint16_t)(freq[c] - kGeoThres[s - 1]) > kGeoThres[s] - kGeoThres[s - 1]) adj(c);
}

inline uint32_t GeomModel::decode(Mux& m, int c)          // geomcodec.h:59-75
{
	const uint32_t k = kGeoK[idx[c]], f = freq[c];
	const int s = kGeoShift[idx[c]];
	uint32_t l = 0;
	while (m.get_bit(f)) {
		freq[c] -= freq[c] >> (3 + s);
		l++;
		if (l > (1u << 20)) break;           // corrupt stream guard
	}
	if (k > 0) l = (l << k) | m.bits_decode(k);
	freq[c] += (4096 - freq[c]) >> (3 + s);
	if ((uint16_t)(freq[c] - kGeoThres[s - 1]) > kGeoThres[s] - kGeoThres[s - 1]) adj(c);
	return l;
}

// ========================================================== band scans
namespace {

template <typename C> constexpr bool is_short() { return sizeof(C) == 2; }

template <typename C>
void pred_t(Mux& m, const BandView& b, bool dec)
{
	static const uint8_t ginit[16] = {9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,15};  // bandcodec.cpp:67-68
	constexpr bool SH = is_short<C>();
	GeomModel g; g.init(ginit);
	C* c = (C*)b.p;
	const long st = b.pitch;
	if (!dec) m.taboo_code(s2u(c[0]));
	else c[0] = (C)u2s((int)m.taboo_decode());
	for (int i = 1; i < b.dx; i++) {
		if (!dec) g.code(m, s2u(c[i] - c[i - 1]), 15);
		else c[i] = (C)tr<SH>(c[i - 1] + u2s((int)g.decode(m, 15)));
	}
	for (int j = 1; j < b.dy; j++) {
		c += st;
		if (!dec) g.code(m, s2u(c[0] - c[-st]), 15);
		else c[0] = (C)tr<SH>(c[-st] + u2s((int)g.decode(m, 15)));
		for (int i = 1; i < b.dx; i++) {
			int a = c[i - 1] - c[i - 1 - st], bb = c[i - st] - c[i - 1 - st];
			int var = bitlen((uint32_t)((a < 0 ? -a : a) + (bb < 0 ? -bb : bb)));
			// the reference indexes its 16 geometric contexts with var
			// unchecked (out of bounds, i.e. undefined, past 15): only a
			// corrupt stream or an out-of-range LL gets there; clamp
			if (var > 15) var = 15;
			if (!dec) g.code(m, s2u(c[i] - c[i - 1] - c[i - st] + c[i - 1 - st]), var);
			else c[i] = (C)tr<SH>(c[i - 1] + c[i - st] - c[i - 1 - st] + u2s((int)g.decode(m, var)));
		}
	}
}


// block_enum (full 4x4), src/lib/bandcodec.cpp:346-403
template <typename C, bool HIGH, bool DEC>
inline int block_full(Mux& m, GeomModel& g, C* blk, long st, int idx)
{
	constexpr bool SH = is_short<C>();
	uint32_t k = 0;
	if (!DEC) {
		int tmp[16];
		uint32_t sig = 0;
		for (int j = 0; j < 4; j++)
			for (int i = 0; i < 4; i++) {
				int v = blk[j * st + i];
				sig <<= 1;
				if (v != 0) { tmp[k++] = v; sig |= 1; }
			}
		const uint16_t e = HIGH ? kHuff_HIGH[idx][k - 1] : kHuff_LOW[idx][k];
		m.bits_code(e >> 5, e & 31);
		if (HIGH || k != 0) {
			if (k != 16) m.enum_code(sig, k, 16);
			for (uint32_t i = 0; i < k; i++) {
				g.code(m, (uc<SH>(tmp[i]) >> 1) - 1, k - 1);
				m.bits_code(tmp[i] & 1, 1);
			}
		}
	} else {
		k = m.huff_decode(HIGH, idx) + (HIGH ? 1 : 0);
		if (HIGH || k != 0) {
			uint32_t sig = 0xFFFF;
			if (k != 16) sig = m.enum_decode(k, 16);
			for (int j = 0; j < 4; j++)
				for (int i = 0; i < 4; i++) {
					if (sig & (1u << 15)) {
						uint32_t u = ((g.decode(m, k - 1) + 1) << 1) | m.bits_decode(1);
						blk[j * st + i] = (C)tr<SH>(u2s_((int)u));
					}
					sig <<= 1;
				}
		}
	}
	return (int)k - (HIGH ? 1 : 0);
}

// block_enum (edge w x h), src/lib/bandcodec.cpp:405-478
template <typename C, bool HIGH, bool DEC>
inline void block_edge(Mux& m, GeomModel& g, C* blk, long st, int w, int h)
{
	constexpr bool SH = is_short<C>();
	uint32_t k = 0;
	const uint32_t cnt = (uint32_t)(w * h);
	if (!DEC) {
		int tmp[16];
		uint32_t sig = 0;
		for (int j = 0; j < h; j++)
			for (int i = 0; i < w; i++) {
				int v = blk[j * st + i];
				sig <<= 1;
				if (v != 0) { tmp[k++] = v; sig |= 1; }
			}
		if (HIGH) m.max_code(k - 1, cnt - 1); else m.max_code(k, cnt);
		if (HIGH || k != 0) {
			if (k != cnt) m.enum_code(sig, k, cnt);
			for (uint32_t i = 0; i < k; i++) {
				g.code(m, (uc<SH>(tmp[i]) >> 1) - 1, kKConv2[kKConv1[cnt]][k - 1]);
				m.bits_code(tmp[i] & 1, 1);
			}
		}
	} else {
		k = HIGH ? m.max_decode(cnt - 1) + 1 : m.max_decode(cnt);
		if (k > cnt) k = cnt;                 // corrupt-stream guard (never on valid data)
		if (HIGH || k != 0) {
			uint32_t sig = 0xFFFF;
			if (k != cnt) sig = m.enum_decode(k, cnt);
			for (int j = 0; j < h; j++)
				for (int i = 0; i < w; i++) {
					if (sig & (1u << (cnt - 1))) {
						uint32_t u = ((g.decode(m, kKConv2[kKConv1[cnt]][k - 1]) + 1) << 1) | m.bits_decode(1);
						blk[j * st + i] = (C)tr<SH>(u2s_((int)u));
					}
					sig <<= 1;
				}
		}
	}
}

// maxLen<2, mode>, src/lib/bandcodec.cpp:324-344
template <typename P, bool DEC>
inline int max_len2(const P* p, long st)
{
	constexpr bool SH = is_short<P>();
	int mx = 0, mn = 0;
	for (int j = 0; j < 2; j++)
		for (int i = 0; i < 2; i++) {
			int v = p[j * st + i];
			if (v > mx) mx = v;
			if (DEC && v < mn) mn = v;
		}
	if (!DEC) return bitlen(uc<SH>(mx) >> 1);
	mn = tr<SH>(mn < 0 ? -mn : mn);
	if (mn > mx) mx = mn;
	return bitlen((uint32_t)mx);
}

// CBandCodec::tree, src/lib/bandcodec.cpp:484-589
template <typename C, typename P, bool HIGH, bool DEC>
void tree_t(Mux& m, const BandView& b, const BandView& par, bool has_child)
{
	constexpr bool SH = is_short<C>();
	static const uint8_t ginit[16] = {5,9,9,9,9,9,9,9,9,9,9,9,10,10,10,11};   // bandcodec.cpp:487
	uint16_t kmean[16] = {2 << 10, 3 << 10, 4 << 10, 5 << 10, 8 << 10, 11 << 10, 13 << 10, 14 << 10,
	                      15 << 10, 15 << 10, 15 << 10, 15 << 10, 15 << 10, 15 << 10, 15 << 10, 15 << 10};
	const long st = b.pitch;
	const int dx = b.dx, dy = b.dy;
	P* pbase = (P*)par.p;
	const long pst = par.pitch;
	const int pdx = par.dx, pdy = par.dy;
	const int mark = has_child ? kInsignif : 0;
	C* band = (C*)b.p;
	if (DEC) for (int j = 0; j < dy; j++) memset(band + j * st, 0, sizeof(C) * dx);   // Clear(), :503
	GeomModel g; g.init(ginit);
	BitModel tree, bord; tree.init(); bord.init();

	auto edge_block = [&](C* c1, int i, int w, int h, P* pp, bool chk_row, int j) {
		if (pp && (i >> 1) < pdx && (!chk_row || (j >> 1) < pdy) && pp[i >> 1] == kInsignif) pp[i >> 1] = 0;
		uint32_t ins;
		if (DEC) ins = bord.decode(m, 0);
		else { ins = c1[i] == (C)kInsignif; bord.code(m, ins, 0); }
		if (ins) { if (!DEC) c1[i] = 0; }
		else block_edge<C, HIGH, DEC>(m, g, c1 + i, st, w, h);
	};

	int j = 0;
	for (; j + 4 <= dy; j += 4) {
		C* c1 = band + j * st;
		C* c2 = c1 + 2 * st;
		P* pp = pbase ? pbase + (long)(j >> 1) * pst : nullptr;
		int i = 0, bs = 4;
		if (j & 4) {
			bs = -4;
			i = dx & ~3;
			if (dx > i) edge_block(c1, i, dx - i, 4, pp, false, j);
			i += bs;
		}
		for (; i >= 0 && i + 4 <= dx; i += bs) {
			int ctx = 15;
			const int k = i >> 1;
			if (pp) ctx = pp[k];
			if (ctx == kInsignif) {
				pp[k] = 0;
				c1[i] = c1[i + 2] = c2[i] = c2[i + 2] = (C)tr<SH>(mark);
				continue;
			}
			if (pp) ctx = max_len2<P, DEC>(pp + k, pst);
			uint32_t ins;
			if (DEC) ins = tree.decode(m, ctx);
			else { ins = c1[i] == (C)kInsignif; tree.code(m, ins, ctx); }
			if (ins) {
				c1[i] = c1[i + 2] = c2[i] = c2[i + 2] = (C)tr<SH>(mark);
			} else {
				const int idx = (kmean[ctx] + (1 << 9)) >> 10;
				const int kk = block_full<C, HIGH, DEC>(m, g, c1 + i, st, idx);
				kmean[ctx] = (uint16_t)(kmean[ctx] + ((uint32_t)kk << 7) - (kmean[ctx] >> 3));
			}
		}
		if (i > 0 && i < dx) edge_block(c1, i, dx - i, 4, pp, false, j);
	}
	if (j < dy) {
		C* c1 = band + j * st;
		P* pp = pbase ? pbase + (long)(j >> 1) * pst : nullptr;
		const int h = dy - j;
		int i = 0, bs = 4;
		if (j & 4) {
			bs = -4;
			i = dx & ~3;
			if (dx > i) edge_block(c1, i, dx - i, h, pp, true, j);
			i += bs;
		}
		for (; i >= 0 && i + 4 <= dx; i += bs) {
			if (pp && (j >> 1) < pdy && pp[i >> 1] == kInsignif) pp[i >> 1] = 0;
			uint32_t ins;
			if (DEC) ins = bord.decode(m, 0);
			else { ins = c1[i] == (C)kInsignif; bord.code(m, ins, 0); }
			if (ins) { if (!DEC) c1[i] = 0; }
			else block_edge<C, HIGH, DEC>(m, g, c1 + i, st, 4, h);
		}
		if (i > 0 && i < dx) edge_block(c1, i, dx - i, h, pp, true, j);
	}
}

// The band writes of tree<encode> alone (src/lib/bandcodec.cpp:510-588): the
// parent's INSIGNIF markers this band consumes are cleared, a skipped or
// insignificant full block gets the marker (or 0 without children) at its
// four child anchors, an insignificant edge block's marker becomes 0.  Run on
// every band in coding order it leaves the pyramid in the state CodeBand
// leaves it in (what a caller of TSUQi after CodeBand dequantises).
template <typename C, typename P>
void tree_state_t(const BandView& b, const BandView& par, bool has_child)
{
	constexpr bool SH = is_short<C>();
	const long st = b.pitch;
	const int dx = b.dx, dy = b.dy;
	P* pbase = (P*)par.p;
	const long pst = par.pitch;
	const int pdx = par.dx, pdy = par.dy;
	const C mark = (C)tr<SH>(has_child ? kInsignif : 0);
	C* band = (C*)b.p;
	auto edge_block = [&](C* c1, int i, P* pp, bool chk_row, int j) {
		if (pp && (i >> 1) < pdx && (!chk_row || (j >> 1) < pdy) && pp[i >> 1] == kInsignif) pp[i >> 1] = 0;
		if (c1[i] == (C)kInsignif) c1[i] = 0;
	};
	int j = 0;
	for (; j + 4 <= dy; j += 4) {
		C* c1 = band + j * st;
		C* c2 = c1 + 2 * st;
		P* pp = pbase ? pbase + (long)(j >> 1) * pst : nullptr;
		int i = 0, bs = 4;
		if (j & 4) {
			bs = -4;
			i = dx & ~3;
			if (dx > i) edge_block(c1, i, pp, false, j);
			i += bs;
		}
		for (; i >= 0 && i + 4 <= dx; i += bs) {
			const int k = i >> 1;
			if (pp && pp[k] == kInsignif) {
				pp[k] = 0;
				c1[i] = c1[i + 2] = c2[i] = c2[i + 2] = mark;
			} else if (c1[i] == (C)kInsignif) {
				c1[i] = c1[i + 2] = c2[i] = c2[i + 2] = mark;
			}
		}
		if (i > 0 && i < dx) edge_block(c1, i, pp, false, j);
	}
	if (j < dy) {
		C* c1 = band + j * st;
		P* pp = pbase ? pbase + (long)(j >> 1) * pst : nullptr;
		int i = 0, bs = 4;
		if (j & 4) {
			bs = -4;
			i = dx & ~3;
			if (dx > i) edge_block(c1, i, pp, true, j);
			i += bs;
		}
		for (; i >= 0 && i + 4 <= dx; i += bs) {
			if (pp && (j >> 1) < pdy && pp[i >> 1] == kInsignif) pp[i >> 1] = 0;
			if (c1[i] == (C)kInsignif) c1[i] = 0;
		}
		if (i > 0 && i < dx) edge_block(c1, i, pp, true, j);
	}
}

template <bool DEC>
void tree_dispatch(Mux& m, const BandView& b, const BandView& par, bool high, bool has_child)
{
	const bool pint = par.p ? par.is_int : b.is_int;
	if (!b.is_int && !pint) {
		if (high) tree_t<int16_t, int16_t, true, DEC>(m, b, par, has_child);
		else tree_t<int16_t, int16_t, false, DEC>(m, b, par, has_child);
	} else if (!b.is_int) {
		if (high) tree_t<int16_t, int32_t, true, DEC>(m, b, par, has_child);
		else tree_t<int16_t, int32_t, false, DEC>(m, b, par, has_child);
	} else {
		if (high) tree_t<int32_t, int32_t, true, DEC>(m, b, par, has_child);
		else tree_t<int32_t, int32_t, false, DEC>(m, b, par, has_child);
	}
}

}  // namespace

// ====================================================== video motion vectors
namespace {

// CHuffCodec (src/lib/huffcodec.{h,cpp}) as the video codec builds it, with
// no initial table (pInitTable 0): adaptive canonical Huffman over n symbols,
// every symbol starting at frequency 8; the code is rebuilt when the
// accumulated count reaches UPDATE_THRES, frequencies halving each time.
// glibc's qsort (2.35) is a stable merge sort here; std::stable_sort matches it.
class AdaptiveHuff {
public:
	AdaptiveHuff(bool enc, unsigned n) : enc_(enc), n_(n)
	{
		for (unsigned i = 0; i < n; i++) freq_[i] = 8;
		update_code();
	}
	void code(Mux& m, unsigned sym)                     // huffcodec.h:80-87
	{
		if (count_ >= kThres) update_code();
		m.bits_code(sym_[sym].code, sym_[sym].len);
		freq_[sym] = (uint16_t)(freq_[sym] + step_);
		count_ += step_;
	}
	unsigned decode(Mux& m)                             // huffcodec.h:89-97
	{
		if (count_ >= kThres) update_code();
		const unsigned sym = lut_[m.huff_decode_table(sym_)];
		freq_[sym] = (uint16_t)(freq_[sym] + step_);
		count_ += step_;
		return sym;
	}

private:
	static constexpr unsigned kStepMin = 128, kStepMax = 2048, kThres = 1u << 14;   // huffcodec.h:32-34
	bool enc_;
	unsigned n_, count_ = 0, step_ = kStepMax;
	uint16_t freq_[256];
	HuffSym sym_[256];
	uint8_t lut_[256];

	// make_len (huffcodec.cpp:83-125): Moffat-Katajainen in place, weights in .code
	static void make_len(HuffSym* s, int n)
	{
		int root = n - 1, leaf = n - 3, next, nodes_left, nb_nodes, depth;
		s[n - 1].code = (uint16_t)(s[n - 1].code + s[n - 2].code);
		for (int i = n - 2; i > 0; i--) {
			if (leaf < 0 || s[root].code < s[leaf].code) {
				s[i].code = s[root].code;
				s[root--].code = (uint16_t)i;
			} else
				s[i].code = s[leaf--].code;
			if (leaf < 0 || (root > i && s[root].code < s[leaf].code)) {
				s[i].code = (uint16_t)(s[i].code + s[root].code);
				s[root--].code = (uint16_t)i;
			} else
				s[i].code = (uint16_t)(s[i].code + s[leaf--].code);
		}
		s[1].code = 0;
		for (int i = 2; i < n; i++) s[i].code = (uint16_t)(s[s[i].code].code + 1);
		nodes_left = 1;
		nb_nodes = depth = 0;
		root = 1;
		next = 0;
		while (nodes_left > 0) {
			while (root < n && s[root].code == depth) { nb_nodes++; root++; }
			while (nodes_left > nb_nodes) { s[next++].len = (uint8_t)depth; nodes_left--; }
			nodes_left = 2 * nb_nodes;
			depth++;
			nb_nodes = 0;
		}
	}
	// make_codes (huffcodec.cpp:149-160): canonical codes, longest (last) = 0
	static void make_codes(HuffSym* s, int n)
	{
		unsigned bits = s[n - 1].len, code = 0;
		s[n - 1].code = 0;
		for (int i = n - 2; i >= 0; i--) {
			code >>= bits - s[i].len;
			bits = s[i].len;
			code++;
			s[i].code = (uint16_t)code;
		}
	}
	// enc2dec (huffcodec.cpp:191-211): one entry per length + the symbol LUT
	static void enc2dec(const HuffSym* s, HuffSym* out, uint8_t* lut, int n)
	{
		unsigned bits = s[0].len, cnt = 0;
		for (int i = 1; i < n; i++) {
			if (s[i].len != bits) {
				bits = s[i].len;
				out[cnt].code = (uint16_t)(s[i - 1].code << (16 - s[i - 1].len));
				out[cnt].len = s[i - 1].len;
				out[cnt++].value = (uint8_t)(s[i - 1].code + i - 1);
			}
		}
		out[cnt].code = (uint16_t)(s[n - 1].code << (16 - s[n - 1].len));
		out[cnt].len = s[n - 1].len;
		out[cnt++].value = (uint8_t)(s[n - 1].code + n - 1);
		for (int i = 0; i < n; i++) lut[i] = s[i].value;
	}
	// update_code (huffcodec.cpp:213-236)
	void update_code()
	{
		HuffSym s[256];
		for (unsigned i = 0; i < n_; i++) {
			s[i].code = freq_[i];
			s[i].value = (uint8_t)i;
			s[i].len = 0;
			freq_[i] = (uint16_t)((freq_[i] + 1) >> 1);
		}
		std::stable_sort(s, s + n_, [](const HuffSym& a, const HuffSym& b) { return a.code > b.code; });   // comp_freq
		make_len(s, (int)n_);
		make_codes(s, (int)n_);
		if (enc_) {
			std::stable_sort(s, s + n_, [](const HuffSym& a, const HuffSym& b) { return a.value < b.value; });  // comp_sym
			memcpy(sym_, s, sizeof(HuffSym) * n_);
		} else {
			enc2dec(s, sym_, lut_, (int)n_);
		}
		count_ = 0;
		step_ >>= 1;
		step_ = std::max(step_, kStepMin);
	}
};

constexpr uint32_t kMvIntra = 0x80008000u;           // MV_INTRA, obmc.h:37

inline int mv_x(uint32_t v) { return (int16_t)(v & 0xFFFF); }
inline int mv_y(uint32_t v) { return (int16_t)(v >> 16); }
inline uint32_t mv_make(int x, int y) { return (uint32_t)(uint16_t)x | ((uint32_t)(uint16_t)y << 16); }
// median (src/lib/utils.h:64-77) on short
inline int med3(int a, int b, int c)
{
	if (b < a) std::swap(a, b);
	if (c <= a) return a;
	if (c <= b) return c;
	return b;
}

// the MV predictor of block (i, j) (obmc.cpp:358-367): the left vector on the
// first row, the one above on the first and last columns, else the median of
// left, above, above-right (ILP32 indexing: pCurMV[i - dimX] is the row above)
inline uint32_t mv_pred(const uint32_t* row, int i, int j, int dimx)
{
	if (j == 0) return i != 0 ? row[i - 1] : 0u;
	if (i == 0 || i == dimx - 1) return row[i - dimx];
	const uint32_t l = row[i - 1], u = row[i - dimx], ur = row[i - dimx + 1];
	return mv_make(med3(mv_x(l), mv_x(u), mv_x(ur)), med3(mv_y(l), mv_y(u), mv_y(ur)));
}

}  // namespace

void mv_encode(Mux& m, const uint32_t* mv, int dimx, int dimy)
{
	BitModel intra, zero;                             // CBitCodec intraCodec, zeroCodec (obmc.cpp:347)
	intra.init();
	zero.init();
	AdaptiveHuff huff_x(true, 128), huff_y(true, 128), huff(true, 255);
	for (int j = 0; j < dimy; j++) {
		const uint32_t* row = mv + (size_t)j * dimx;
		for (int i = 0; i < dimx; i++) {
			if (row[i] == kMvIntra) { intra.code(m, 1, 0); continue; }
			intra.code(m, 0, 0);
			const uint32_t p = mv_pred(row, i, j, dimx);
			if (mv_x(row[i]) == mv_x(p) && mv_y(row[i]) == mv_y(p)) { zero.code(m, 0, 0); continue; }
			zero.code(m, 1, 0);
			const int x = s2u(mv_x(row[i]) - mv_x(p)), y = s2u(mv_y(row[i]) - mv_y(p));
			huff.code(m, (unsigned)((std::min(x, 15) | (std::min(y, 15) << 4)) - 1));
			if (x >= 15) {
				huff_x.code(m, (unsigned)std::min(x - 15, 127));
				if (x >= 127 + 15) m.golomb_lin_code((uint32_t)(x - 127 - 15), 5, 0);
			}
			if (y >= 15) {
				huff_y.code(m, (unsigned)std::min(y - 15, 127));
				if (y >= 127 + 15) m.golomb_lin_code((uint32_t)(y - 127 - 15), 5, 0);
			}
		}
	}
}

void mv_decode(Mux& m, uint32_t* mv, int dimx, int dimy)
{
	BitModel intra, zero;
	intra.init();
	zero.init();
	AdaptiveHuff huff_x(false, 128), huff_y(false, 128), huff(false, 255);
	for (int j = 0; j < dimy; j++) {
		uint32_t* row = mv + (size_t)j * dimx;
		for (int i = 0; i < dimx; i++) {
			if (intra.decode(m, 0)) { row[i] = kMvIntra; continue; }
			const uint32_t p = mv_pred(row, i, j, dimx);
			if (zero.decode(m, 0)) {
				const int tmp = (int)huff.decode(m) + 1;
				int x = tmp & 0xF, y = tmp >> 4;
				if (x == 15) {
					x += (int)huff_x.decode(m);
					if (x == 127 + 15) x += (int)m.golomb_lin_decode(5, 0);
				}
				const int nx = u2s(x) + mv_x(p);
				if (y == 15) {
					y += (int)huff_y.decode(m);
					if (y == 127 + 15) y += (int)m.golomb_lin_decode(5, 0);
				}
				row[i] = mv_make(nx, u2s(y) + mv_y(p));
			} else {
				row[i] = p;
			}
		}
	}
}

void pred_encode(Mux& m, const BandView& b)
{
	if (b.is_int) pred_t<int32_t>(m, b, false); else pred_t<int16_t>(m, b, false);
}
void pred_decode(Mux& m, const BandView& b)
{
	if (b.is_int) pred_t<int32_t>(m, b, true); else pred_t<int16_t>(m, b, true);
}
void tree_encode(Mux& m, const BandView& b, const BandView& par, bool high, bool has_child)
{
	tree_dispatch<false>(m, b, par, high, has_child);
}
void tree_decode(Mux& m, const BandView& b, const BandView& par, bool high, bool has_child)
{
	tree_dispatch<true>(m, b, par, high, has_child);
}
void tree_encode_state(const BandView& b, const BandView& par, bool has_child)
{
	const bool pint = par.p ? par.is_int : b.is_int;
	if (!b.is_int && !pint) tree_state_t<int16_t, int16_t>(b, par, has_child);
	else if (!b.is_int) tree_state_t<int16_t, int32_t>(b, par, has_child);
	else tree_state_t<int32_t, int32_t>(b, par, has_child);
}

}  // namespace ric
