// entropy.h -- the serial part of the .ric path, on the host: the multiplexed
// carry-less range coder / raw-bit packer (CMuxCodec, src/lib/muxcodec.*), the
// adaptive binary and geometric models (CBitCodec src/lib/bitcodec.*,
// CGeomCodec src/lib/geomcodec.*) and the per-band zerotree / LL-DPCM scans
// (CBandCodec::tree / pred, src/lib/bandcodec.cpp:62-104, 484-589).
//
// Everything here is inherently sequential (one adaptive state per band, one
// range-coder state per stream: SURVEY.md §7.1); the data-parallel stages
// (DWT, RD quantiser, dequantiser, inverse DWT) run on the GPU.
#pragma once
#include <vector>
#include <algorithm>
#include <cstdint>
#include <cstddef>
#include <cstring>
#include "ric_types.h"

namespace ric {

// sHuffSym (src/lib/muxcodec.h:42-46): a Huffman table entry
struct HuffSym {
	uint16_t code;
	uint8_t len;
	uint8_t value;
};

// ------------------------------------------------------------------ mux
class Mux {
public:
	// encoder over [buf, buf + cap); first two bytes are the reference's
	// firstWord slots (src/lib/muxcodec.cpp:36-49)
	void init_encoder(uint8_t* buf, size_t cap, uint16_t first_word = 0);
	// decoder over a copy of [buf, buf + len) padded with zeros
	void init_decoder(const uint8_t* buf, size_t len);
	// decoder over a .ric payload (the bytes after the 9-byte header): the
	// same as init_decoder on two zero bytes followed by the payload
	void init_decoder_payload(const uint8_t* payload, size_t n);
	// decoder reading buf + 2 in place with no end (the reference's
	// CMuxCodec(pStream), src/lib/muxcodec.cpp:31-34, 51-61): the caller's
	// buffer must outlive it and hold the stream
	void init_decoder_inplace(const uint8_t* buf);
	// CMuxCodec::initCoder(firstWord, pStream) (src/lib/muxcodec.cpp:36-49):
	// resets the coder state; a non-null buf also restarts the output there
	// (cap bytes; SIZE_MAX: no bound, like the reference), a null buf keeps
	// the current output position, as the reference does.
	void reinit_encoder(uint8_t* buf, size_t cap, uint16_t first_word);
	// CMuxCodec::initDecoder(pStream) (src/lib/muxcodec.cpp:51-61): resets the
	// range and bit buffer; a non-null buf restarts the input there (len bytes
	// copied with zero padding; len 0: read in place with no end, like the
	// reference), a null buf keeps the read position.
	void reinit_decoder(const uint8_t* buf, size_t len);
	Mux() = default;
	Mux(const Mux&) = delete;
	Mux& operator=(const Mux&) = delete;
	~Mux();

	uint8_t* end_coding();                  // endCoding, muxcodec.cpp:87-106
	size_t size() const { return (size_t)(p_ - init_); }   // getSize
	bool overflow() const { return overflow_; }
	uint8_t* buffer() const { return base_; }

	inline void code_bin(uint32_t freq, uint32_t bit)    // codeBin, muxcodec.h:156-163
	{
		if (range_ <= 4096u) normalize_enc();
		const uint32_t t = (range_ * freq) >> 12;
		low_ += t & (0u - bit);
		range_ = t + ((range_ - 2 * t) & (0u - bit));
	}
	inline uint32_t get_bit(uint32_t freq)                // getBit, muxcodec.h:205-213
	{
		if (range_ <= 4096u) normalize_dec();
		const uint32_t t = (range_ * freq) >> 12;
		const uint32_t tst = (uint32_t)(low_ < t) - 1u;
		low_ -= t & tst;
		range_ = t + ((range_ - 2 * t) & tst);
		return 0u - tst;
	}
	// bitsCode, muxcodec.h:225-231.  The encoder keeps a 64-bit FIFO: between
	// two range-coder normalisations only the order of the bits matters, and
	// every normalisation first writes all complete bytes (flushBuffer<false>),
	// so batching the byte writes does not move any byte.  len <= 56.
	inline void bits_code(uint32_t bits, uint32_t len)
	{
		if (ebits_ + len > 64) empty_buffer();
		ebuf_ = (ebuf_ << len) | bits;
		ebits_ += len;
	}
	inline uint32_t bits_decode(uint32_t len)             // bitsDecode, muxcodec.h:233-239
	{
		if (nbits_ < len) fill_buffer(len);
		nbits_ -= len;
		return (buffer_ >> nbits_) & ((1u << len) - 1);
	}
	// canonical-table Huffman decode (huffDecode, muxcodec.h:241-276)
	uint32_t huff_decode(int table_is_high, int idx);
	// huffDecode(const sHuffSym*) (muxcodec.h:242-253): one entry per code
	// length, codes left-aligned to 16 bits, longest last (code 0)
	uint32_t huff_decode_table(const HuffSym* table);
	void golomb_lin_code(uint32_t nb, int k, int m);          // muxcodec.cpp:466-493
	uint32_t golomb_lin_decode(int k, int m);                 // muxcodec.cpp:495-514

	void taboo_code(uint32_t nb);           // muxcodec.cpp:210-240 (n = 2)
	uint32_t taboo_decode();                // muxcodec.cpp:242-280
	void enum_code(uint32_t bits, uint32_t k, uint32_t nmax);   // muxcodec.cpp:341-365
	uint32_t enum_decode(uint32_t k, uint32_t nmax);            // muxcodec.cpp:381-405
	void max_code(uint32_t value, uint32_t max);                // muxcodec.cpp:516-524
	uint32_t max_decode(uint32_t max);                          // muxcodec.cpp:526-534

	// decoder state, copied into registers by the band decoder (decoder.cpp)
	struct DecState {
		uint32_t range, low, code, nbits, buffer;
		const uint8_t* p;
		const uint8_t* limit;
		bool ovf;
	};
	DecState dec_state() const { return {range_, low_, code_, nbits_, buffer_, p_, limit_, overflow_}; }
	// encoder state, copied into registers by the record encoder (encoder.cpp)
	struct EncState {
		uint32_t range, low, outcount, ebits;
		uint64_t ebuf;
		uint8_t *p, *limit, *reserved;
		uint8_t* last[4];
		bool ovf;
	};
	EncState enc_state() const
	{
		return {range_, low_, outcount_, ebits_, ebuf_, p_, limit_, reserved_, {last_[0], last_[1], last_[2], last_[3]}, overflow_};
	}
	void set_enc_state(const EncState& e)
	{
		range_ = e.range; low_ = e.low; outcount_ = e.outcount; ebits_ = e.ebits; ebuf_ = e.ebuf;
		p_ = e.p; reserved_ = e.reserved; overflow_ = e.ovf;
		for (int i = 0; i < 4; i++) last_[i] = e.last[i];
	}
	void set_dec_state(const DecState& d)
	{
		range_ = d.range; low_ = d.low; code_ = d.code; nbits_ = d.nbits; buffer_ = d.buffer;
		p_ = const_cast<uint8_t*>(d.p); overflow_ = d.ovf;
	}

private:
	void normalize_enc();
	void normalize_dec();
	void empty_buffer();
	void flush_buffer(bool end);
	void fill_buffer(uint32_t len);
	inline void put(uint8_t* slot, uint8_t v) { if (slot < limit_) *slot = v; else overflow_ = true; }

	uint8_t *base_ = nullptr, *p_ = nullptr, *init_ = nullptr, *limit_ = nullptr;
	uint8_t *last_[4] = {nullptr, nullptr, nullptr, nullptr}, *reserved_ = nullptr;
	uint8_t* owned_ = nullptr;              // decoder copy
	size_t owned_cap_ = 0;                  // its size when reused (init_decoder_payload)
	uint32_t range_ = 0, low_ = 0, code_ = 0, outcount_ = 0, nbits_ = 0, buffer_ = 0;
	uint64_t ebuf_ = 0;                     // encoder raw-bit FIFO
	uint32_t ebits_ = 0;
	bool overflow_ = false;
};

// ---------------------------------------------------------------- models
struct BitModel {                           // CBitCodec (16 contexts)
	uint16_t freq[16];
	uint8_t shift[16], mps[16];
	void init();
	inline void adj(int c);
	inline void code(Mux& m, uint32_t sym, int c);
	inline uint32_t decode(Mux& m, int c);
};

struct GeomModel {                          // CGeomCodec (16 contexts)
	uint16_t freq[16];
	uint8_t idx[16];
	void init(const uint8_t* kinit);
	inline void adj(int c);
	inline void code(Mux& m, uint32_t sym, int c);
	inline uint32_t decode(Mux& m, int c);
	// code sym then one raw sign bit, the remainder and the sign as one chunk
	inline void code_signed(Mux& m, uint32_t sym, uint32_t sign, int c);
};

// --------------------------------------------------------- band scans
// Views of a band in host memory (arena layout: pitch in elements).
struct BandView {
	void* p = nullptr;
	int pitch = 0, dx = 0, dy = 0, is_int = 0;
};

// CBandCodec::pred (LL DPCM), src/lib/bandcodec.cpp:62-104
void pred_encode(Mux& m, const BandView& b);
void pred_decode(Mux& m, const BandView& b);
// CBandCodec::tree, src/lib/bandcodec.cpp:484-589.  par.p == nullptr: no parent.
void tree_encode(Mux& m, const BandView& b, const BandView& par, bool high, bool has_child);
void tree_decode(Mux& m, const BandView& b, const BandView& par, bool high, bool has_child);
// The band writes of tree<encode> without the coding (entropy.cpp): applied
// coarse -> fine after the record encoder, the pyramid ends in CodeBand's state.
void tree_encode_state(const BandView& b, const BandView& par, bool has_child);
// Register-resident decoder of one band (decoder.cpp), same semantics as
// tree_decode.
void tree_decode_fast(Mux& m, const BandView& b, const BandView& par, bool high, bool has_child);
// The video codec's motion-vector field (COBMC::encode / decode,
// src/lib/obmc.cpp:344-440): dimx x dimy vectors, x in the low 16 bits, y in
// the high 16 (sMotionVector, obmc.h:29-35), MV_INTRA = 0x80008000.
void mv_encode(Mux& m, const uint32_t* mv, int dimx, int dimy);
void mv_decode(Mux& m, uint32_t* mv, int dimx, int dimy);
// Encoder over GPU block records (symbols.h), coder state in registers
// (encoder.cpp): rec / pin in raster block order; pin == nullptr for a band
// without a parent (the coarsest level).
void tree_encode_records_fast(Mux& m, const uint64_t* rec, const uint8_t* pin, const BandView& b, bool high);
// The same for a 16-bit band whose values come from the frame's compacted
// stream (compact.hip) instead of b's samples (b gives the geometry): *cp is
// advanced past the band's values.
// tree_decode_fast of a finest-level 16-bit band (no children) into the
// compacted layout k_cmp_expand reads: per block in walk order its mask of
// decoded positions (mask[], one per block), every 64 blocks the value count
// so far (chunk_off[]), the values in walk order (vals[]); returns the value
// count.  b gives the geometry (its samples are not written).
uint32_t tree_decode_compact(Mux& m, const BandView& b, const BandView& par, uint16_t* mask, uint32_t* chunk_off,
                             int16_t* vals);
void tree_encode_records_compact(Mux& m, const uint64_t* rec, const uint8_t* pin, const BandView& b, bool high,
                                 const int16_t** cp);
// The same band split in two halves (encoder.cpp): the modelling alone,
// recording the coder calls as events into ev (grown as needed; returns the
// count) -- bands model independently, every model is per band
// (bandcodec.cpp:487-507) -- and the serial replay of those events into the
// stream.  tree_model_records + replay_events == tree_encode_records_fast.
struct EvBuf {                     // a growable event list (no zero fill), kept across frames
	uint64_t* p = nullptr;
	size_t cap = 0;
	EvBuf() = default;
	EvBuf(const EvBuf&) = delete;
	EvBuf& operator=(const EvBuf&) = delete;
	EvBuf(EvBuf&& o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr; o.cap = 0; }
	EvBuf& operator=(EvBuf&& o) noexcept { std::swap(p, o.p); std::swap(cap, o.cap); return *this; }
	~EvBuf() { delete[] p; }
	void grow(size_t n)
	{
		uint64_t* q = new uint64_t[n];
		if (p) { std::copy(p, p + std::min(cap, n), q); delete[] p; }
		p = q;
		cap = n;
	}
};
size_t tree_model_records(EvBuf& ev, const uint64_t* rec, const uint8_t* pin, const BandView& b, bool high);
void replay_events(Mux& m, const uint64_t* ev, size_t n);

// One plane's CodeBand serial half with the bands modelled in parallel
// (encoder.cpp): LL DPCM (pred_encode) on the calling thread, every band's
// modelling a task of `pool` (largest bands first), the replays in coding
// order on the calling thread as each band's events complete.  Byte-identical
// to pred_encode + tree_encode_records_fast over the same bands in order.
struct BandRecs {
	const uint64_t* rec;
	const uint8_t* pin;
	BandView v;
	bool high;
	// a compacted payload (compact.hip): this band's values in walk order,
	// read in place of the dense band; null: the band itself
	const int16_t* cvals = nullptr;
};
// the values a band's walk consumes from a compacted payload: the popcount of
// every block's record mask (read or skipped)
size_t band_value_count(const uint64_t* rec, const BandView& b);
class Pool;
void encode_bands_split(Mux& m, Pool& pool, std::vector<EvBuf>& bufs, const BandView& ll, const BandRecs* bands, int n);

}  // namespace ric
