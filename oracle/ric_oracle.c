/* oracle/ric_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + "port" CPU
 * baseline).  Never linked into, or called by, the product path.
 *
 * Clean-room C restatement of the reference .ric encode/decode path.  Every
 * function cites the reference file:line it restates (paths relative to the
 * reference repository root).  Pinned against the reference library itself
 * (oracle/_ref, built from the reference sources by oracle/Makefile) and the
 * committed golden vectors in tests/golden/.
 *
 * Integer semantics: the reference stores bands as `short` above level_chg and
 * `int` at or below it, truncating at every C-typed store.  Here every band is
 * held as int32 and TR() truncates to int16 exactly where the reference stores
 * a short.  Built with -fwrapv, so int overflow wraps like the reference's x86
 * build does.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "ric_oracle.h"
#include "huff_tables.inc"

#define MAXLEV 16
#define INSIGNIF (-0x8000)          /* src/lib/bandcodec.cpp:113 */

/* ---------------------------------------------------------------- helpers */
/* src/lib/utils.h:79-138 */
static inline int s2u(int s) { int u = -(2 * s + 1); return u ^ (u >> 31); }
static inline int u2s(int u) { return (u >> 1) ^ -(u & 1); }
static inline int s2u_(int s) { int m = s >> 31; return (2 * s + m) ^ (m * 2); }
static inline int u2s_(int u) { int m = -(u & 1); return ((u >> 1) + m) ^ m; }
static inline int iabs(int s) { return s < 0 ? -s : s; }
static inline int bitlen(uint32_t v) { int r = 0; while (v) { r++; v >>= 1; } return r; }

/* C-typed store / unsigned view: sh != 0 means the band type is `short` */
static inline int TR(int sh, int v) { return sh ? (int)(int16_t)v : v; }
static inline uint32_t UC(int sh, int v) { return sh ? (uint32_t)(uint16_t)v : (uint32_t)v; }

/* CWavelet2D::mult08, src/lib/wavelet2d.cpp:307-318.  It is a template on
 * its argument's type: mult08(i[1]) runs on C (short truncations), but the
 * calls on a sum, mult08(i[1] + i[3]), deduce C = int -- the sum is not
 * truncated and the steps run in int (sh 0 here). */
static inline int mult08(int sh, int a)
{
	a = TR(sh, a);
	a = TR(sh, a - (a >> 2));
	a = TR(sh, a + (a >> 4));
	return TR(sh, a + (a >> 8));
}

/* ------------------------------------------------------- 1-D lifting lines */
/* Each line is a strided int32 view.  The reference runs the same lifting on
 * rows (TransLine*) and, through its rolling row window, on columns; both are
 * the same 4-step (9/7) or 2-step (5/3) lifting with symmetric boundaries. */
#define X(n) x[(long)(n) * st]

/* TransLine97, src/lib/wavelet2d.cpp:320-359 (len >= 4) */
static void line97(int sh, int32_t* x, long st, int len)
{
	int last = len - 1, n, t;
	/* P1 on even samples */
	X(0) = TR(sh, X(0) - X(1) * 3);
	for (n = 2; n < last; n += 2) { t = TR(sh, X(n - 1) + X(n + 1)); X(n) = TR(sh, X(n) - (t + (t >> 1))); }
	if (!(len & 1) == 0) X(last) = TR(sh, X(last) - (X(last - 1) * 2 + X(last - 1)));
	/* U1 on odd samples */
	for (n = 1; n < last; n += 2) X(n) = TR(sh, X(n) - ((X(n - 1) + X(n + 1)) >> 4));
	if (!(len & 1)) X(last) = TR(sh, X(last) - (X(last - 1) >> 3));
	/* P2 on even samples */
	X(0) = TR(sh, X(0) + 2 * mult08(sh, X(1)));
	for (n = 2; n < last; n += 2) X(n) = TR(sh, X(n) + mult08(0, X(n - 1) + X(n + 1)));
	if (len & 1) X(last) = TR(sh, X(last) + 2 * mult08(sh, X(last - 1)));
	/* U2 on odd samples */
	for (n = 1; n < last; n += 2) { t = TR(sh, X(n - 1) + X(n + 1)); X(n) = TR(sh, X(n) + ((t >> 1) - (t >> 5))); }
	if (!(len & 1)) X(last) = TR(sh, X(last) + (X(last - 1) - (X(last - 1) >> 4)));
}

/* TransLine97I, src/lib/wavelet2d.cpp:361-405 */
static void line97i(int sh, int32_t* x, long st, int len)
{
	int last = len - 1, n, t;
	for (n = 1; n < last; n += 2) { t = TR(sh, X(n - 1) + X(n + 1)); X(n) = TR(sh, X(n) - ((t >> 1) - (t >> 5))); }
	if (!(len & 1)) X(last) = TR(sh, X(last) - (X(last - 1) - (X(last - 1) >> 4)));
	X(0) = TR(sh, X(0) - 2 * mult08(sh, X(1)));
	for (n = 2; n < last; n += 2) X(n) = TR(sh, X(n) - mult08(0, X(n - 1) + X(n + 1)));
	if (len & 1) X(last) = TR(sh, X(last) - 2 * mult08(sh, X(last - 1)));
	for (n = 1; n < last; n += 2) X(n) = TR(sh, X(n) + ((X(n - 1) + X(n + 1)) >> 4));
	if (!(len & 1)) X(last) = TR(sh, X(last) + (X(last - 1) >> 3));
	X(0) = TR(sh, X(0) + X(1) * 3);
	for (n = 2; n < last; n += 2) { t = TR(sh, X(n - 1) + X(n + 1)); X(n) = TR(sh, X(n) + (t + (t >> 1))); }
	if (len & 1) X(last) = TR(sh, X(last) + X(last - 1) * 3);
}

/* TransLine53, src/lib/wavelet2d.cpp:593-611 (len >= 2) */
static void line53(int sh, int32_t* x, long st, int len)
{
	int last = len - 1, n;
	X(0) = TR(sh, X(0) - X(1));
	for (n = 2; n < last; n += 2) X(n) = TR(sh, X(n) - ((X(n - 1) + X(n + 1)) >> 1));
	if (len & 1) X(last) = TR(sh, X(last) - X(last - 1));
	for (n = 1; n < last; n += 2) X(n) = TR(sh, X(n) + ((X(n - 1) + X(n + 1)) >> 2));
	if (!(len & 1)) X(last) = TR(sh, X(last) + (X(last - 1) >> 1));
}

/* TransLine53I, src/lib/wavelet2d.cpp:613-634 */
static void line53i(int sh, int32_t* x, long st, int len)
{
	int last = len - 1, n;
	for (n = 1; n < last; n += 2) X(n) = TR(sh, X(n) - ((X(n - 1) + X(n + 1)) >> 2));
	if (!(len & 1)) X(last) = TR(sh, X(last) - (X(last - 1) >> 1));
	X(0) = TR(sh, X(0) + X(1));
	for (n = 2; n < last; n += 2) X(n) = TR(sh, X(n) + ((X(n - 1) + X(n + 1)) >> 1));
	if (len & 1) X(last) = TR(sh, X(last) + X(last - 1));
}

/* TransLineHaar(I), src/lib/wavelet2d.cpp:766-786: pairs only, an odd tail is untouched */
static void linehaar(int sh, int32_t* x, long st, int len)
{
	for (int n = 0; n + 1 < len; n += 2) {
		X(n) = TR(sh, X(n) - X(n + 1));
		X(n + 1) = TR(sh, X(n + 1) + (X(n) >> 1));
	}
}
static void linehaari(int sh, int32_t* x, long st, int len)
{
	for (int n = 0; n + 1 < len; n += 2) {
		X(n + 1) = TR(sh, X(n + 1) - (X(n) >> 1));
		X(n) = TR(sh, X(n) + X(n + 1));
	}
}
#undef X

/* ----------------------------------------------------------- band pyramid */
typedef struct {
	int dx, dy, sh;          /* dims, short-typed? */
	float weight;
	int32_t* v;              /* dx*dy, row-major */
	uint32_t* rd;            /* pRD, ceil(dx/4)*ceil(dy/4) */
} band_t;

enum { BD = 0, BH = 1, BV = 2, BL = 3 };

typedef struct {
	int nlev;                /* levels actually built */
	int w[MAXLEV], h[MAXLEV];/* input dims per level (0 = finest) */
	int sh[MAXLEV];
	band_t b[MAXLEV][4];     /* L only used at the coarsest level */
} pyr_t;

/* CWavelet2D::Init, src/lib/wavelet2d.cpp:69-81; CBand::Init src/lib/band.cpp:51-65 */
static void pyr_init(pyr_t* p, int w, int h, int levels, int lc)
{
	memset(p, 0, sizeof(*p));
	int l = 0, lev = levels;
	while (1) {
		p->w[l] = w; p->h[l] = h;
		p->sh[l] = !(lev <= lc);
		int dims[4][2] = {{(w + 1) >> 1, (h + 1) >> 1}, {w >> 1, (h + 1) >> 1},
		                  {(w + 1) >> 1, h >> 1}, {w >> 1, h >> 1}};
		int last = !(lev > 1 && w > 15 && h > 15);
		for (int b = 0; b < (last ? 4 : 3); b++) {
			band_t* B = &p->b[l][b];
			B->dx = dims[b][0]; B->dy = dims[b][1]; B->sh = p->sh[l];
			B->weight = 1.f;
			B->v = calloc((size_t)B->dx * B->dy + 1, sizeof(int32_t));
			B->rd = calloc((size_t)((B->dx + 3) / 4) * ((B->dy + 3) / 4) + 1, sizeof(uint32_t));
		}
		l++;
		if (last) break;
		w >>= 1; h >>= 1; lev--;
	}
	p->nlev = l;
}

static void pyr_free(pyr_t* p)
{
	for (int l = 0; l < p->nlev; l++)
		for (int b = 0; b < 4; b++) { free(p->b[l][b].v); free(p->b[l][b].rd); }
}

/* CWavelet2D::SetWeight, src/lib/wavelet2d.cpp:1009-1032 (float32) */
static void pyr_weights(pyr_t* p, int trans)
{
	float scale = trans == 0 ? 1.149604398f * 1.149604398f : 2.f;
	float bw = 1.f;
	float pv = 0, pl = 0;    /* finer level's V and L weights */
	for (int l = 0; l < p->nlev; l++) {
		float d, v, hh, ll;
		if (l == 0) { d = bw / scale; v = bw; hh = bw; ll = bw * scale; }
		else { d = pv; v = pl; hh = v; ll = v * scale; }
		p->b[l][BD].weight = d; p->b[l][BV].weight = v; p->b[l][BH].weight = hh; p->b[l][BL].weight = ll;
		pv = v; pl = ll;
	}
}

static band_t* coarsest_ll(pyr_t* p) { return &p->b[p->nlev - 1][BL]; }

/* ---------------------------------------------------------- forward DWT */
/* CWavelet2D::Transform + Transform97/53/Haar, src/lib/wavelet2d.cpp:407-492,
 * 636-692, 788-819, 926-956.  Rows first, then columns (the reference's rolling
 * window applies the column lifting after each row is row-transformed, which is
 * the same computation), then (even,even)->D, (even,odd)->H, (odd,even)->V,
 * (odd,odd)->LL.  The LL feeds the next level; at the short->int switch it is
 * widened exactly (src/lib/wavelet2d.cpp:937-950). */
static void pyr_forward(pyr_t* p, const int32_t* img, int trans)
{
	int32_t* cur = malloc(sizeof(int32_t) * (size_t)p->w[0] * p->h[0]);
	memcpy(cur, img, sizeof(int32_t) * (size_t)p->w[0] * p->h[0]);
	for (int l = 0; l < p->nlev; l++) {
		int w = p->w[l], h = p->h[l], sh = p->sh[l];
		for (long i = 0; i < (long)w * h; i++) cur[i] = TR(sh, cur[i]);
		if (trans == 0) {
			for (int y = 0; y < h; y++) line97(sh, cur + (long)y * w, 1, w);
			for (int x = 0; x < w; x++) line97(sh, cur + x, w, h);
		} else if (trans == 1) {
			for (int y = 0; y < h; y++) line53(sh, cur + (long)y * w, 1, w);
			for (int x = 0; x < w; x++) line53(sh, cur + x, w, h);
		} else {
			for (int y = 0; y < h; y++) linehaar(sh, cur + (long)y * w, 1, w);
			for (int x = 0; x < w; x++) linehaar(sh, cur + x, w, h);
		}
		int last = l == p->nlev - 1;
		int32_t* nxt = malloc(sizeof(int32_t) * ((size_t)(w >> 1) * (h >> 1) + 1));
		/* Haar only emits complete row pairs (src/lib/wavelet2d.cpp:802) */
		int hrows = trans == 2 ? (h & ~1) : h;
		for (int y = 0; y < hrows; y++)
			for (int x = 0; x < w; x++) {
				int v = cur[(long)y * w + x];
				if (!(y & 1)) {
					band_t* B = &p->b[l][(x & 1) ? BH : BD];
					B->v[(long)(y >> 1) * B->dx + (x >> 1)] = v;
				} else if (!(x & 1)) {
					band_t* B = &p->b[l][BV];
					B->v[(long)(y >> 1) * B->dx + (x >> 1)] = v;
				} else {
					if (last) { band_t* B = &p->b[l][BL]; B->v[(long)(y >> 1) * B->dx + (x >> 1)] = v; }
					else nxt[(long)(y >> 1) * (w >> 1) + (x >> 1)] = v;
				}
			}
		free(cur);
		cur = nxt;
	}
	free(cur);
}

/* --------------------------------------------------------- inverse DWT */
/* CBand::Init row alignment, src/lib/band.cpp:57 (ALIGN = 32 bytes) */
static long align_row(int dx, int sh) { int ss = sh ? 2 : 4; return ((long)dx * ss + 31) / 32 * 32 / ss; }

/* CWavelet2D::TransformI + Transform97I/53I/HaarI, src/lib/wavelet2d.cpp:494-591,
 * 694-764, 821-855, 960-990.  Coarsest level first; the int->short copy-back at
 * the switch truncates (src/lib/wavelet2d.cpp:971-980). */
static void pyr_inverse(pyr_t* p, int trans, int32_t* out)
{
	int32_t* ll = NULL;
	for (int l = p->nlev - 1; l >= 0; l--) {
		int w = p->w[l], h = p->h[l], sh = p->sh[l];
		int last = l == p->nlev - 1;
		int32_t* cur = calloc((size_t)w * h + 1, sizeof(int32_t));
		int hrows = trans == 2 ? (h & ~1) : h;
		for (int y = 0; y < hrows; y++)
			for (int x = 0; x < w; x++) {
				int v;
				if (trans == 1 && y == 2 && (x & 1)) {
					/* Transform53I, src/lib/wavelet2d.cpp:715 reads the second H row
					 * with the D band's stride: in[3][in_stride[2] + k/2].  Replay
					 * it on the reference's 32-byte-aligned row layout; alignment
					 * padding reads as 0 (the decoder Clear()s every band). */
					band_t* D = &p->b[l][BD]; band_t* H = &p->b[l][BH];
					long f = align_row(D->dx, D->sh) + (x >> 1);
					long ha = align_row(H->dx, H->sh);
					long r = f / ha, c = f % ha;
					v = c < H->dx ? H->v[r * H->dx + c] : 0;
				} else if (!(y & 1)) {
					band_t* B = &p->b[l][(x & 1) ? BH : BD];
					v = B->v[(long)(y >> 1) * B->dx + (x >> 1)];
				} else if (!(x & 1)) {
					band_t* B = &p->b[l][BV];
					v = B->v[(long)(y >> 1) * B->dx + (x >> 1)];
				} else if (last) {
					band_t* B = &p->b[l][BL];
					v = B->v[(long)(y >> 1) * B->dx + (x >> 1)];
				} else {
					v = ll[(long)(y >> 1) * (w >> 1) + (x >> 1)];
				}
				cur[(long)y * w + x] = TR(sh, v);
			}
		if (trans == 0) {
			for (int x = 0; x < w; x++) line97i(sh, cur + x, w, h);
			for (int y = 0; y < h; y++) line97i(sh, cur + (long)y * w, 1, w);
		} else if (trans == 1) {
			for (int x = 0; x < w; x++) line53i(sh, cur + x, w, h);
			for (int y = 0; y < h; y++) line53i(sh, cur + (long)y * w, 1, w);
		} else {
			for (int x = 0; x < w; x++) linehaari(sh, cur + x, w, hrows);
			for (int y = 0; y < hrows; y++) linehaari(sh, cur + (long)y * w, 1, w);
		}
		free(ll);
		/* the reconstructed LL of the finer level is stored as the finer level's C */
		if (l > 0) for (long i = 0; i < (long)w * h; i++) cur[i] = TR(p->sh[l - 1], cur[i]);
		ll = cur;
	}
	memcpy(out, ll, sizeof(int32_t) * (size_t)p->w[0] * p->h[0]);
	free(ll);
}

/* ------------------------------------------------------------------ mux */
/* CMuxCodec, src/lib/muxcodec.h:66-277, src/lib/muxcodec.cpp */
typedef struct {
	uint8_t *p, *init, *last[4], *reserved, *end;   /* end: decoder read guard */
	uint32_t range, low, code, outcount, nbits, buffer;
	uint32_t nbtaboo[32], sumtaboo[32], ntaboo;
} mux_t;

static void mux_taboo(mux_t* m, uint32_t k)   /* initTaboo, muxcodec.cpp:113-129 */
{
	uint32_t i;
	m->nbtaboo[0] = 1; m->ntaboo = k;
	for (i = 1; i < k; i++) m->nbtaboo[i] = 1u << (i - 1);
	for (i = k; i < 32; i++) {
		uint32_t acc = m->nbtaboo[i - k];
		for (uint32_t j = i - k + 1; j < i; j++) acc += m->nbtaboo[j];
		m->nbtaboo[i] = acc;
	}
	m->sumtaboo[0] = m->nbtaboo[0];
	for (i = 1; i < 32; i++) m->sumtaboo[i] = m->sumtaboo[i - 1] + m->nbtaboo[i];
}

static void mux_enc_init(mux_t* m, uint8_t* buf)     /* initCoder, muxcodec.cpp:36-49 */
{
	memset(m, 0, sizeof(*m));
	m->low = 0; m->range = 1u << 16;
	m->p = buf + 4; m->init = buf + 2;
	for (int i = 0; i < 4; i++) m->last[i] = buf + i;
	mux_taboo(m, 2);
}

static void mux_dec_init(mux_t* m, uint8_t* buf)     /* initDecoder, muxcodec.cpp:51-61 */
{
	memset(m, 0, sizeof(*m));
	m->range = 1u << 16;
	m->init = buf + 2; m->p = buf + 2;
	m->code = m->low = (m->p[0] << 8) | m->p[1];
	m->p += 2;
	m->end = NULL;
	mux_taboo(m, 2);
}

/* Decoder read guard: a desynchronised stream (the reference's maxDecode(0)
 * case, muxcodec.cpp:526-534) can walk off the buffer; valid streams never get
 * close.  The reference has no guard (it may crash there). */
static inline uint8_t next_byte(mux_t* m)
{
	if (m->end && m->p >= m->end) return 0;
	return *m->p++;
}

static void mux_empty(mux_t* m)                      /* emptyBuffer, muxcodec.cpp:536-548 */
{
	do {
		m->nbits -= 8;
		uint8_t b = (uint8_t)(m->buffer >> m->nbits);
		if (!m->reserved) *m->p++ = b; else { *m->reserved = b; m->reserved = 0; }
	} while (m->nbits >= 8);
}

static void mux_flush(mux_t* m, int end)             /* flushBuffer, muxcodec.cpp:550-570 */
{
	if (m->nbits >= 8) mux_empty(m);
	if (m->nbits > 0) {
		if (end) {
			uint8_t b = (uint8_t)(m->buffer << (8 - m->nbits));
			if (!m->reserved) *m->p++ = b; else { *m->reserved = b; m->reserved = 0; }
			m->nbits = 0;
		} else if (!m->reserved) {
			m->reserved = m->p++;
		}
	}
}

static void mux_norm_enc(mux_t* m)                   /* normalize_enc, muxcodec.cpp:63-74 */
{
	mux_flush(m, 0);
	do {
		*m->last[m->outcount++ & 3] = (uint8_t)(m->low >> 24);
		if (((m->low + m->range - 1) ^ m->low) >= 0x01000000u)
			m->range = -m->low & 4095u;
		m->last[(m->outcount + 3) & 3] = m->p++;
		m->range <<= 8;
		m->low <<= 8;
	} while (m->range <= 4096u);
}

static void mux_norm_dec(mux_t* m)                   /* normalize_dec, muxcodec.cpp:76-85 */
{
	do {
		if (((m->code - m->low + m->range - 1) ^ (m->code - m->low)) >= 0x01000000u)
			m->range = (m->low - m->code) & 4095u;
		uint8_t b = next_byte(m);
		m->low = (m->low << 8) | b;
		m->code = (m->code << 8) | b;
		m->range <<= 8;
	} while (m->range <= 4096u);
}

static uint8_t* mux_end(mux_t* m)                    /* endCoding, muxcodec.cpp:87-106 */
{
	mux_flush(m, 1);
	if (m->range <= 4096u) mux_norm_enc(m);
	uint32_t last_out = 0x200 | 'W';
	if ((m->low & 4095u) > (last_out & 4095u)) m->low += 4096u;
	m->low = (m->low & ~4095u) | (last_out & 4095u);
	*m->last[m->outcount & 3] = (uint8_t)(m->low >> 24);
	*m->last[(m->outcount + 1) & 3] = (uint8_t)(m->low >> 16);
	*m->last[(m->outcount + 2) & 3] = (uint8_t)(m->low >> 8);
	*m->last[(m->outcount + 3) & 3] = (uint8_t)m->low;
	return m->p;
}

static inline void code_bin(mux_t* m, uint32_t freq, int bit)  /* codeBin, muxcodec.h:156-163 */
{
	if (m->range <= 4096u) mux_norm_enc(m);
	uint32_t tmp = (m->range * freq) >> 12;
	m->low += tmp & -(uint32_t)bit;
	m->range = tmp + ((m->range - 2 * tmp) & -(uint32_t)bit);
}

static inline int get_bit(mux_t* m, uint32_t freq)             /* getBit, muxcodec.h:205-213 */
{
	if (m->range <= 4096u) mux_norm_dec(m);
	uint32_t tmp = (m->range * freq) >> 12;
	uint32_t tst = (uint32_t)((m->low < tmp) - 1);
	m->low -= tmp & tst;
	m->range = tmp + ((m->range - 2 * tmp) & tst);
	return (int)(0u - tst);
}

static inline void bits_code(mux_t* m, uint32_t bits, uint32_t len)  /* bitsCode, muxcodec.h:225-231 */
{
	if (m->nbits + len > 32) mux_empty(m);
	m->buffer = (m->buffer << len) | bits;
	m->nbits += len;
}

static void mux_fill(mux_t* m, uint32_t len)                    /* fillBuffer, muxcodec.cpp:572-579 */
{
	if (len > 32) len = 32;
	do {
		m->nbits += 8;
		m->buffer = (m->buffer << 8) | next_byte(m);
	} while (m->nbits < len);
}

static inline uint32_t bits_decode(mux_t* m, uint32_t len)     /* bitsDecode, muxcodec.h:233-239 */
{
	if (len > 24) len = 24;                           /* desync guard only */
	if (m->nbits < len) mux_fill(m, len);
	m->nbits -= len;
	return (m->buffer >> m->nbits) & ((1u << len) - 1);
}

/* tabooCode / tabooDecode (n = 2), muxcodec.cpp:210-280 */
static void taboo_code(mux_t* m, uint32_t nb)
{
	int i = 0, l;
	uint32_t r = 0, nt = m->ntaboo;
	while (m->sumtaboo[i] <= nb) i++;
	if (i == 0) { bits_code(m, 0, nt); return; }
	l = i; i--;
	nb -= m->sumtaboo[i];
	while (i > (int)nt) {
		uint32_t k = i - nt + 1, cnt = m->nbtaboo[k], j = 0;
		while (nb >= cnt) cnt += m->nbtaboo[k + ++j];
		nb -= cnt - m->nbtaboo[k + j];
		j = nt - j;
		r = (r << j) | 1;
		i -= j;
	}
	if (i == (int)nt) nb++;
	r = ((((r << i) | (nb & ((1u << i) - 1))) << 1) | 1) << nt;
	bits_code(m, r, l + nt);
}

static uint32_t taboo_decode(mux_t* m)
{
	int i, l = m->ntaboo;
	uint32_t nb = 0, nt = m->ntaboo;
	if (m->nbits < nt) mux_fill(m, nt);
	uint32_t t = ((1u << nt) - 1) << (m->nbits - nt);
	while ((~m->buffer & t) != t) {
		l++;
		if (l > (int)m->nbits) { mux_fill(m, l); t <<= 8; }
		t >>= 1;
	}
	m->nbits -= l;
	uint32_t cd = m->buffer >> (m->nbits + nt + 1);
	i = l - nt;
	if (i > 0) { i--; nb += m->sumtaboo[i]; }
	while (i > (int)nt) {
		uint32_t j = 1;
		while (((cd >> (i - j)) & 1) == 0) j++;
		nb += m->sumtaboo[i - j] - m->sumtaboo[i - nt];
		i -= j;
	}
	if (i == (int)nt) nb -= 1;
	nb += cd & ((1u << i) - 1);
	return nb;
}

/* enumerative codes, muxcodec.cpp:282-413 */
static uint16_t CNK[8][16];
static const uint8_t CNK_LEN[16][8] = {
	{0,0,0,0,0,0,0,0},{1,0,0,0,0,0,0,0},{2,2,0,0,0,0,0,0},{2,3,2,0,0,0,0,0},
	{3,4,4,3,0,0,0,0},{3,4,5,4,3,0,0,0},{3,5,6,6,5,3,0,0},{3,5,6,7,6,5,3,0},
	{4,6,7,7,7,7,6,4},{4,6,7,8,8,8,7,6},{4,6,8,9,9,9,9,8},{4,7,8,9,10,10,10,9},
	{4,7,9,10,11,11,11,11},{4,7,9,10,11,12,12,12},{4,7,9,11,12,13,13,13},{4,7,10,11,13,13,14,14}};
static const uint16_t CNK_LOST[16][8] = {
	{0,0,0,0,0,0,0,0},{0,0,0,0,0,0,0,0},{1,1,0,0,0,0,0,0},{0,2,0,0,0,0,0,0},
	{3,6,6,3,0,0,0,0},{2,1,12,1,2,0,0,0},{1,11,29,29,11,1,0,0},{0,4,8,58,8,4,0,0},
	{7,28,44,2,2,44,28,7},{6,19,8,46,4,46,8,19},{5,9,91,182,50,50,182,91},
	{4,62,36,17,232,100,232,17},{3,50,226,309,761,332,332,761},{2,37,148,23,46,1093,664,1093},
	{1,23,57,683,1093,3187,1757,1757},{0,8,464,228,3824,184,4944,3514}};

static void cnk_init(void)
{
	/* Cnk[k][n] = C(n, k+1): the binomial table of muxcodec.cpp:282-292 */
	for (int k = 0; k < 8; k++)
		for (int n = 0; n < 16; n++) {
			uint32_t c = 1; int kk = k + 1;
			if (n < kk) { CNK[k][n] = 0; continue; }
			for (int i = 1; i <= kk; i++) c = c * (n - kk + i) / i;
			CNK[k][n] = (uint16_t)c;
		}
}

static void enum_code(mux_t* m, uint32_t bits, uint32_t k, uint32_t nmax)
{
	uint32_t code = 0, n = 0, row = 0;
	if (k > ((nmax + 1) >> 1)) { k = nmax - k; bits ^= (1u << nmax) - 1; }
	do {
		if (bits & 1) { code += CNK[row][n]; row++; }
		n++; bits >>= 1;
	} while (bits != 0);
	uint32_t lost = CNK_LOST[nmax - 1][k - 1], len = CNK_LEN[nmax - 1][k - 1];
	if (code < lost) bits_code(m, code, len - 1);
	else bits_code(m, code + lost, len);
}

static uint32_t enum_decode(mux_t* m, uint32_t k, uint32_t nmax)
{
	if (k == 0 || k >= nmax) return k ? (1u << nmax) - 1 : 0;   /* desync guard only */
	int n = nmax - 1;
	uint32_t bits = 0;
	if (k > ((nmax + 1) >> 1)) { k = nmax - k; bits ^= (1u << nmax) - 1; }
	int row = k - 1;
	uint32_t lost = CNK_LOST[nmax - 1][k - 1];
	uint32_t code = bits_decode(m, CNK_LEN[nmax - 1][k - 1] - 1);
	if (code >= lost) code = ((code << 1) | bits_decode(m, 1)) - lost;
	do {
		if (n < 0) break;
		if (code >= CNK[row][n]) { bits ^= 1u << n; code -= CNK[row][n]; row--; }
		n--;
	} while (row >= 0);
	return bits;
}

/* maxCode / maxDecode, muxcodec.cpp:516-534 (incl. the max == 0 asymmetry) */
static void max_code(mux_t* m, uint32_t value, uint32_t max)
{
	uint32_t len = bitlen(max), lost = (1u << len) - max - 1;
	if (value < lost) bits_code(m, value, len - 1);
	else bits_code(m, value + lost, len);
}

static uint32_t max_decode(mux_t* m, uint32_t max)
{
	uint32_t value = 0, len = bitlen(max), lost = (1u << len) - max - 1;
	if (len > 1) value = bits_decode(m, len - 1);
	if (value >= lost) value = ((value << 1) | bits_decode(m, 1)) - lost;
	return value;
}

/* Huffman decode of the static tables: huffDecode, muxcodec.h:241-276.  The
 * symbol is found from the {code,len} encoder table by prefix match; the
 * stream pointer / bit-buffer bookkeeping is the reference's. */
static uint32_t huff_decode(mux_t* m, const uint16_t* tab, int nsym)
{
	uint32_t code = (((m->buffer << 16) | (m->p[0] << 8) | m->p[1]) >> m->nbits) & 0xFFFF;
	int s, len = 0;
	for (s = 0; s < nsym; s++) {
		len = tab[s] & 31;
		if ((code >> (16 - len)) == (uint32_t)(tab[s] >> 5)) break;
	}
	if (s == nsym) { s = 0; len = tab[0] & 31; }  /* corrupt stream: any defined behaviour */
	m->p -= (int)(m->nbits - len) >> 3;
	if (m->end && m->p > m->end) m->p = m->end;
	if ((int)m->nbits < len) m->buffer = m->p[-1];
	m->nbits = (m->nbits - len) & 7;
	return s;
}

/* --------------------------------------------------------- bit models */
/* CBitCodec, src/lib/bitcodec.h:38-93, src/lib/bitcodec.cpp:31-42 */
static const uint16_t BIT_THRES[11] = {2584, 1512, 745, 371, 185, 92, 46, 23, 12, 6, 3};
typedef struct { uint16_t freq[16]; uint8_t shift[16], mps[16]; } bitm_t;

static void bitm_init(bitm_t* b)
{
	for (int i = 0; i < 16; i++) { b->freq[i] = 2048; b->shift[i] = 0; b->mps[i] = 0; }
}

static inline void bitm_adj(bitm_t* b, int c)
{
	if (b->freq[c] > BIT_THRES[b->shift[c]]) {
		if (b->shift[c] == 0) { b->mps[c] ^= 1; b->freq[c] = 4096 - b->freq[c]; b->shift[c] = 1; }
		else b->shift[c]--;
	} else if (b->shift[c] < 9) b->shift[c]++;
}

static inline int bitm_code(bitm_t* b, mux_t* m, int sym, int c)
{
	uint32_t s = sym ^ b->mps[c];
	code_bin(m, b->freq[c], s ^ 1);
	int sp = 9 - b->shift[c], de = 12 - sp;
	b->freq[c] = (uint16_t)(b->freq[c] + (s << sp) - (b->freq[c] >> de));
	if ((uint16_t)(b->freq[c] - BIT_THRES[b->shift[c] + 1]) > BIT_THRES[b->shift[c]] - BIT_THRES[b->shift[c] + 1])
		bitm_adj(b, c);
	return sym;
}

static inline int bitm_decode(bitm_t* b, mux_t* m, int c)
{
	uint32_t sym = get_bit(m, b->freq[c]) ^ 1;
	int sp = 9 - b->shift[c], de = 12 - sp;
	b->freq[c] = (uint16_t)(b->freq[c] + (sym << sp) - (b->freq[c] >> de));
	sym ^= b->mps[c];
	if ((uint16_t)(b->freq[c] - BIT_THRES[b->shift[c] + 1]) > BIT_THRES[b->shift[c]] - BIT_THRES[b->shift[c] + 1])
		bitm_adj(b, c);
	return sym;
}

/* CGeomCodec, src/lib/geomcodec.h:33-99, src/lib/geomcodec.cpp:31-54 */
static const uint16_t GEO_THRES[11] = {1512, 2584, 3351, 3725, 3911, 4004, 4050, 4073, 4084, 4090, 4093};
static const uint8_t GEO_K[25] = {0,0,0,0,0,0,0,0,0,0,1,2,3,4,5,6,7,8,9,10,11,12,13,14, 14};
static const uint8_t GEO_SHIFT[25] = {10,9,8,7,6,5,4,3,2,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1, 1};
typedef struct { uint16_t freq[16]; uint8_t idx[16]; } geom_t;

static void geom_init(geom_t* g, const uint8_t* kinit)
{
	for (int c = 0; c < 16; c++) {
		g->idx[c] = kinit[c];
		if (g->idx[c] >= 9) g->freq[c] = 2048;
		else g->freq[c] = (GEO_THRES[g->idx[c] - 1] + GEO_THRES[g->idx[c]]) >> 1;
	}
}

static inline void geom_adj(geom_t* g, int c)
{
	int s = GEO_SHIFT[g->idx[c]];
	if (g->freq[c] < GEO_THRES[s - 1]) g->idx[c]++;
	else if (g->idx[c] > 0) g->idx[c]--;
	if (g->idx[c] >= 9) g->freq[c] = 2048;
}

static void geom_code(geom_t* g, mux_t* m, uint32_t sym, int c)
{
	uint32_t k = GEO_K[g->idx[c]], f = g->freq[c];
	int s = GEO_SHIFT[g->idx[c]];
	for (uint32_t l = sym >> k; l > 0; l--) {
		code_bin(m, f, 1);
		g->freq[c] -= g->freq[c] >> (3 + s);
	}
	code_bin(m, f, 0);
	if (k > 0) bits_code(m, sym & ((1u << k) - 1), k);
	g->freq[c] += (4096 - g->freq[c]) >> (3 + s);
	if ((uint16_t)(g->freq[c] - GEO_THRES[s - 1]) > GEO_THRES[s] - GEO_THRES[s - 1]) geom_adj(g, c);
}

static uint32_t geom_decode(geom_t* g, mux_t* m, int c)
{
	uint32_t k = GEO_K[g->idx[c]], f = g->freq[c];
	int s = GEO_SHIFT[g->idx[c]];
	uint32_t l = 0;
	while (get_bit(m, f)) { g->freq[c] -= g->freq[c] >> (3 + s); if (++l > (1u << 20)) break; }
	if (k > 0) l = (l << k) | bits_decode(m, k);
	g->freq[c] += (4096 - g->freq[c]) >> (3 + s);
	if ((uint16_t)(g->freq[c] - GEO_THRES[s - 1]) > GEO_THRES[s] - GEO_THRES[s - 1]) geom_adj(g, c);
	return l;
}

/* ------------------------------------------------------- quantisation */
static const int BLEN[17] = {20, 40, 55, 66, 75, 81, 85, 88, 89, 88, 85, 81, 75, 66, 55, 40, 20};

/* CBandCodec::clen, src/lib/bandcodec.cpp:135-147 (only coef == 1 is used) */
static int clen1(int cnt)
{
	static const uint8_t k[] = {0,0,0,0,0,0,0,0,0,0,0,1,1,1,1,2};
	static const uint8_t lps[] = {3,3,2,2,2,1,1,1,1,1,1,1,1,1,1,1};
	static const uint8_t mps[] = {1,1,2,2,2,5,5,5,5,5,5,5,5,5,5,5};
	(void)lps;
	cnt--;
	return (k[cnt] + 1) * 5 + mps[cnt];
}

/* CBandCodec::makeThres, src/lib/bandcodec.cpp:149-157 */
static void make_thres(int sh, int* thres, int quant, int lambda)
{
	for (int i = 0; i < 16; i++) {
		int t = TR(sh, (quant + ((lambda * (BLEN[i + 1] - BLEN[i] + clen1(i + 1)) + 8) >> 4)) & 0xFFFE);
		if (t > quant * 2) t = TR(sh, quant * 2);
		if (t < (quant & 0xFFFE)) t = TR(sh, quant & 0xFFFE);
		thres[i] = t;
	}
}

/* CBandCodec::tsuqBlock (RD), src/lib/bandcodec.cpp:159-213; returns the
 * non-zero count (the dist/rate book-keeping there is dead). */
static int tsuq_block(int sh, int32_t* cur, int stride, int Q, int iQ, const int* thres)
{
	int var_cnt = 0, cnt = 0;
	int32_t* var[16];
	int T = TR(sh, Q >> 1);
	for (int j = 0; j < 4; j++) {
		int32_t* r = cur + (long)j * stride;
		for (int i = 0; i < 4; i++) {
			int v = r[i];
			if ((uint32_t)(v + T) <= (uint32_t)(2 * T)) { r[i] = 0; continue; }
			v = TR(sh, s2u_(v));
			r[i] = v;
			if (UC(sh, v) < UC(sh, thres[0])) var[var_cnt++] = r + i;
			else {
				cnt++;
				int tmp = (int)(UC(sh, v) >> 1);
				int q = (tmp * iQ + (1 << 15)) >> 16;
				r[i] = TR(sh, (q << 1) | (v & 1));
			}
		}
	}
	if (var_cnt > 0) {
		/* inSort, src/lib/bandcodec.cpp:115-127: stable, unsigned key descending */
		for (int i = 1; i < var_cnt; i++) {
			int32_t* t = var[i];
			int j = i;
			while (j > 0 && UC(sh, *var[j - 1]) < UC(sh, *t)) { var[j] = var[j - 1]; j--; }
			var[j] = t;
		}
		int i = var_cnt - 1;
		while (i >= 0 && *var[i] < thres[i + cnt]) *var[i--] = 0;
		cnt += i + 1;
		for (; i >= 0; i--) *var[i] = TR(sh, 2 | (*var[i] & 1));
	}
	return cnt;
}

/* edge tsuqBlock, src/lib/bandcodec.cpp:215-237 */
static int tsuq_edge(int sh, int32_t* cur, int stride, int Q, int iQ, int width, int height)
{
	int cnt = 0;
	int T = TR(sh, (Q + ((Q - (Q >> 2)) >> 1)) >> 1);
	for (int j = 0; j < height; j++) {
		int32_t* r = cur + (long)j * stride;
		for (int i = 0; i < width; i++) {
			int v = r[i];
			if ((uint32_t)(v + T) <= (uint32_t)(2 * T)) { r[i] = 0; continue; }
			v = TR(sh, s2u_(v));
			cnt++;
			int tmp = (int)(UC(sh, v) >> 1);
			int q = (tmp * iQ + (1 << 15)) >> 16;
			r[i] = TR(sh, (q << 1) | (v & 1));
		}
	}
	return cnt;
}

/* CBandCodec::buildTree, src/lib/bandcodec.cpp:239-319, iterative over the
 * parent chain (finest -> coarsest) for one orientation b. */
static void build_tree(pyr_t* p, int b, int quant, int lambda)
{
	int qin = quant;
	for (int l = 0; l < p->nlev; l++) {
		band_t* B = &p->b[l][b];
		int sh = B->sh;
		qin = TR(sh, qin);                              /* Quant passed as C */
		int lbda = (int)((float)lambda / B->weight);
		int Q = TR(sh, (int16_t)(int)((float)qin / B->weight));
		if (Q == 0) Q = 1;
		int iQ = (1 << 16) / Q;
		int thres[16];
		make_thres(sh, thres, Q, lbda);
		int dx = B->dx, dy = B->dy, rs = (dx + 3) / 4;
		band_t* C = l ? &p->b[l - 1][b] : NULL;
		int crs = C ? (C->dx + 3) / 4 : 0;
		int by, bx;
		for (by = 0; by + 4 <= dy; by += 4) {
			int k;
			for (bx = 0, k = 0; bx + 4 <= dx; bx += 4, k++) {
				int32_t* cur = B->v + (long)by * dx + bx;
				long long dist = tsuq_block(sh, cur, dx, Q, iQ, thres);
				if (C) {
					uint32_t* c0 = C->rd + (long)(by / 4) * 2 * crs;
					uint32_t* c1 = c0 + crs;
					dist += (uint32_t)(c0[2 * k] + c0[2 * k + 1] + c1[2 * k] + c1[2 * k + 1]);
				}
				if (dist <= 0) { cur[0] = INSIGNIF; B->rd[(by / 4) * rs + k] = 0; }
				else B->rd[(by / 4) * rs + k] = dist > 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)dist;
			}
			if (bx < dx) {
				int32_t* cur = B->v + (long)by * dx + bx;
				int dist = tsuq_edge(sh, cur, dx, Q, iQ, dx - bx, 4);
				if (dist <= 0) { cur[0] = INSIGNIF; B->rd[(by / 4) * rs + k] = 0; }
				else B->rd[(by / 4) * rs + k] = dist;
			}
		}
		if (dy & 3) {
			int k;
			for (bx = 0, k = 0; bx + 4 <= dx; bx += 4, k++) {
				int32_t* cur = B->v + (long)by * dx + bx;
				int dist = tsuq_edge(sh, cur, dx, Q, iQ, 4, dy & 3);
				if (dist <= 0) { cur[0] = INSIGNIF; B->rd[(by / 4) * rs + k] = 0; }
				else B->rd[(by / 4) * rs + k] = dist;
			}
			if (bx < dx) {
				int32_t* cur = B->v + (long)by * dx + bx;
				int dist = tsuq_edge(sh, cur, dx, Q, iQ, dx - bx, dy & 3);
				if (dist <= 0) { cur[0] = INSIGNIF; B->rd[(by / 4) * rs + k] = 0; }
				else B->rd[(by / 4) * rs + k] = dist;
			}
		}
	}
}

/* CBand::TSUQ, src/lib/band.h:65-92 (used for the coarsest LL, Thres 0.5) */
static void tsuq_ll(band_t* B, int quant, float thres)
{
	int sh = B->sh;
	int Q = (int)((float)quant / B->weight);
	if (Q == 0) Q = 1;
	int iQ = (1 << 16) / Q;
	int T = TR(sh, (int)(thres * (float)Q));
	for (long n = 0; n < (long)B->dx * B->dy; n++) {
		int v = B->v[n];
		if ((uint32_t)(v + T) <= (uint32_t)(2 * T)) B->v[n] = 0;
		else B->v[n] = TR(sh, (v * iQ + (1 << 15)) >> 16);
	}
}

/* CBand::TSUQi, src/lib/band.h:94-107; CWavelet2D::TSUQi wavelet2d.cpp:248-268 */
static void tsuqi_band(band_t* B, int quant)
{
	int sh = B->sh;
	int q = TR(sh, quant);                     /* the int Quant is passed as C */
	q = TR(sh, (int)((float)q / B->weight));
	if (q == 0) q = 1;
	for (long n = 0; n < (long)B->dx * B->dy; n++) B->v[n] = TR(sh, B->v[n] * q);
}

static void pyr_tsuqi(pyr_t* p, int quant)
{
	for (int l = 0; l < p->nlev; l++) {
		tsuqi_band(&p->b[l][BD], quant);
		tsuqi_band(&p->b[l][BH], quant);
		tsuqi_band(&p->b[l][BV], quant);
	}
	tsuqi_band(coarsest_ll(p), quant);
}

/* ------------------------------------------------------- LL predictor */
/* CBandCodec::pred, src/lib/bandcodec.cpp:62-104 */
static void pred(band_t* B, mux_t* m, int decode)
{
	static const uint8_t ginit[16] = {9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,15};
	geom_t g; geom_init(&g, ginit);
	int sh = B->sh, dx = B->dx;
	int32_t* c = B->v;
	if (!decode) taboo_code(m, s2u(c[0])); else c[0] = TR(sh, u2s(taboo_decode(m)));
	for (int i = 1; i < dx; i++) {
		if (!decode) geom_code(&g, m, s2u(c[i] - c[i - 1]), 15);
		else c[i] = TR(sh, c[i - 1] + u2s(geom_decode(&g, m, 15)));
	}
	for (int j = 1; j < B->dy; j++) {
		c += dx;
		if (!decode) geom_code(&g, m, s2u(c[0] - c[-dx]), 15);
		else c[0] = TR(sh, c[-dx] + u2s(geom_decode(&g, m, 15)));
		for (int i = 1; i < dx; i++) {
			int var = bitlen(iabs(c[i - 1] - c[i - 1 - dx]) + iabs(c[i - dx] - c[i - 1 - dx]));
			if (!decode) geom_code(&g, m, s2u(c[i] - c[i - 1] - c[i - dx] + c[i - 1 - dx]), var);
			else c[i] = TR(sh, c[i - 1] + c[i - dx] - c[i - 1 - dx] + u2s(geom_decode(&g, m, var)));
		}
	}
}

/* --------------------------------------------------------- zerotree */
static const uint8_t K_CONV2[9][16] = {
	{15}, {7,15}, {4,10,15}, {3,7,11,15}, {2,4,7,10,12,15}, {1,3,5,7,9,11,13,15},
	{1,3,4,6,8,10,11,13,15}, {0,2,3,4,6,7,8,10,11,12,14,15},
	{0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15}};
static const uint8_t K_CONV1[16] = {0,1,2,3,0,4,0,5,6,0,0,7,0,0,0,8};

/* CBandCodec::block_enum (full 4x4), src/lib/bandcodec.cpp:346-403 */
static int block_full(int sh, int32_t* blk, int stride, mux_t* m, geom_t* g, int idx, int high, int decode)
{
	uint32_t k = 0;
	if (!decode) {
		int tmp[16];
		uint32_t sig = 0;
		for (int j = 0; j < 4; j++)
			for (int i = 0; i < 4; i++) {
				int v = blk[(long)j * stride + i];
				sig <<= 1;
				if (v != 0) { tmp[k++] = v; sig |= 1; }
			}
		uint16_t e = high ? HUF_HIGH[idx][k - 1] : HUF_LOW[idx][k];
		bits_code(m, e >> 5, e & 31);
		if (high || k != 0) {
			if (k != 16) enum_code(m, sig, k, 16);
			for (uint32_t i = 0; i < k; i++) {
				geom_code(g, m, (UC(sh, tmp[i]) >> 1) - 1, k - 1);
				bits_code(m, tmp[i] & 1, 1);
			}
		}
	} else {
		if (high) k = huff_decode(m, HUF_HIGH[idx], 16) + 1;
		else k = huff_decode(m, HUF_LOW[idx], 17);
		if (high || k != 0) {
			uint32_t sig = 0xFFFF;
			if (k != 16) sig = enum_decode(m, k, 16);
			for (int j = 0; j < 4; j++)
				for (int i = 0; i < 4; i++) {
					if (sig & (1u << 15)) {
						uint32_t u = ((geom_decode(g, m, k - 1) + 1) << 1) | bits_decode(m, 1);
						blk[(long)j * stride + i] = TR(sh, u2s_((int)u));
					}
					sig <<= 1;
				}
		}
	}
	return (int)k - (high != 0);
}

/* CBandCodec::block_enum (edge w x h), src/lib/bandcodec.cpp:405-478 */
static void block_edge(int sh, int32_t* blk, int stride, mux_t* m, geom_t* g, int w, int h, int high, int decode)
{
	uint32_t k = 0, cnt = w * h;
	if (!decode) {
		int tmp[16];
		uint32_t sig = 0;
		for (int j = 0; j < h; j++)
			for (int i = 0; i < w; i++) {
				int v = blk[(long)j * stride + i];
				sig <<= 1;
				if (v != 0) { tmp[k++] = v; sig |= 1; }
			}
		if (high) max_code(m, k - 1, cnt - 1); else max_code(m, k, cnt);
		if (high || k != 0) {
			if (k != cnt) enum_code(m, sig, k, cnt);
			for (uint32_t i = 0; i < k; i++) {
				geom_code(g, m, (UC(sh, tmp[i]) >> 1) - 1, K_CONV2[K_CONV1[cnt]][k - 1]);
				bits_code(m, tmp[i] & 1, 1);
			}
		}
	} else {
		if (high) k = max_decode(m, cnt - 1) + 1; else k = max_decode(m, cnt);
		if (k > cnt) k = cnt;                    /* desync guard only */
		if (high || k != 0) {
			uint32_t sig = 0xFFFF;
			if (k != cnt) sig = enum_decode(m, k, cnt);
			for (int j = 0; j < h; j++)
				for (int i = 0; i < w; i++) {
					if (sig & (1u << (cnt - 1))) {
						uint32_t u = ((geom_decode(g, m, K_CONV2[K_CONV1[cnt]][k - 1]) + 1) << 1) | bits_decode(m, 1);
						blk[(long)j * stride + i] = TR(sh, u2s_((int)u));
					}
					sig <<= 1;
				}
		}
	}
}

/* CBandCodec::maxLen<2,mode>, src/lib/bandcodec.cpp:324-344 */
static int max_len2(int psh, const int32_t* p, int stride, int decode)
{
	int mx = 0, mn = 0;
	for (int j = 0; j < 2; j++)
		for (int i = 0; i < 2; i++) {
			int v = p[(long)j * stride + i];
			if (v > mx) mx = v;
			if (decode && v < mn) mn = v;
		}
	if (!decode) return bitlen(UC(psh, mx) >> 1);
	mn = TR(psh, iabs(mn));
	if (mn > mx) mx = mn;
	return bitlen((uint32_t)mx);
}

/* CBandCodec::tree, src/lib/bandcodec.cpp:484-589 */
static void tree(pyr_t* p, int l, int b, mux_t* m, int high, int decode)
{
	static const uint8_t ginit[16] = {5,9,9,9,9,9,9,9,9,9,9,9,10,10,10,11};
	uint16_t kmean[16] = {2<<10, 3<<10, 4<<10, 5<<10, 8<<10, 11<<10, 13<<10, 14<<10,
	                      15<<10, 15<<10, 15<<10, 15<<10, 15<<10, 15<<10, 15<<10, 15<<10};
	band_t* B = &p->b[l][b];
	band_t* P = l + 1 < p->nlev ? &p->b[l + 1][b] : NULL;
	int has_child = l > 0;
	int sh = B->sh, dx = B->dx, dy = B->dy;
	int psh = P ? P->sh : 0, pdx = P ? P->dx : 0;
	int mark = has_child ? INSIGNIF : 0;
	if (decode) memset(B->v, 0, sizeof(int32_t) * (size_t)dx * dy);
	geom_t g; geom_init(&g, ginit);
	bitm_t tr, bo; bitm_init(&tr); bitm_init(&bo);

	int j;
	for (j = 0; j + 4 <= dy; j += 4) {
		int32_t* c1 = B->v + (long)j * dx;
		int32_t* c2 = c1 + 2 * dx;
		int32_t* pp = P ? P->v + (long)(j >> 1) * pdx : NULL;
		int i = 0, bs = 4;
		if (j & 4) {
			bs = -4;
			i = dx & ~3;
			if (dx > i) {
				if (pp && (i >> 1) < pdx && pp[i >> 1] == INSIGNIF) pp[i >> 1] = 0;
				int ins = decode ? bitm_decode(&bo, m, 0) : bitm_code(&bo, m, c1[i] == INSIGNIF, 0);
				if (ins) { if (!decode) c1[i] = 0; }
				else block_edge(sh, c1 + i, dx, m, &g, dx - i, 4, high, decode);
			}
			i += bs;
		}
		for (; i >= 0 && i + 4 <= dx; i += bs) {
			int ctx = 15, k = i >> 1;
			if (pp) ctx = pp[k];
			if (ctx == INSIGNIF) {
				pp[k] = 0;
				c1[i] = c1[i + 2] = c2[i] = c2[i + 2] = TR(sh, mark);
				continue;
			}
			if (pp) ctx = max_len2(psh, pp + k, pdx, decode);
			int ins = decode ? bitm_decode(&tr, m, ctx) : bitm_code(&tr, m, c1[i] == INSIGNIF, ctx);
			if (ins) {
				c1[i] = c1[i + 2] = c2[i] = c2[i + 2] = TR(sh, mark);
			} else {
				int idx = (kmean[ctx] + (1 << 9)) >> 10;
				int kk = block_full(sh, c1 + i, dx, m, &g, idx, high, decode);
				kmean[ctx] = (uint16_t)(kmean[ctx] + ((unsigned)kk << 7) - (kmean[ctx] >> 3));
			}
		}
		if (i > 0 && i < dx) {
			if (pp && (i >> 1) < pdx && pp[i >> 1] == INSIGNIF) pp[i >> 1] = 0;
			int ins = decode ? bitm_decode(&bo, m, 0) : bitm_code(&bo, m, c1[i] == INSIGNIF, 0);
			if (ins) { if (!decode) c1[i] = 0; }
			else block_edge(sh, c1 + i, dx, m, &g, dx - i, 4, high, decode);
		}
	}
	if (j < dy) {
		int32_t* c1 = B->v + (long)j * dx;
		int32_t* pp = P ? P->v + (long)(j >> 1) * pdx : NULL;
		int pdy = P ? P->dy : 0;
		int i = 0, bs = 4;
		if (j & 4) {
			bs = -4;
			i = dx & ~3;
			if (dx > i) {
				if (pp && (i >> 1) < pdx && (j >> 1) < pdy && pp[i >> 1] == INSIGNIF) pp[i >> 1] = 0;
				int ins = decode ? bitm_decode(&bo, m, 0) : bitm_code(&bo, m, c1[i] == INSIGNIF, 0);
				if (ins) { if (!decode) c1[i] = 0; }
				else block_edge(sh, c1 + i, dx, m, &g, dx - i, dy - j, high, decode);
			}
			i += bs;
		}
		for (; i >= 0 && i + 4 <= dx; i += bs) {
			if (pp && (j >> 1) < pdy && pp[i >> 1] == INSIGNIF) pp[i >> 1] = 0;
			int ins = decode ? bitm_decode(&bo, m, 0) : bitm_code(&bo, m, c1[i] == INSIGNIF, 0);
			if (ins) { if (!decode) c1[i] = 0; }
			else block_edge(sh, c1 + i, dx, m, &g, 4, dy - j, high, decode);
		}
		if (i > 0 && i < dx) {
			if (pp && (i >> 1) < pdx && (j >> 1) < pdy && pp[i >> 1] == INSIGNIF) pp[i >> 1] = 0;
			int ins = decode ? bitm_decode(&bo, m, 0) : bitm_code(&bo, m, c1[i] == INSIGNIF, 0);
			if (ins) { if (!decode) c1[i] = 0; }
			else block_edge(sh, c1 + i, dx, m, &g, dx - i, dy - j, high, decode);
		}
	}
}

/* CWavelet2D::CodeBand / DecodeBand, src/lib/wavelet2d.cpp:83-222 */
static void code_bands(pyr_t* p, mux_t* m, int quant, int lambda)
{
	build_tree(p, BD, quant, lambda);
	build_tree(p, BH, quant, lambda);
	build_tree(p, BV, quant, lambda);
	band_t* L = coarsest_ll(p);
	tsuq_ll(L, quant, 0.5f);
	pred(L, m, 0);
	for (int l = p->nlev - 1; l >= 0; l--) {
		tree(p, l, BV, m, l == 0, 0);
		tree(p, l, BH, m, l == 0, 0);
		tree(p, l, BD, m, l == 0, 0);
	}
}

static void decode_bands(pyr_t* p, mux_t* m)
{
	pred(coarsest_ll(p), m, 1);
	for (int l = p->nlev - 1; l >= 0; l--) {
		tree(p, l, BV, m, l == 0, 1);
		tree(p, l, BH, m, l == 0, 1);
		tree(p, l, BD, m, l == 0, 1);
	}
}

static long dump(pyr_t* p, int32_t* out)
{
	int32_t* o = out;
	for (int l = 0; l < p->nlev; l++) {
		const int order[3] = {BD, BH, BV};
		for (int k = 0; k < 3; k++) {
			band_t* B = &p->b[l][order[k]];
			memcpy(o, B->v, sizeof(int32_t) * (size_t)B->dx * B->dy);
			o += (long)B->dx * B->dy;
		}
	}
	band_t* L = coarsest_ll(p);
	memcpy(o, L->v, sizeof(int32_t) * (size_t)L->dx * L->dy);
	o += (long)L->dx * L->dy;
	return (long)(o - out);
}

static void load(pyr_t* p, const int32_t* in)
{
	for (int l = 0; l < p->nlev; l++) {
		const int order[3] = {BD, BH, BV};
		for (int k = 0; k < 3; k++) {
			band_t* B = &p->b[l][order[k]];
			memcpy(B->v, in, sizeof(int32_t) * (size_t)B->dx * B->dy);
			in += (long)B->dx * B->dy;
		}
	}
	band_t* L = coarsest_ll(p);
	memcpy(L->v, in, sizeof(int32_t) * (size_t)L->dx * L->dy);
}

/* ------------------------------------------------------------ public API */
static int g_init = 0;
static void once(void) { if (!g_init) { cnk_init(); g_init = 1; } }

int ricor_layout(int w, int h, int levels, int lc, int32_t* out)
{
	pyr_t p; pyr_init(&p, w, h, levels, lc);
	int n = 0;
	for (int l = 0; l < p.nlev; l++) {
		const int order[3] = {BD, BH, BV};
		for (int k = 0; k < 3; k++, n++)
			if (out) { band_t* B = &p.b[l][order[k]]; out[3*n] = B->dx; out[3*n+1] = B->dy; out[3*n+2] = !B->sh; }
	}
	band_t* L = coarsest_ll(&p);
	if (out) { out[3*n] = L->dx; out[3*n+1] = L->dy; out[3*n+2] = !L->sh; }
	n++;
	pyr_free(&p);
	return n;
}

long ricor_bands(const int16_t* img, int w, int h, int levels, int lc, int trans,
                 int stage, int quant, int lambda, int32_t* out)
{
	once();
	pyr_t p; pyr_init(&p, w, h, levels, lc); pyr_weights(&p, trans);
	int32_t* x = malloc(sizeof(int32_t) * (size_t)w * h);
	for (long i = 0; i < (long)w * h; i++) x[i] = img[i];
	pyr_forward(&p, x, trans);
	free(x);
	if (stage == 1) {
		build_tree(&p, BD, quant, lambda); build_tree(&p, BH, quant, lambda); build_tree(&p, BV, quant, lambda);
		tsuq_ll(coarsest_ll(&p), quant, 0.5f);
	} else if (stage == 2) {
		uint8_t* s = calloc((size_t)w * h * 4 + 4096, 1);
		mux_t m; mux_enc_init(&m, s);
		code_bands(&p, &m, quant, lambda);
		free(s);
	}
	long n = dump(&p, out);
	pyr_free(&p);
	return n;
}

long ricor_encode_planes(const int16_t* planes, int nplanes, int w, int h, int levels,
                         int lc, int trans, const int* quant, const int* lambda,
                         uint8_t* out, long cap)
{
	once();
	size_t n = (size_t)w * h;
	uint8_t* s = calloc(n * nplanes * 4 + 4096, 1);
	mux_t m; mux_enc_init(&m, s);
	pyr_t p; pyr_init(&p, w, h, levels, lc); pyr_weights(&p, trans);
	int32_t* x = malloc(sizeof(int32_t) * n);
	for (int k = 0; k < nplanes; k++) {
		for (size_t i = 0; i < n; i++) x[i] = planes[k * n + i];
		pyr_forward(&p, x, trans);
		code_bands(&p, &m, quant[k], lambda[k]);
	}
	uint8_t* end = mux_end(&m);
	long len = (long)(end - s);
	free(x); pyr_free(&p);
	if (len > cap) { free(s); return -len; }
	memcpy(out, s, len);
	free(s);
	return len;
}

long ricor_decode_planes(const uint8_t* in, long len, int nplanes, int w, int h, int levels,
                         int lc, int trans, const int* quant, int16_t* planes_out,
                         int32_t* bands_out)
{
	once();
	size_t n = (size_t)w * h;
	size_t slen = (size_t)(len > 0 ? len : 0) + n * nplanes + 4096;
	uint8_t* s = calloc(slen, 1);
	memcpy(s, in, len);
	mux_t m; mux_dec_init(&m, s);
	m.end = s + slen - 8;
	pyr_t p; pyr_init(&p, w, h, levels, lc); pyr_weights(&p, trans);
	int32_t* x = malloc(sizeof(int32_t) * n);
	for (int k = 0; k < nplanes; k++) {
		decode_bands(&p, &m);
		if (bands_out && k == nplanes - 1) dump(&p, bands_out);
		if (quant[k] != 0) pyr_tsuqi(&p, quant[k]);
		pyr_inverse(&p, trans, x);
		for (size_t i = 0; i < n; i++) planes_out[k * n + i] = (int16_t)x[i];
	}
	free(x); pyr_free(&p); free(s);
	return 0;
}

long ricor_inverse(const int32_t* bands, int w, int h, int levels, int lc, int trans,
                   int16_t* plane_out)
{
	pyr_t p; pyr_init(&p, w, h, levels, lc);
	load(&p, bands);
	int32_t* x = malloc(sizeof(int32_t) * (size_t)w * h);
	pyr_inverse(&p, trans, x);
	for (long i = 0; i < (long)w * h; i++) plane_out[i] = (int16_t)x[i];
	free(x); pyr_free(&p);
	return 0;
}

/* The video driver's closed loop on one plane (src/lib/rududucodec.cpp:67-74):
 * Transform, CodeBand (the bands keep the scan's final sign-magnitude state),
 * TSUQi on that state, TransformI.  Dumps the bands after TSUQi (bands_out,
 * optional) and the reconstructed plane. */
long ricor_closed_loop(const int16_t* img, int w, int h, int levels, int lc, int trans, int quant, int lambda,
                       int dq, int16_t* plane_out, int32_t* bands_out)
{
	once();
	pyr_t p; pyr_init(&p, w, h, levels, lc); pyr_weights(&p, trans);
	int32_t* x = malloc(sizeof(int32_t) * (size_t)w * h);
	for (long i = 0; i < (long)w * h; i++) x[i] = img[i];
	pyr_forward(&p, x, trans);
	uint8_t* s = calloc((size_t)w * h * 4 + 4096, 1);
	mux_t m; mux_enc_init(&m, s);
	code_bands(&p, &m, quant, lambda);
	free(s);
	pyr_tsuqi(&p, dq);
	long n = bands_out ? dump(&p, bands_out) : 0;
	pyr_inverse(&p, trans, x);
	for (long i = 0; i < (long)w * h; i++) plane_out[i] = (int16_t)x[i];
	free(x); pyr_free(&p);
	return n;
}

/* src/ric/ric.cpp:42-49 */
short ricor_quants(int idx)
{
	static const unsigned short Q[5] = {0x8000, 0x9000, 0xA800, 0xC000, 0xE000};
	if (idx <= 0) return 0;
	idx--;
	int r = 14 - idx / 5;
	return (short)((Q[idx % 5] + (1 << (r - 1))) >> r);
}

/* CompressImage, src/ric/ric.cpp:123-180 */
long ricor_encode_ric(const uint8_t* pix, int w, int h, int channels, int q, int trans,
                      uint8_t* out, long cap)
{
	size_t n = (size_t)w * h;
	int color = channels == 3;
	int16_t* img = malloc(sizeof(int16_t) * n * channels);
	for (size_t i = 0; i < n * channels; i++) img[i] = pix[i];
	int16_t* planes = malloc(sizeof(int16_t) * n * channels);
	int qs[3], ls[3];
	if (color) {
		for (size_t i = 0; i < n; i++) {           /* RGBtoYCoCg, src/ric/ric.cpp:76-91 */
			int16_t R = img[i], G = img[n + i], B = img[2 * n + i];
			R -= B; B += R >> 1; G -= B; B += (G >> 1) - 128;
			if (q) { R = (int16_t)(R << 3); G = (int16_t)(G << 3); B = (int16_t)(B << 4); }
			planes[i] = B; planes[n + i] = G; planes[2 * n + i] = R;   /* Y, Cg, Co */
		}
		for (int k = 0; k < 3; k++) {
			int boost = k ? 8 : 0;
			qs[k] = q ? ricor_quants(q + 20 + boost) : 0;
			ls[k] = q ? ricor_quants(q + 13 + boost) : 0;
		}
	} else {
		for (size_t i = 0; i < n; i++) planes[i] = q ? (int16_t)((img[i] - 128) << 4) : (int16_t)(img[i] - 128);
		qs[0] = q ? ricor_quants(q + 20) : 0;
		ls[0] = q ? ricor_quants(q + 13) : 0;
	}
	long scap = (long)(n * channels * 4 + 4096);
	uint8_t* s = malloc(scap);
	long len = ricor_encode_planes(planes, channels, w, h, 5, 1, trans, qs, ls, s, scap);
	free(img); free(planes);
	long total = 9 + len - 2;
	if (total > cap) { free(s); return -total; }
	memcpy(out, "RUD2", 4);
	out[4] = w & 255; out[5] = w >> 8; out[6] = h & 255; out[7] = h >> 8;
	out[8] = (uint8_t)((q & 31) | (color << 5) | ((trans & 3) << 6));
	memcpy(out + 9, s + 2, len - 2);
	free(s);
	return total;
}

static int16_t clip255(int v) { return (int16_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

/* DecompressImage, src/ric/ric.cpp:182-251 (+ dither :51-74, YCoCgtoRGB :93-112) */
long ricor_decode_ric(const uint8_t* ric, long len, int dither_on, int16_t* planes_out,
                      uint8_t* pix_out, int32_t* dims)
{
	if (len < 9 || memcmp(ric, "RUD2", 4) != 0) return -2;
	int w = ric[4] | (ric[5] << 8), h = ric[6] | (ric[7] << 8);
	int q = ric[8] & 31, color = (ric[8] >> 5) & 1, trans = (ric[8] >> 6) & 3;
	int channels = color ? 3 : 1;
	if (dims) { dims[0] = w; dims[1] = h; dims[2] = channels; dims[3] = q; dims[4] = trans; }
	if (!pix_out && !planes_out) return 0;
	size_t n = (size_t)w * h;
	long slen = (long)(n * channels + 4096);
	uint8_t* s = calloc(slen, 1);
	long pay = len - 9 < (long)(n * channels) ? len - 9 : (long)(n * channels);
	memcpy(s + 2, ric + 9, pay);
	int qs[3];
	qs[0] = q ? ricor_quants(q + 20) : 0;
	qs[1] = qs[2] = q ? ricor_quants(q + 28) : 0;
	int16_t* dec = malloc(sizeof(int16_t) * n * channels);
	ricor_decode_planes(s, slen, channels, w, h, 5, 1, trans, qs, dec, NULL);
	free(s);
	int16_t* img = malloc(sizeof(int16_t) * n * channels);
	if (color) for (int k = 0; k < 3; k++) memcpy(img + (2 - k) * n, dec + k * n, sizeof(int16_t) * n);
	else memcpy(img, dec, sizeof(int16_t) * n);
	free(dec);
	if (!color) {
		if (q == 0) {
			for (size_t i = 0; i < n; i++) img[i] += 128;
		} else if (dither_on) {
			int16_t* pi = img;
			for (int j = 0; j < h - 1; j++) {
				pi[0] = clip255(128 + ((pi[0] + 8) >> 4));
				for (int i = 1; i < w - 1; i++) {
					int16_t tmp = pi[i] + 8;
					pi[i] = tmp >> 4;
					tmp -= pi[i] << 4;
					pi[i + 1] += (tmp >> 1) - (tmp >> 4);
					pi[i + w - 1] += (tmp >> 3) + (tmp >> 4);
					pi[i + w] += (tmp >> 2) + (tmp >> 4);
					pi[i + w + 1] += tmp >> 4;
					pi[i] = clip255(pi[i] + 128);
				}
				pi += w;
				pi[-1] = clip255(128 + ((pi[-1] + 8) >> 4));
			}
			for (int i = 0; i < w; i++) pi[i] = clip255(128 + ((pi[i] + 8) >> 4));
		} else {
			for (size_t i = 0; i < n; i++) img[i] = clip255((int16_t)(128 + ((img[i] + 8) >> 4)));
		}
	} else {
		for (size_t i = 0; i < n; i++) {
			int16_t R = img[i], G = img[n + i], B = img[2 * n + i];
			if (q) { R = (R + 4) >> 3; G = (G + 4) >> 3; B = (B + 8) >> 4; }
			B -= (G >> 1) - 128; G += B; B -= R >> 1; R += B;
			if (q) { R = clip255(R); G = clip255(G); B = clip255(B); }
			img[i] = R; img[n + i] = G; img[2 * n + i] = B;
		}
	}
	if (planes_out) memcpy(planes_out, img, sizeof(int16_t) * n * channels);
	if (pix_out) for (size_t i = 0; i < n * channels; i++) pix_out[i] = (uint8_t)clip255(img[i]);
	free(img);
	return 0;
}

/* SURVEY.md §8(d) synthetic generator (integer-only, bit-reproducible) */
void ricor_synth(int w, int h, int channels, int frame, uint8_t* out)
{
	for (int c = 0; c < channels; c++) {
		uint32_t s = 0x9E3779B9u + 0x1000u * (uint32_t)frame + (uint32_t)c;
		int phase = 32 * c;
		for (int y = 0; y < h; y++)
			for (int x = 0; x < w; x++) {
				s ^= s << 13; s ^= s >> 17; s ^= s << 5;
				int noise = (int)(s >> 28) - 8;
				int grad = ((x * 255) / (w - 1) + (y * 255) / (h - 1)) >> 2;
				int t = (x + 2 * y + phase) & 127;
				t = t < 64 ? t : 127 - t;
				int v = grad + t + noise + 32;
				out[(size_t)c * w * h + (size_t)y * w + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
			}
	}
}
