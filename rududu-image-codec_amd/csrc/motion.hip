// motion.hip -- the video codec's data-parallel stages on CDNA4 (see motion.h):
// pixel input, frame add/subtract, the quarter-pel interpolation and border
// extension of CImageBuffer::calc_sub, the EPZS motion search and OBMC.
// All arithmetic is the reference's: int expressions stored to `short`.
#include <hip/hip_runtime.h>
#include "motion.h"

namespace ric {

namespace {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ int mvx(uint32_t v) { return (int16_t)(v & 0xFFFF); }
__device__ __forceinline__ int mvy(uint32_t v) { return (int16_t)(v >> 16); }
__device__ __forceinline__ uint32_t mvmake(int x, int y) { return (uint32_t)(uint16_t)x | ((uint32_t)(uint16_t)y << 16); }

// ----------------------------------------------------------- pixels
// CImage::inputSGI<unsigned char>(pIn, stride, -128), image.cpp:96-123
__global__ void k_vid_input(const uint8_t* __restrict__ rgb, int stride, int16_t* __restrict__ img, int w, int h,
                            int S, long P)
{
	const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
	if (x >= w) return;
	const long ps = (long)stride * h, src = (long)(h - 1 - y) * stride + x;   // bottom row first
	const int R = rgb[src], G = rgb[ps + src], B = rgb[2 * ps + src];
	const int16_t Co = (int16_t)(R - B);
	int16_t Y = (int16_t)(B + (Co >> 1));
	const int16_t Cg = (int16_t)(G - Y);
	Y = (int16_t)(Y + ((Cg >> 1) - 128));
	const long o = (long)y * S + x;
	img[o] = (int16_t)(Y * 16);
	img[P + o] = (int16_t)(Co * 8);
	img[2 * P + o] = (int16_t)(Cg * 8);
}

// CImage::operator-= / += (image.cpp:216-246)
__global__ void k_vid_addsub(int16_t* __restrict__ img, const int16_t* __restrict__ pred, int w, int S, long P, int sign)
{
	const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
	if (x >= w) return;
	const long o = blockIdx.z * P + (long)y * S + x;
	img[o] = (int16_t)(sign > 0 ? img[o] + pred[o] : img[o] - pred[o]);
}

// ------------------------------------------------ quarter-pel planes
// the three interpolators of interH / interV (image.cpp:288-298, 320-330):
// taps at -1, 0, +1, +2
template <int pos>
__device__ __forceinline__ int interp(int m, int a, int b, int c)
{
	if (pos == 1) return (53 * a + 18 * b - 4 * m - 3 * c + 32) >> 6;
	if (pos == 2) return ((a + b) * 9 - m - c + 8) >> 4;
	return (18 * a + 53 * b - 3 * m - 4 * c + 32) >> 6;
}

// calc_sub's interpolation (imagebuffer.cpp:92-116), one thread per sample of
// one plane: sub[4p] = interH<p>(sub[0]) and sub[i + q] = interV<q>(sub[i]),
// i = 0, 4, 8, 12.  interH reads sub[0] one column past each edge and interV
// reads its input one row above and two below, before extend() rewrites the
// borders: those samples are whatever the buffers hold (for sub[4p], its own
// border, not an interpolated value), as in the reference.
__global__ void k_vid_interp(VidSubs s, int w, int h, int S, long P)
{
	const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
	if (x >= w) return;
	const long pc = blockIdx.z * P;
	const int16_t* s0 = s.p[0] + pc;
	int a[4][4];
#pragma unroll
	for (int r = 0; r < 4; r++)
#pragma unroll
		for (int k = 0; k < 4; k++) a[r][k] = s0[(long)(y - 1 + r) * S + x - 1 + k];
	int hv[3][4];
#pragma unroll
	for (int r = 0; r < 4; r++) {
		const int yy = y - 1 + r;
		if (yy >= 0 && yy < h) {
			hv[0][r] = (int16_t)interp<1>(a[r][0], a[r][1], a[r][2], a[r][3]);
			hv[1][r] = (int16_t)interp<2>(a[r][0], a[r][1], a[r][2], a[r][3]);
			hv[2][r] = (int16_t)interp<3>(a[r][0], a[r][1], a[r][2], a[r][3]);
		} else {
			const long o = pc + (long)yy * S + x;
			hv[0][r] = s.p[4][o];
			hv[1][r] = s.p[8][o];
			hv[2][r] = s.p[12][o];
		}
	}
	const long o = pc + (long)y * S + x;
	s.p[4][o] = (int16_t)hv[0][1];
	s.p[8][o] = (int16_t)hv[1][1];
	s.p[12][o] = (int16_t)hv[2][1];
#pragma unroll
	for (int i = 0; i < 4; i++) {
		int c0, c1, c2, c3;
		if (i == 0) { c0 = a[0][1]; c1 = a[1][1]; c2 = a[2][1]; c3 = a[3][1]; }
		else { c0 = hv[i - 1][0]; c1 = hv[i - 1][1]; c2 = hv[i - 1][2]; c3 = hv[i - 1][3]; }
		s.p[4 * i + 1][o] = (int16_t)interp<1>(c0, c1, c2, c3);
		s.p[4 * i + 2][o] = (int16_t)interp<2>(c0, c1, c2, c3);
		s.p[4 * i + 3][o] = (int16_t)interp<3>(c0, c1, c2, c3);
	}
}

// CImage::extend (image.cpp:190-214): the 15-sample border replicates the
// nearest edge sample (corners: the corner sample).  One thread per border
// sample of the area any stage reads (rows and columns -15 .. +14 past the
// edges); blockIdx.y = plane, blockIdx.z = image.
__global__ void k_vid_extend(VidSubs s, int w, int h, int S, long P)
{
	constexpr int B = kVidBorder;
	const int t = blockIdx.x * blockDim.x + threadIdx.x;
	const int wb = w + 2 * B, tb = 2 * B * wb;
	if (t >= tb + 2 * B * h) return;
	int x, y;
	if (t < tb) {
		const int r = t / wb;
		x = t - r * wb - B;
		y = r < B ? r - B : h + r - B;
	} else {
		const int u = t - tb;
		y = u / (2 * B);
		const int k = u - y * 2 * B;
		x = k < B ? k - B : w + k - B;
	}
	int16_t* p = s.p[blockIdx.z] + blockIdx.y * P;
	p[(long)y * S + x] = p[(long)clampi(y, 0, h - 1) * S + clampi(x, 0, w - 1)];
}

// ------------------------------------------------------- motion search
struct EpzsArgs {
	const int16_t* cur;          // current frame, plane 0
	VidSubs ref;                 // reference frame's quarter-pel planes (plane 0 used)
	uint32_t* mv;
	uint16_t* dist;
	uint64_t* gran;              // per block {vector, epoch} hand-off granules
	uint32_t* status;
	uint32_t epoch;
	int w, h, S, bx, by;
};

// sum over the 64 lanes, returned to every lane (uniform): DPP adds within
// each 16-lane row, then row_bcast15 / row_bcast31 carry the row sums into
// lane 63, read back with readlane -- no LDS round trips
__device__ __forceinline__ int wave_sum(int v)
{
	v += __builtin_amdgcn_update_dpp(0, v, 0xb1, 0xf, 0xf, false);    // quad_perm [1,0,3,2]
	v += __builtin_amdgcn_update_dpp(0, v, 0x4e, 0xf, 0xf, false);    // quad_perm [2,3,0,1]
	v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, false);   // row_half_mirror
	v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xf, 0xf, false);   // row_mirror
	v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast15 into rows 1, 3
	v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast31 into rows 2, 3
	return __builtin_amdgcn_readlane(v, 63);
}

// one lane's sample of the 8x8 block at (px, py) after CHECK_MV's clamp
// (obme.cpp:59-68: x, y into [-7, im - 1])
__device__ __forceinline__ int ref_px(const int16_t* ref, const EpzsArgs& a, int px, int py, int lane)
{
	px = clampi(px, -7, a.w - 1);
	py = clampi(py, -7, a.h - 1);
	return ref[(long)(py + (lane >> 3)) * a.S + px + (lane & 7)];
}

// COBME::SAD<8> (obme.cpp:44-57), the sum clipped to 65535
__device__ __forceinline__ int sad_of(int diff) { return min(wave_sum(diff), 65535); }

constexpr int kUp = 1, kDown = 2, kLeft = 4, kRight = 8;   // utils.h:30-35

// the row above's granule k of this search (an sc1 load: it bypasses the
// CU's L1, and the 8 bytes arrive whole), polled until its tag is this
// search's; false once the wait gives up (~2 s) or another row has
__device__ __forceinline__ bool await_granule(const EpzsArgs& a, const uint64_t* g, uint32_t* out, int lane)
{
	for (long spins = 0;; spins++) {
		const uint64_t v = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if ((uint32_t)(v >> 32) == a.epoch) {
			*out = (uint32_t)v;
			return true;
		}
		__builtin_amdgcn_s_sleep(1);
		if ((spins & 255) == 255 &&
		    (spins > (1l << 24) || __hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
			if (lane == 0) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			return false;
		}
	}
}

// COBME::EPZS(CImageBuffer&) first loop (obme.cpp:185-222): one wave per block
// row, blocks left to right; block (i, j) needs row j - 1's vectors i and
// i + 1 (its above and above-right predictors).  Each block's vector is handed
// to the row below as one data-tagged granule {vector, epoch}: an 8-byte sc1
// store the reader polls with sc1 loads (MI355X_MICROARCH.md, handoff-1to1) --
// no release / acquire fences, which would write back and invalidate caches
// per block.  A wait that gives up raises *status and ends the wave (every
// wave reaches an exit).  The previous frame's vector of the block is read
// before this frame's overwrites it.
__global__ __launch_bounds__(64) void k_vid_epzs_full(EpzsArgs a)
{
	const int j = blockIdx.x, lane = threadIdx.x;
	const int16_t* ref = a.ref.p[0];
	uint32_t* row = a.mv + (long)j * a.bx;
	const uint64_t* gabove = a.gran + (long)(j - 1) * a.bx;
	uint64_t* grow = a.gran + (long)j * a.bx;
	uint32_t left = 0, u = 0, ur = 0;
	if (j > 0 && !await_granule(a, gabove, &ur, lane)) return;
	for (int i = 0; i < a.bx; i++) {
		if (j > 0) {
			u = ur;                                         // above[i], received last block
			if (i + 1 < a.bx && !await_granule(a, gabove + i + 1, &ur, lane)) return;
		}
		const int cx = 8 * i, cy = 8 * j;
		const int cur = a.cur[(long)(cy + (lane >> 3)) * a.S + cx + (lane & 7)];
		// predictors (obme.cpp:187-212): [0] the spatial one, the three
		// neighbours inside the frame, the previous frame's vector (full pel),
		// the zero vector
		uint32_t cand[6];
		int n = 1;
		cand[0] = 0;
		if (j == 0) {
			if (i != 0) cand[0] = left;
		} else if (i == 0 || i == a.bx - 1) {
			cand[0] = u;
		} else {
			int mx0 = mvx(left), mx1 = mvx(u), mx2 = mvx(ur), my0 = mvy(left), my1 = mvy(u), my2 = mvy(ur);
			// median (utils.h:64-77)
			auto med = [](int p, int q, int r) {
				if (q < p) { int t = p; p = q; q = t; }
				return r <= p ? p : (r <= q ? r : q);
			};
			cand[0] = mvmake(med(mx0, mx1, mx2), med(my0, my1, my2));
			cand[n++] = left;
			cand[n++] = u;
			cand[n++] = ur;
		}
		const uint32_t prev = row[i];
		cand[n++] = mvmake((mvx(prev) + 2) >> 2, (mvy(prev) + 2) >> 2);
		cand[n++] = 0;
		for (int k = n; k < 6; k++) cand[k] = 0;
		if (cand[0] == kVidIntra) cand[0] = 0;
		// every predictor's SAD at once (which ones count is decided below)
		int px[6];
#pragma unroll
		for (int k = 0; k < 6; k++) px[k] = ref_px(ref, a, cx + mvx(cand[k]), cy + mvy(cand[k]), lane);
		int sd[6];
#pragma unroll
		for (int k = 0; k < 6; k++) sd[k] = sad_of(abs(cur - px[k]));
		uint32_t best = cand[0];
		int bd = sd[0];
		if (bd >= 1024) {                                   // THRES_A (obme.cpp:148)
			for (int k = 1; k < n; k++)                     // sets B and C (:151-161)
				if (cand[k] != kVidIntra && bd > sd[k]) { best = cand[k]; bd = sd[k]; }
			// DiamondSearch (obme.cpp:79-108): the four neighbours of the
			// centre, never straight back along the last two moves; one step
			// per round of 4 loads.  (Loading the 12 positions within two
			// moves to take two steps per round halves the rounds but was
			// slower: 2.58 against 1.97 ms per 1080p frame)
			const int dx[4] = {0, 0, -1, 1}, dy[4] = {-1, 1, 0, 0};
			const int tst[4] = {kDown, kUp, kRight, kLeft}, stp[4] = {kUp, kDown, kLeft, kRight};
			int last = 0, last2 = 0;
			for (int it = 0; it < 65536; it++) {
				const int bxv = mvx(best), byv = mvy(best);
				int d4[4];
#pragma unroll
				for (int k = 0; k < 4; k++)
					d4[k] = sad_of(abs(cur - ref_px(ref, a, cx + (int16_t)(bxv + dx[k]), cy + (int16_t)(byv + dy[k]), lane)));
				int move = 0;
#pragma unroll
				for (int k = 0; k < 4; k++)
					if (!(last2 & tst[k]) && bd > d4[k]) {
						best = mvmake(bxv + dx[k], byv + dy[k]);
						bd = d4[k];
						move = stp[k];
					}
				last2 = move | last;
				last = move;
				if (!last) break;
			}
		}
		if (lane == 0) {
			__hip_atomic_store(grow + i, ((uint64_t)a.epoch << 32) | best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			row[i] = best;
			a.dist[(long)j * a.bx + i] = (uint16_t)bd;
		}
		left = best;
	}
}

// COBME::EPZS second loop (obme.cpp:224-243): every block independently --
// quarter-pel refinement subpxl<1> then subpxl<0> (obme.cpp:110-132) around
// the full-pel vector, or MV_INTRA when the full-pel SAD saturated
__global__ __launch_bounds__(64) void k_vid_epzs_sub(EpzsArgs a)
{
	// XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs,
	// so workgroup g takes block (g % 8) * C + g / 8 -- each XCD refines one
	// contiguous run of blocks, whose candidate windows overlap in its L2
	const int nb = a.bx * a.by, C = (nb + 7) >> 3;
	const int b = (int)(blockIdx.x & 7) * C + (int)(blockIdx.x >> 3), lane = threadIdx.x;
	if (b >= nb) return;
	const int i = b % a.bx, j = b / a.bx;
	const uint32_t m = a.mv[b];
	int bd = a.dist[b];
	if (bd >= 65535) {                                       // THRES_D
		if (lane == 0) a.mv[b] = kVidIntra;
		return;
	}
	const int cx = 8 * i, cy = 8 * j;
	const int cur = a.cur[(long)(cy + (lane >> 3)) * a.S + cx + (lane & 7)];
	int bx4 = (int16_t)(mvx(m) * 4), by4 = (int16_t)(mvy(m) * 4);
	// the 8 neighbours in subpxl's order (cumulative x_mov / y_mov)
	const int ox[8] = {1, 1, 0, -1, -1, -1, 0, 1}, oy[8] = {0, -1, -1, -1, 0, 1, 1, 1};
#pragma unroll
	for (int level = 1; level >= 0; level--) {
		int tx[8], ty[8], q[8];
#pragma unroll
		for (int k = 0; k < 8; k++) {
			tx[k] = (int16_t)(bx4 + (ox[k] << level));
			ty[k] = (int16_t)(by4 + (oy[k] << level));
			const int pic = ((tx[k] & 3) << 2) | (ty[k] & 3);
			q[k] = ref_px(a.ref.p[pic], a, cx + (tx[k] >> 2), cy + (ty[k] >> 2), lane);
		}
		int d8[8];
#pragma unroll
		for (int k = 0; k < 8; k++) d8[k] = sad_of(abs(cur - q[k]));
		int nx = bx4, ny = by4;
#pragma unroll
		for (int k = 0; k < 8; k++)
			if (bd > d8[k]) { nx = tx[k]; ny = ty[k]; bd = d8[k]; }
		bx4 = nx;
		by4 = ny;
	}
	if (lane == 0) {
		a.mv[b] = mvmake(bx4, by4);
		a.dist[b] = (uint16_t)bd;
	}
}

// ----------------------------------------------------------------- OBMC
// COBMC::apply_mv (obmc.cpp:278-332) gathered per output sample.  Block
// (bi, bj) writes a 16x16 window at (8 bi - 4, 8 bj - 4) in raster order, so a
// sample receives, in order, the bottom-right quadrant of block (a-1, b-1),
// the bottom-left of (a, b-1), the top-right of (a-1, b) and the top-left of
// (a, b), where (a, b) = ((x + 4) >> 3, (y + 4) >> 3).  Each quadrant applies
// the statement obmc_block<flags> (obmc.cpp:80-177) has for it -- edge blocks
// (TOP / BOTTOM / LEFT / RIGHT) skip the half outside the frame and fold the
// missing neighbour's weight in -- and stores to short.  The value before the
// first statement is the previous prediction (the LEFT column's first
// statement accumulates onto it: obmc.cpp:158).  Intra blocks contribute 0
// (obmc_block_intra, :179-250).
// One workgroup per 64-column x 4 RW-row tile, a lane per column, wave w
// owning tile rows w RW .. w RW + RW - 1.  Every (block, window sample) pair
// feeds exactly one output sample, so the 12 B per sample are already the
// minimum.  The tile's blocks (10 columns x (RW/2 + 2) rows around it) are
// resolved once into a window-origin address in LDS (motion vector ->
// quarter-pel plane, get_pos clamping; 1 = intra, 0 = outside the frame); a
// lane then issues its RW prediction loads and all 4 RW window gathers before
// the first statement, so a tile costs two dependent memory trips (vectors,
// then samples) rather than two per quadrant.  The quadrant of each of the
// four contributions is static (k = 0..3: bottom-right, bottom-left,
// top-right, top-left), the window row is wave-uniform and the column is the
// lane's (x + 4) mod 8, so the weights are nibbles of two packed window rows.
// What bounds it: the windows' 32-byte rows sit in lines of
// their own when neighbouring blocks' vectors differ, so the L2 fetches whole
// lines for a quarter of their bytes; staging the window rows in LDS with
// aligned 16-byte loads (a quarter of the load instructions) and a persistent
// one-wave-per-strip form that prefetches the next strip's vectors were both
// slower (52.9 and 42.5 us against 40.7 at 1080p).
__constant__ uint32_t kWinRow[8] = {   // COBMC::window (obmc.cpp:56-66): window[j][i] at bits 4 i of word j
	0x11110000u, 0x22211100u, 0x44322110u, 0x66543210u, 0x98754211u, 0xB9975321u, 0xDC986421u, 0xEDB96421u};

// one statement of obmc_block<flags> (obmc.cpp:80-177) for the quadrant (top, left) of a block with
// edge flags T, Bo, L, R at window row jj / column cu, stored to short as the reference stores it
__device__ __forceinline__ int obmc_statement(int dd, int sv, bool top, bool left, bool T, bool Bo, bool L, bool R, int jj,
                                             int cu)
{
	const uint32_t rj = kWinRow[jj], rm = kWinRow[7 - jj];
	const int wl = (rj >> (4 * cu)) & 15, wr = (rj >> (28 - 4 * cu)) & 15;
	const int wlm = (rm >> (4 * cu)) & 15, wrm = (rm >> (28 - 4 * cu)) & 15;
	int q;
	if (top && left) {                             // top-left: the block's own quadrant
		if (T && L) q = sv;
		else if (T) q = (dd + sv * (wl + wlm) + 8) >> 4;
		else if (L) q = (dd + sv * (wl + wr) + 8) >> 4;
		else q = (dd + sv * wl + 8) >> 4;
	} else if (top) {                              // top-right
		if (T && R) q = sv;
		else if (T) q = sv * (wr + wrm);
		else if (R) q = (dd + sv * (wr + wl) + 8) >> 4;
		else q = dd + sv * wr;
	} else if (left) {                             // bottom-left
		if (Bo && L) q = sv;
		else if (Bo) q = (dd + sv * (wl + wlm) + 8) >> 4;
		else if (L) q = dd + sv * (wl + wr);
		else q = dd + sv * wl;
	} else {                                       // bottom-right
		if (Bo && R) q = sv;
		else if (Bo) q = sv * (wr + wrm);
		else if (R) q = sv * (wr + wl);
		else q = sv * wr;
	}
	return (int16_t)q;
}

typedef const __attribute__((address_space(1))) int16_t* gsamples;

template <int RW>
__global__ __launch_bounds__(256) void k_vid_obmc(VidSubs ref, const uint32_t* __restrict__ mv, int16_t* __restrict__ pred,
                                                  int16_t* __restrict__ img, int w, int h, int S, long P, int bx, int by,
                                                  int ntx, int nty)
{
	constexpr int TR = 4 * RW, NJ = TR / 8 + 2, NI = 10;
	__shared__ unsigned long long blk[NJ * NI];
	// XCD-aware tile order (as k_vid_epzs_sub): workgroup g takes tile
	// (g % 8) C + g / 8, so each XCD sweeps one band of tile rows and the
	// windows a tile shares with the one above it are still in its L2
	const int nt = ntx * nty * 3, C = (nt + 7) >> 3;
	const int tile = (int)(blockIdx.x & 7) * C + (int)(blockIdx.x >> 3);
	if (tile >= nt) return;
	const int X0 = tile % ntx * 64, Y0 = tile / ntx % nty * TR, J0 = Y0 / 8 - 1;
	const long pc = tile / (ntx * nty) * P;
	const int t = threadIdx.x;
	if (t < NJ * NI) {
		const int bi = X0 / 8 - 1 + t % NI, bj = J0 + t / NI;
		unsigned long long e = 0;
		if (bi >= 0 && bi < bx && bj >= 0 && bj < by) {
			const uint32_t m = mv[(long)bj * bx + bi];
			e = 1;
			if (m != kVidIntra) {
				const int mx = mvx(m), my = mvy(m);
				int px = 8 * bi + (mx >> 2) - 4, py = 8 * bj + (my >> 2) - 4;   // get_pos, obmc.cpp:252-263
				px = px < -15 ? -15 : px >= w ? w - 1 : px;
				py = py < -15 ? -15 : py >= h ? h - 1 : py;
				e = (unsigned long long)(ref.p[((mx & 3) << 2) | (my & 3)] + pc + (long)py * S + px);
			}
		}
		blk[t] = e;
	}
	const int lane = t & 63, wv = __builtin_amdgcn_readfirstlane(t >> 6);
	// with img (the encoder) the tiles cover the whole w x h plane: the
	// residual img - prediction is taken here (CImage::operator-=), also on
	// the columns / rows past the last whole block that OBMC leaves alone
	const int x = X0 + lane, xe = img ? w : 8 * bx, ye = img ? h : 8 * by;
	const bool xin = x < 8 * bx;
	int d[RW], c[RW];
#pragma unroll
	for (int r = 0; r < RW; r++) {
		const int y = Y0 + wv * RW + r;
		const bool ok = x < xe && y < ye;
		d[r] = ok ? pred[pc + (long)y * S + x] : 0;
		c[r] = ok && img ? img[pc + (long)y * S + x] : 0;
	}
	__syncthreads();
	if (x >= xe) return;
	const int a0 = (x + 4) >> 3, cu = x + 4 - 8 * a0, ia = a0 - (X0 / 8 - 1);
	const bool Lm = a0 - 1 == 0, Rm = a0 - 1 == bx - 1, La = a0 == 0, Ra = a0 == bx - 1;
	int s[RW][4];
#pragma unroll
	for (int r = 0; r < RW; r++) {
		const int y = Y0 + wv * RW + r;
		const int b0 = (y + 4) >> 3, cv = y + 4 - 8 * b0;
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const int sel = (k & 2) ? 1 : 0, bq = ia - ((k & 1) ? 0 : 1);
			const unsigned long long e = blk[(b0 - 1 + sel - J0) * NI + bq];
			const int u = cu + ((k & 1) ? 0 : 8), v = cv + (sel ? 0 : 8);
			s[r][k] = 0;
			if (xin && y < 8 * by && e > 1) s[r][k] = ((gsamples)e)[(long)v * S + u];
		}
	}
#pragma unroll
	for (int r = 0; r < RW; r++) {
		const int y = Y0 + wv * RW + r;
		if (y >= ye) continue;
		const long o = pc + (long)y * S + x;
		const int b0 = (y + 4) >> 3, cv = y + 4 - 8 * b0;
		const bool inb = xin && y < 8 * by;
		int dd = d[r];
#pragma unroll
		for (int k = 0; k < 4 && inb; k++) {
			const bool top = k & 2, left = k & 1;
			const int bj = b0 - (top ? 0 : 1);
			if (blk[(bj - J0) * NI + ia - (left ? 0 : 1)] == 0) continue;   // outside the frame
			const bool T = bj == 0, Bo = bj == by - 1, L = left ? La : Lm, R = left ? Ra : Rm;
			const int jj = top ? cv : 7 - cv;             // the window row (the bottom half counts down)
			if (top ? (T && jj < 4) : (Bo && jj < 4)) continue;
			if (left ? (L && cu < 4) : (R && cu >= 4)) continue;
			dd = obmc_statement(dd, s[r][k], top, left, T, Bo, L, R, jj, cu);
		}
		if (inb) pred[o] = (int16_t)dd;
		if (img) img[o] = (int16_t)(c[r] - dd);
	}
}

// ------------------------------------------- TransformI's side effect
__global__ void k_vid_tinv_side(int16_t* __restrict__ plane, const int16_t* __restrict__ ll1, long pitch, int dx1,
                                int dy1, int w, int h, int S)
{
	const int cc = blockIdx.x * blockDim.x + threadIdx.x, k = blockIdx.y;
	if (cc >= dx1) return;
	int row = h - dy1 + k, colp = kVidBorder + S - dx1 + cc;   // physical column (pImage sits at column 15)
	if (colp >= S) { row++; colp -= S; }
	const int col = colp - kVidBorder;
	if (row >= 0 && row < h && col >= 0 && col < w) return;    // the level-0 output owns the plane itself
	plane[(long)row * S + col] = ll1[(long)k * pitch + cc];
}

int launched() { return hipGetLastError() == hipSuccess ? 0 : -1; }

}  // namespace

int launch_vid_input(const VidGeom& g, const uint8_t* rgb, int stride, int16_t* img, hipStream_t st)
{
	hipLaunchKernelGGL(k_vid_input, dim3((g.w + 255) / 256, g.h), dim3(256), 0, st, rgb, stride, img, g.w, g.h, g.S, g.P);
	return launched();
}

int launch_vid_addsub(const VidGeom& g, int16_t* img, const int16_t* pred, int sign, hipStream_t st)
{
	hipLaunchKernelGGL(k_vid_addsub, dim3((g.w + 255) / 256, g.h, 3), dim3(256), 0, st, img, pred, g.w, g.S, g.P, sign);
	return launched();
}

int launch_vid_interp(const VidGeom& g, const VidSubs& s, hipStream_t st)
{
	hipLaunchKernelGGL(k_vid_interp, dim3((g.w + 127) / 128, g.h, 3), dim3(128), 0, st, s, g.w, g.h, g.S, g.P);
	return launched();
}

int launch_vid_extend(const VidGeom& g, const VidSubs& s, int n, hipStream_t st)
{
	const int total = 2 * kVidBorder * (g.w + 2 * kVidBorder) + 2 * kVidBorder * g.h;
	hipLaunchKernelGGL(k_vid_extend, dim3((total + 255) / 256, 3, n), dim3(256), 0, st, s, g.w, g.h, g.S, g.P);
	return launched();
}

int launch_vid_epzs(const VidGeom& g, const int16_t* cur, const VidSubs& ref, uint32_t* mv, uint16_t* dist,
                    uint64_t* gran, uint32_t epoch, uint32_t* status, hipStream_t st)
{
	if (g.bx < 1 || g.by < 1) return 0;
	if (epoch == 0) return -1;
	EpzsArgs a;
	a.cur = cur; a.ref = ref; a.mv = mv; a.dist = dist; a.gran = gran; a.epoch = epoch; a.status = status;
	a.w = g.w; a.h = g.h; a.S = g.S; a.bx = g.bx; a.by = g.by;
	hipLaunchKernelGGL(k_vid_epzs_full, dim3(g.by), dim3(64), 0, st, a);
	if (launched()) return -1;
	hipLaunchKernelGGL(k_vid_epzs_sub, dim3(8 * ((g.bx * g.by + 7) / 8)), dim3(64), 0, st, a);
	return launched();
}

int launch_vid_obmc(const VidGeom& g, const uint32_t* mv, const VidSubs& ref, int16_t* pred, int16_t* residual,
                    hipStream_t st)
{
	static const int rw = [] { const char* e = getenv("RIC_OBMC_RW"); return e && atoi(e) == 8 ? 8 : 4; }();   // A/B knob
	const int xe = residual ? g.w : 8 * g.bx, ye = residual ? g.h : 8 * g.by;
	const int ntx = (xe + 63) / 64, nty = (ye + 4 * rw - 1) / (4 * rw), C = (ntx * nty * 3 + 7) / 8;
	if (ntx < 1 || nty < 1) return 0;
	hipLaunchKernelGGL(rw == 8 ? k_vid_obmc<8> : k_vid_obmc<4>, dim3(8 * C), dim3(256), 0, st, ref, mv, pred, residual, g.w,
	                   g.h, g.S, g.P, g.bx, g.by, ntx, nty);
	return launched();
}

int launch_vid_tinv_side(const VidGeom& g, int16_t* plane, const int16_t* ll1, long ll1_pitch, int dx1, int dy1,
                         hipStream_t st)
{
	if (dx1 < 1 || dy1 < 1) return 0;
	hipLaunchKernelGGL(k_vid_tinv_side, dim3((dx1 + 127) / 128, dy1), dim3(128), 0, st, plane, ll1, ll1_pitch, dx1, dy1,
	                   g.w, g.h, g.S);
	return launched();
}

}  // namespace ric
