// compact.hip -- the host coder's payload of a frame, compacted on the GPU.
//
// The host encoder (encoder.cpp tree_rec_core) reads, per coded block, the
// values at the set bits of its significance mask, in the walk order of
// CBandCodec::tree<encode> (bandcodec.cpp:509-523: block rows serpentine,
// coarse levels first, V, H, D).  A 16-bit band at C3 q9 is ~55 % zeros, so
// instead of the dense bands (2 B per coefficient) the frame's short bands go
// to the host as one stream of just those values, in the order the walk
// consumes them: every block contributes popcount(mask) values (insignificant
// blocks have an empty mask; a propagated block's values are skipped by the
// walk, which still steps over them).  The int bands (the coarsest levels),
// the LL, the block records and the parent info stay dense.
//
// Three passes per group of frames (blockIdx.z = frame): counts per chunk of
// 64 blocks, one exclusive scan per frame, then the chunk's values written at
// its offset (a wave-level prefix places each block).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include "ric_types.h"
#include "symbols.h"
#include "compact.h"

namespace ric {
namespace {

// global-address-space views of device pointers: global (not flat) loads and
// stores, counted by vmcnt alone, so a wave's waits on its LDS and scalar
// loads do not also wait for the loads it issued ahead
#define GAS __attribute__((address_space(1)))
template <typename T> __device__ __forceinline__ const GAS T* gp(const T* p) { return (const GAS T*)p; }
template <typename T> __device__ __forceinline__ GAS T* gp(T* p) { return (GAS T*)p; }

__device__ __forceinline__ int lane64() { return (int)(threadIdx.x & 63); }

__device__ __forceinline__ int wave_excl(int v, int& total)
{
	// inclusive scan over the 64 lanes by shuffles, then exclusive
	int x = v;
	const int l = (int)__lane_id();
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const int y = __shfl_up(x, o, 64);
		if (l >= o) x += y;
	}
	total = __shfl(x, 63, 64);
	return x - v;
}

// the band of flattened chunk index c (bands in coding order), searched from
// band b0: a wave's chunks only ever move forward, so it passes each band
// boundary once (a search from band 0 per chunk is a chain of up to 14
// dependent scalar loads, which bound these kernels)
__device__ __forceinline__ int band_of(const CmpArgs& a, int c, int b0 = 0)
{
	int b = b0;
	while (b + 1 < a.nb && c >= a.band[b + 1].chunk0) b++;
	return b;
}

// the mask of the block at scan position s0 + lane
__device__ __forceinline__ uint32_t block_mask(const CmpArgs& a, const char* arena, int b, int s0)
{
	const CmpBand& B = a.band[b];
	if (s0 + lane64() >= B.nblk) return 0;
	int bx, by;
	scan_block(s0 + lane64(), B.dx, B.dy, bx, by);
	const uint64_t r = gp((const uint64_t*)(arena + B.rec_off))[(long)by * ((B.dx + 3) >> 2) + bx];
	return BlockRec::mask(r);
}

// exclusive prefix over the wave's lanes of v < 32, and the wave's total: a
// ballot per bit of v (five), each lane's count of the set lanes below it
__device__ __forceinline__ uint32_t wave_prefix5(uint32_t v, uint32_t& tot)
{
	uint32_t o = 0, t = 0;
#pragma unroll
	for (int b = 0; b < 5; b++) {
		const uint64_t bb = __ballot((v >> b) & 1u);
		o += __builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u)) << b;
		t += (uint32_t)__popcll(bb) << b;
	}
	tot = t;
	return o;
}

// (bx, by) of scan position s0 + lane (s0 wave-uniform, scan_block's order):
// a chunk of a band at least 64 blocks wide spans at most two block rows, so
// the row is one scalar division per chunk and a compare per lane instead of
// a division per lane
__device__ __forceinline__ void chunk_block(int s0, int lane, int dx, int dy, int& bx, int& by)
{
	const int bw = (dx + 3) >> 2, nfx = dx >> 2;
	if (bw < 64) { scan_block(s0 + lane, dx, dy, bx, by); return; }
	const int by0 = s0 / bw;
	int p = s0 - by0 * bw + lane;
	by = by0;
	if (p >= bw) { p -= bw; by++; }
	if (!(by & 1)) bx = p;
	else if (nfx < bw) bx = p == 0 ? nfx : nfx - p;
	else bx = nfx - 1 - p;
}

// A few workgroups of 4 waves per frame, each wave striding over the chunks:
// a workgroup per chunk would be hundreds of thousands of tiny dispatches,
// which crawl when the stream coder's waves fill the CUs.
constexpr int kCmpWaves = 4;
// (readfirstlane: the wave's index is uniform, so its chunk index, band and
// band fields are scalar -- else every band field is a per-lane vector load
// waited on before the next)
__device__ __forceinline__ int wave_gid()
{
	return (int)(blockIdx.x * kCmpWaves + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6));
}
__device__ __forceinline__ int wave_count() { return (int)(gridDim.x * kCmpWaves); }

// four chunks per step, their record loads issued together
__global__ __launch_bounds__(64 * kCmpWaves) void k_cmp_count(const CmpArgs* __restrict__ ap)
{
	const CmpArgs& a = *ap;
	const int f = blockIdx.z;
	const char* arena = a.arena + (size_t)f * a.astride;
	const int W = wave_count();
	int bu[4] = {0, 0, 0, 0};
	for (int c0 = wave_gid(); c0 < a.nchunk; c0 += 4 * W) {
		int n[4];
#pragma unroll
		for (int u = 0; u < 4; u++) {
			const int c = c0 + u * W;
			n[u] = 0;
			if (c < a.nchunk) {
				const int b = bu[u] = band_of(a, c, bu[u]);
				n[u] = __popc(block_mask(a, arena, b, (c - a.band[b].chunk0) * 64));
			}
		}
#pragma unroll
		for (int u = 0; u < 4; u++) {
			const int c = c0 + u * W;
#pragma unroll
			for (int o = 32; o > 0; o >>= 1) n[u] += __shfl_xor(n[u], o, 64);
			if (c < a.nchunk && lane64() == 0) gp(a.cnt)[(size_t)f * a.cstride + c] = (uint32_t)n[u];
		}
	}
}

// one workgroup per frame: exclusive scan of the chunk counts in place, the
// frame's total to total[f]
__global__ __launch_bounds__(1024) void k_cmp_scan(const CmpArgs* __restrict__ ap)
{
	const CmpArgs& a = *ap;
	const int f = blockIdx.z;
	uint32_t* cnt = a.cnt + (size_t)f * a.cstride;
	__shared__ uint32_t part[16];
	__shared__ uint32_t carry;
	if (threadIdx.x == 0) carry = 0;
	__syncthreads();
	const int l = (int)threadIdx.x & 63, w = (int)threadIdx.x >> 6;
	for (int base = 0; base < a.nchunk; base += 1024) {
		const int i = base + (int)threadIdx.x;
		const int v = i < a.nchunk ? (int)cnt[i] : 0;
		int tot;
		const int ex = wave_excl(v, tot);
		if (l == 0) part[w] = (uint32_t)tot;
		__syncthreads();
		uint32_t before = carry;
		for (int k = 0; k < w; k++) before += part[k];
		if (i < a.nchunk) cnt[i] = before + (uint32_t)ex;
		__syncthreads();
		if (threadIdx.x == 0) {
			uint32_t t = 0;
			for (int k = 0; k < 16; k++) t += part[k];
			carry += t;
		}
		__syncthreads();
	}
	if (threadIdx.x == 0) {
		a.total[f] = carry;
		if (a.vcap && carry > a.vcap && a.status) atomicOr((int32_t*)(a.status + (size_t)f * a.sstride), kCmpOverCap);
	}
}

// Each wave gathers its chunk's values into LDS (a lane holds its block's rows
// as 8-byte words, its values go to the chunk's slots from its prefix), then
// writes the chunk's run out with consecutive lanes on consecutive values: one
// coalesced store per 64 values instead of a lane-strided store per value.
// A wave's loads for its next chunk (record, rows, offset) are issued before
// it works on the current one: with every load of a chunk independent of the
// others, a wave keeps two chunks of loads in flight instead of waiting for
// the record, then the rows, chunk after chunk.
struct CmpChunk {
	uint64_t rec;                    // the lane's block record (0: past the band)
	uint64_t v[4];                   // its rows (valid up to its height)
	uint32_t base;                   // the chunk's first value
	int b, s;                        // band, scan position
	int bx, by;                      // the lane's block
};

template <bool BASE = true>
__device__ __forceinline__ void cmp_load(const CmpArgs& a, const char* arena, const char* bsrc, int f, int c, int b0,
                                         CmpChunk& L)
{
	const int b = band_of(a, c, b0);
	const CmpBand& B = a.band[b];
	const int s0 = (c - B.chunk0) * 64, s = s0 + lane64();
	L.b = b; L.s = s;
	L.base = BASE ? gp(a.cnt)[(size_t)f * a.cstride + c] : 0u;
	L.rec = 0;
	L.v[0] = L.v[1] = L.v[2] = L.v[3] = 0;
	int bx, by;
	chunk_block(s0, lane64(), B.dx, B.dy, bx, by);
	L.bx = bx; L.by = by;
	if (s < B.nblk) {
		L.rec = gp((const uint64_t*)(arena + B.rec_off))[(long)by * ((B.dx + 3) >> 2) + bx];
		const int h = B.dy - by * 4;
		// rows of the block: an 8-byte word each (the row pitch keeps the
		// block's 4 columns inside the row's allocation), rows past the band not read
		const int16_t* band = (const int16_t*)(bsrc + B.off) + (long)by * 4 * B.pitch + bx * 4;
#pragma unroll
		for (int r = 0; r < 4; r++)
			if (r < h) L.v[r] = *gp((const uint64_t*)(band + (long)r * B.pitch));
	}
}

// one chunk's values out: the lane's block holds its values from o on (its
// prefix in the chunk), the chunk's tot values start at base.  They are
// gathered in the wave's LDS slots sv, then stored with consecutive lanes on
// consecutive values.
__device__ __forceinline__ void cmp_put(const CmpArgs& a, int16_t* out, int16_t* sv, const CmpChunk& cur, uint32_t o,
                                        uint32_t tot, uint32_t base)
{
	const int l = lane64();
	uint32_t m = BlockRec::mask(cur.rec);
	// over the pool's capacity: flagged (k_cmp_scan / k_cmp_one), nothing written
	if (a.vcap && base + tot > a.vcap) return;
	const CmpBand& B = a.band[cur.b];
	const int w = B.dx - cur.bx * 4 < 4 ? B.dx - cur.bx * 4 : 4;
	uint32_t k = o;
	if (w == 4) {
		// the 16 positions in raster order, straight through: a kept
		// value to its slot, the others to the lane's dump slot
		const uint32_t dump = 1024u + (uint32_t)l;
#pragma unroll
		for (int i = 0; i < 16; i++) {
			const uint32_t bit = (m >> i) & 1u;
			sv[bit ? k : dump] = (int16_t)(cur.v[i >> 2] >> (16 * (i & 3)));
			k += bit;
		}
	} else if (m) {
		// a block cut by the band's right edge: w values per row
#pragma unroll
		for (int r = 0; r < 4; r++) {
			const uint32_t rm = m & ((1u << w) - 1u);
			m >>= w;
			for (uint32_t q = rm; q; q &= q - 1) sv[k++] = (int16_t)(cur.v[r] >> (16 * __builtin_ctz(q)));
		}
	}
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	for (uint32_t i = (uint32_t)l; i < tot; i += 64) gp(out)[base + i] = sv[i];
	__builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(64 * kCmpWaves) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_cmp_write(const CmpArgs* __restrict__ ap)
{
	const CmpArgs& a = *ap;
	const int f = blockIdx.z;
	const char* arena = a.arena + (size_t)f * a.astride;
	const char* bsrc = a.bsrc ? a.bsrc + (size_t)f * a.bstride : arena;
	int16_t* out = (int16_t*)(a.out + (size_t)f * a.ostride);
	// a chunk's values, then one dump slot per lane (the writes of the
	// positions a lane does not keep)
	__shared__ int16_t stage[kCmpWaves][64 * 16 + 64];
	int16_t* sv = stage[threadIdx.x >> 6];
	const int l = lane64();
	int c = wave_gid();
	CmpChunk cur, nxt;
	if (c < a.nchunk) cmp_load(a, arena, bsrc, f, c, 0, cur);
	for (; c < a.nchunk; c += wave_count()) {
		const int cn = c + wave_count();
		if (cn < a.nchunk) cmp_load(a, arena, bsrc, f, cn, cur.b, nxt);
		uint32_t tot;
		const uint32_t o = wave_prefix5((uint32_t)__popc(BlockRec::mask(cur.rec)), tot);
		cmp_put(a, out, sv, cur, o, tot, cur.base);
		cur = nxt;
	}
}

// ---- one pass (RIC_CMP_PASS=1; the default is the three kernels above).
// Counts, the frame's running value offset and the values in one kernel: a
// workgroup takes the next ticket of its frame (an atomic counter, so every
// lower ticket belongs to a workgroup already running), loads its kCpg chunks
// once (records and band rows, all in flight together), publishes its value
// count and looks back over the tickets before it for its offset (decoupled
// look-back: the nearest inclusive prefix plus the counts between), then
// writes its values.  The records are read once instead of twice, and the
// scan pass and two launches are gone.
// Per frame, the cnt array holds the ticket counter (u32 0) and one u64 status
// per ticket from byte 8: epoch << 34 | flag << 32 | value, flag 1 = the
// ticket's count, 2 = the count of every value up to and including it.  The
// epoch (a per-launch number) tells this launch's words from the previous
// ones', so nothing is reset between launches; the last ticket resets the
// counter.  A look-back that waits too long (never on a working device) gives
// up, sets kCmpLookback in the frame's status word and writes nothing.
// Measured in the C3 serving step (profiles/r06_cmp_onepass_ab.txt), per frame:
// 4 chunks per wave 45.7 us, 8 chunks 36.9, 4 at issue priority 3 41.4, 8 at
// priority 3 31.9 -- against 32.3 for the three passes (count 7.3 + scan 2.4
// + write 22.9): the look-back's round trips (ticket, status words) and its
// waits on slower predecessors beside the coder waves cost what the saved
// record reads and launches gain.  Kept as the opt-in form at 8 / 3.
#ifndef RIC_CMP_CPW
#define RIC_CMP_CPW 8
#endif
#ifndef RIC_CMP_PRIO
#define RIC_CMP_PRIO 3
#endif
constexpr int kCpw = RIC_CMP_CPW;                // chunks per wave
constexpr int kCpg = kCmpWaves * kCpw;           // chunks per workgroup (ticket)
constexpr uint32_t kLbAgg = 1u, kLbInc = 2u;
constexpr int kLbPolls = 1 << 20;

__device__ __forceinline__ uint64_t lb_word(uint32_t epoch, uint32_t flag, uint32_t v)
{
	return (uint64_t)epoch << 34 | (uint64_t)flag << 32 | v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
	return v;
}

// (one wave) the values before ticket t; ok false: gave up
__device__ __forceinline__ uint32_t lookback(uint64_t* stat, int t, uint32_t epoch, bool& ok)
{
	const int l = lane64();
	uint32_t acc = 0;
	int hi = t - 1, polls = 0;
	while (hi >= 0) {
		const int i = hi - l;
		const uint64_t v = i >= 0 ? __hip_atomic_load(stat + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
		                          : lb_word(epoch, kLbInc, 0);
		const uint32_t fl = (uint32_t)(v >> 32) & 3u;
		const bool valid = (uint32_t)(v >> 34) == epoch && fl != 0;
		const uint64_t incm = __ballot(valid && fl == kLbInc);
		const uint64_t bad = __ballot(!valid);
		// the lanes needed: up to the nearest inclusive prefix, or all 64
		const int lim = incm ? __builtin_ctzll(incm) : 63;
		const uint64_t need = lim == 63 ? ~0ull : ((2ull << lim) - 1);
		if (bad & need) {
			if (++polls > kLbPolls) { ok = false; return 0; }
			__builtin_amdgcn_s_sleep(2);
			continue;
		}
		acc += wave_sum(l <= lim ? (uint32_t)v : 0u);
		if (incm) break;
		hi -= 64;
	}
	ok = true;
	return acc;
}

__global__ __launch_bounds__(64 * kCmpWaves) void k_cmp_one(const CmpArgs* __restrict__ ap, uint32_t epoch)
{
	const CmpArgs& a = *ap;
	const int f = blockIdx.z;
	const char* arena = a.arena + (size_t)f * a.astride;
	const char* bsrc = a.bsrc ? a.bsrc + (size_t)f * a.bstride : arena;
	int16_t* out = (int16_t*)(a.out + (size_t)f * a.ostride);
	uint32_t* fc = a.cnt + (size_t)f * a.cstride;
	uint64_t* stat = (uint64_t*)(fc + 2);
	__shared__ int16_t stage[kCmpWaves][64 * 16 + 64];
	__shared__ uint32_t s_t, s_pre, s_ok, s_wtot[kCmpWaves];
	const int G = (int)gridDim.x;
	if (RIC_CMP_PRIO) __builtin_amdgcn_s_setprio(RIC_CMP_PRIO);
	if (threadIdx.x == 0) {
		const uint32_t t = atomicAdd(fc, 1u);
		// every ticket of this launch is taken: the counter back to 0 for the next
		if (t == (uint32_t)G - 1) __hip_atomic_store(fc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		s_t = t;
	}
	__syncthreads();
	const int t = (int)__builtin_amdgcn_readfirstlane(s_t);
	const int w = (int)__builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
	const int l = lane64();
	int16_t* sv = stage[w];
	const int c0 = t * kCpg + w * kCpw;
	CmpChunk ch[kCpw];
	int b = 0;
#pragma unroll
	for (int u = 0; u < kCpw; u++) {
		if (c0 + u < a.nchunk) {
			cmp_load<false>(a, arena, bsrc, f, c0 + u, b, ch[u]);
			b = ch[u].b;
		} else {
			ch[u].rec = 0; ch[u].b = b; ch[u].s = 0; ch[u].bx = ch[u].by = 0; ch[u].base = 0;
		}
	}
	uint32_t op[kCpw], tot[kCpw], cb[kCpw], wsum = 0;
#pragma unroll
	for (int u = 0; u < kCpw; u++) {
		op[u] = wave_prefix5((uint32_t)__popc(BlockRec::mask(ch[u].rec)), tot[u]);
		cb[u] = wsum;
		wsum += tot[u];
	}
	if (l == 0) s_wtot[w] = wsum;
	__syncthreads();
	uint32_t wpre = 0, gtot = 0;
#pragma unroll
	for (int k = 0; k < kCmpWaves; k++) {
		const uint32_t v = s_wtot[k];
		if (k < w) wpre += v;
		gtot += v;
	}
	if (w == 0) {
		uint32_t pre = 0;
		bool ok = true;
		if (t == 0) {
			if (l == 0) __hip_atomic_store(stat, lb_word(epoch, kLbInc, gtot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		} else {
			if (l == 0) __hip_atomic_store(stat + t, lb_word(epoch, kLbAgg, gtot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
			pre = lookback(stat, t, epoch, ok);
			if (l == 0 && ok)
				__hip_atomic_store(stat + t, lb_word(epoch, kLbInc, pre + gtot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		}
		if (l == 0) { s_pre = pre; s_ok = ok; }
	}
	__syncthreads();
	if (!s_ok) {
		if (threadIdx.x == 0 && a.status) atomicOr((int32_t*)(a.status + (size_t)f * a.sstride), kCmpLookback);
		return;
	}
	const uint32_t base0 = s_pre + wpre;
	if (t == G - 1 && threadIdx.x == 0) {
		const uint32_t total = s_pre + gtot;
		a.total[f] = total;
		if (a.vcap && total > a.vcap && a.status) atomicOr((int32_t*)(a.status + (size_t)f * a.sstride), kCmpOverCap);
	}
#pragma unroll
	for (int u = 0; u < kCpw; u++)
		if (c0 + u < a.nchunk) cmp_put(a, out, sv, ch[u], op[u], tot[u], base0 + cb[u]);
}

// the decode side: one wave per chunk of 64 blocks (flattened over the three
// bands), every position of each block written, a value where its mask bit is
// set.  The chunk's values are contiguous (its offset to the next chunk's, or
// the band's count).  A wave loads the next chunk's masks, offsets and values
// while it writes the current one: the values as 16-byte words (the chunk's
// run rounded out to 16-byte boundaries, at most 3 words a lane), staged in
// LDS at the chunk's start; then each lane assembles its block's rows and
// writes each as one 8-byte word (a narrow edge block value by value).
// (Round 5 loaded a chunk's values 2 bytes a lane once the chunk started:
// 23 us per C3 frame alone, 0.44 of HBM peak.)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kDcmpW = 3;                 // 16-byte value words per lane: 3 x 64 x 8 >= 1024 + 14 values
struct DcmpChunk {
	uint32_t m;                      // the lane's block mask (loaded)
	uint32_t o0, tot;                // the chunk's first value and count
	uint32_t a0;                     // o0 rounded down to 8 values (16 bytes)
	u32x4 w[kDcmpW];                 // values a0 + 8 (lane + 64 i) .. + 7
	int b, s;
};

__device__ __forceinline__ void dcmp_load(const DcmpArgs& a, const char* in, int c, DcmpChunk& L)
{
	const uint32_t* nval = (const uint32_t*)in;
	const int b = c >= a.chunk0[2] ? 2 : c >= a.chunk0[1] ? 1 : 0;
	const int ch = c - a.chunk0[b];
	const int s = ch * 64 + lane64();
	const uint32_t* coff = (const uint32_t*)(in + a.coff_off[b]);
	uint32_t vbase = 0;
	for (int k = 0; k < b; k++) vbase += nval[k];
	L.b = b; L.s = s;
	L.o0 = vbase + coff[ch];
	L.tot = (ch + 1 < a.chunk0[b + 1] - a.chunk0[b] ? coff[ch + 1] : nval[b]) - coff[ch];
	L.m = s < a.nblk[b] ? gp((const uint16_t*)(in + a.mask_off[b]))[s] : 0u;
	// the value words: none past the pool's capacity (a frame the coder left
	// to the host holds no valid offsets; the capacity's block is rounded up
	// to 256 bytes, so a word ending past vcap but below vcap rounded to 8 is
	// inside it)
	L.a0 = L.o0 & ~7u;
	const uint32_t tot = L.tot < 1024u ? L.tot : 1024u;
	const uint32_t nw = (L.o0 + tot - L.a0 + 7u) >> 3;
	const uint32_t lim = a.vcap ? ((a.vcap + 7u) >> 3) : 0xFFFFFFFFu;
	const u32x4* vw = (const u32x4*)(in + a.vals_off);
#pragma unroll
	for (int i = 0; i < kDcmpW; i++) {
		const uint32_t j = (uint32_t)lane64() + 64u * (uint32_t)i;
		const uint32_t wi = (L.a0 >> 3) + j;
		u32x4 v = {0, 0, 0, 0};
		if (j < nw && wi < lim) v = *gp(vw + wi);
		L.w[i] = v;
	}
}

__global__ __launch_bounds__(64 * kCmpWaves) void k_dcmp_expand(DcmpArgs a)
{
	const int f = blockIdx.z;
	const char* in = a.in + (size_t)f * a.istride;
	__shared__ u32x4 stage[kCmpWaves][64 * kDcmpW];
	int16_t* sv = (int16_t*)stage[threadIdx.x >> 6];
	const int l = lane64();
	int c = wave_gid();
	DcmpChunk cur, nxt;
	if (c < a.chunk0[3]) dcmp_load(a, in, c, cur);
	for (; c < a.chunk0[3]; c += wave_count()) {
		// the chunk's value words into LDS
#pragma unroll
		for (int i = 0; i < kDcmpW; i++) ((u32x4*)sv)[l + 64 * i] = cur.w[i];
		const int cn = c + wave_count();
		if (cn < a.chunk0[3]) dcmp_load(a, in, cn, nxt);
		const uint32_t m = cur.m;
		uint32_t ptot;
		// value k of the chunk is sv[sh + k]; past the capacity it reads as 0
		const uint32_t sh = cur.o0 - cur.a0;
		uint32_t k = wave_prefix5((uint32_t)__popc(m), ptot);
		const uint32_t kcap = a.vcap ? (a.vcap > cur.o0 ? a.vcap - cur.o0 : 0u) : 0xFFFFFFFFu;
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		const int b = cur.b, s = cur.s;
		int bx, by;
		chunk_block(s - l, l, a.dx[b], a.dy[b], bx, by);
		if (s < a.nblk[b]) {
			const int w = a.dx[b] - bx * 4 < 4 ? a.dx[b] - bx * 4 : 4, h = a.dy[b] - by * 4 < 4 ? a.dy[b] - by * 4 : 4;
			int16_t* band = (int16_t*)(a.arena + (size_t)f * a.astride + a.off[b]) + (long)by * 4 * a.pitch[b] + bx * 4;
			auto val = [&](uint32_t kk) -> uint32_t { return kk < kcap && kk < 1024u ? (uint16_t)sv[sh + kk] : 0u; };
			if (w == 4 && h == 4) {
				// straight through the 16 positions: a kept position takes the
				// lane's next value, the others read a slot and drop it
#pragma unroll
				for (int r = 0; r < 4; r++) {
					uint64_t word = 0;
#pragma unroll
					for (int q = 0; q < 4; q++) {
						const uint32_t bit = (m >> (4 * r + q)) & 1u;
						const uint32_t v = val(bit ? k : 0u);
						word |= (uint64_t)(bit ? v : 0u) << (16 * q);
						k += bit;
					}
					*gp((uint64_t*)(band + (long)r * a.pitch[b])) = word;
				}
			} else {
				// a block cut by the band's right or bottom edge
				uint32_t mm = m;
				for (int r = 0; r < h; r++) {
					uint64_t word = 0;
					for (int q = 0; q < w; q++, mm >>= 1)
						if (mm & 1u) word |= (uint64_t)val(k++) << (16 * q);
					if (w == 4) *gp((uint64_t*)(band + (long)r * a.pitch[b])) = word;
					else
						for (int q = 0; q < w; q++) gp(band)[(long)r * a.pitch[b] + q] = (int16_t)(word >> (16 * q));
				}
			}
		}
		__builtin_amdgcn_wave_barrier();
		cur = nxt;
	}
}

// the group's value streams straight into the host mirrors (pinned memory,
// device-mapped): frame f's total[f] values, 16 bytes per lane per step, so
// the host tasks find them in place once the group's event has passed
__global__ __launch_bounds__(256) void k_cmp_to_host(const char* __restrict__ src, size_t sstride, char* dst,
                                                     size_t dstride, const uint32_t* __restrict__ total)
{
	const int f = blockIdx.z;
	const size_t n16 = ((size_t)total[f] * 2 + 15) / 16;
	const uint4* s = (const uint4*)(src + (size_t)f * sstride);
	uint4* d = (uint4*)(dst + (size_t)f * dstride);
	for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) d[i] = s[i];
}

}  // namespace

int launch_cmp_to_host(const char* src, size_t sstride, char* dst, size_t dstride, const uint32_t* total, int nframes,
                       hipStream_t st)
{
	if (nframes <= 0) return 0;
	hipLaunchKernelGGL(k_cmp_to_host, dim3(32, 1, nframes), dim3(256), 0, st, src, sstride, dst, dstride, total);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

DcmpLayout dcmp_layout(const Pyramid& P)
{
	DcmpLayout L;
	const int order[3] = {BV, BH, BD};
	size_t off = 16;
	for (int k = 0; k < 3; k++) {
		const Band& B = P.L[0].b[order[k]];
		L.band[k] = order[k];
		L.nblk[k] = B.bw() * B.bh();
		L.nch[k] = (L.nblk[k] + 63) / 64;
		L.mask_off[k] = off;
		off += ((size_t)L.nblk[k] * 2 + 15) / 16 * 16;
	}
	for (int k = 0; k < 3; k++) {
		L.coff_off[k] = off;
		off += ((size_t)L.nch[k] * 4 + 15) / 16 * 16;
	}
	L.vals_off = off;
	L.ok = P.nlev >= 2 && !P.L[0].b[BD].is_int;
	return L;
}

int launch_dcmp_expand(const DcmpArgs& a, int nframes, hipStream_t st)
{
	if (nframes <= 0 || a.chunk0[3] <= 0) return 0;
	const int g = std::min(128, (a.chunk0[3] + 4 * kCmpWaves - 1) / (4 * kCmpWaves));
	hipLaunchKernelGGL(k_dcmp_expand, dim3(g, 1, nframes), dim3(64 * kCmpWaves), 0, st, a);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

void cmp_args(const Pyramid& P, CmpArgs& a)
{
	a.nb = 0;
	int chunk = 0;
	const int order[3] = {BV, BH, BD};
	for (int l = P.nlev - 1; l >= 0; l--)
		for (int k = 0; k < 3; k++) {
			const Band& B = P.L[l].b[order[k]];
			if (B.is_int) continue;                      // int bands stay dense
			CmpBand& d = a.band[a.nb++];
			d.off = (uint32_t)B.off;
			d.rec_off = (uint32_t)P.rec_off[l][order[k]];
			d.dx = B.dx; d.dy = B.dy; d.pitch = B.pitch;
			d.nblk = B.bw() * B.bh();
			d.chunk0 = chunk;
			chunk += (d.nblk + 63) / 64;
		}
	a.nchunk = chunk;
}

size_t cmp_values(const Pyramid& P)
{
	size_t n = 0;
	for (int l = 0; l < P.nlev; l++)
		for (int b = 0; b < 3; b++)
			if (!P.L[l].b[b].is_int) n += (size_t)P.L[l].b[b].dx * P.L[l].b[b].dy;
	return n;
}

size_t cmp_dense_from(const Pyramid& P)
{
	for (int l = 0; l < P.nlev; l++)
		if (P.L[l].b[BD].is_int) return P.L[l].b[BD].off;
	return P.L[P.nlev - 1].b[BL].off;
}

int launch_compact(const CmpArgs* dev_args, int nchunk, int nframes, hipStream_t st)
{
	if (nframes <= 0 || nchunk <= 0) return 0;
	// (read per call: a test runs both forms in one process)
	const char* pe = getenv("RIC_CMP_PASS");
	if (pe && atoi(pe) == 1) {
		// the look-back words: per frame, 8 + 8 G bytes of the cnt array's
		// up(nchunk, 64) words (cstride, batch.cpp), G = nchunk / 16 rounded up
		static std::atomic<uint32_t> epoch{0};
		uint32_t e = (epoch.fetch_add(1) + 1) & 0x3FFFFFFFu;
		if (!e) e = (epoch.fetch_add(1) + 1) & 0x3FFFFFFFu;
		const int g = (nchunk + kCpg - 1) / kCpg;
		hipLaunchKernelGGL(k_cmp_one, dim3(g, 1, nframes), dim3(64 * kCmpWaves), 0, st, dev_args, e);
		return hipGetLastError() == hipSuccess ? 0 : -1;
	}
	// about 4 chunks per wave, at most 128 workgroups per frame
	const int g = std::min(128, (nchunk + 4 * kCmpWaves - 1) / (4 * kCmpWaves));
	hipLaunchKernelGGL(k_cmp_count, dim3(g, 1, nframes), dim3(64 * kCmpWaves), 0, st, dev_args);
	hipLaunchKernelGGL(k_cmp_scan, dim3(1, 1, nframes), dim3(1024), 0, st, dev_args);
	hipLaunchKernelGGL(k_cmp_write, dim3(g, 1, nframes), dim3(64 * kCmpWaves), 0, st, dev_args);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace ric
