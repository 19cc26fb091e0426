// gcoder.hip -- the serial .ric coder on the GPU: one wave per stream.
//
// The .ric payload is one adaptive range-coder stream with a raw-bit FIFO
// multiplexed into it (CMuxCodec, src/lib/muxcodec.*); its state crosses every
// band, so a stream is inherently sequential.  What is
// parallel is the set of streams: a batch holds many independent frames.  Each
// frame's stream runs on one wave:
//  * every piece of coder state is wave-uniform: the compiler keeps it in
//    SGPRs and runs the coder on the scalar unit (SALU + scalar branches);
//  * the 16-context adaptive models (CBitCodec, CGeomCodec, k_mean) and the
//    small format tables live one context per lane of a VGPR ("lane arrays"),
//    read with v_readlane and written with a lane-select;
//  * the 64 lanes are the wave's load engine: they fetch the next 64 block
//    records and the next groups of block coefficients (4 blocks x 16 lanes)
//    ahead of the scalar walk, so the walk reads registers, not memory;
//  * stores (the coded bytes, decoded coefficients) go out from lane 0 as
//    vector stores.
// Output is byte-identical to the host coder (encoder.cpp / entropy.cpp),
// i.e. to the reference's tree<encode> / pred<encode> / CMuxCodec.
#include <hip/hip_runtime.h>
#include <mutex>
#include <vector>
#include <cstdlib>
#include <cstdint>
#include <cstdlib>

#include "ric_types.h"
#include "symbols.h"
#include "coder_tables.h"
#include "gcoder.h"

#ifndef RIC_GC_UNIFORM
#define RIC_GC_UNIFORM 0
#endif
#ifndef RIC_GC_ELOW_V
#define RIC_GC_ELOW_V 0
#endif
// RIC_GC_EVALU: the encoder's range coder (range, low) on the VALU, its
// branch conditions read back from lane 0.  The CU's one scalar unit serves
// the coder waves of all four SIMDs and ran at 0.70 instructions per cycle in
// the serving step (profiles/r06_stream_coder_sq.json); with the waves
// levelled (level_apply) they all encode at the same time, the encoder's
// bins then queueing on it.  Measured (one C3 serving step, 3072 streams,
// same box, r6ev): 10.02 s against 10.40 s per launch, 12,185-12,306 against
// 11,906 Mpix/s.
#ifndef RIC_GC_EVALU
#define RIC_GC_EVALU 1
#endif
// RIC_GC_UCOND: the decoder's state stays in VGPRs (the balanced SALU / VALU
// mix, see GDec::enum16) but its branch conditions are read from lane 0
// (v_readfirstlane): scalar branches instead of exec-mask ones
// Measured (one C3 serving step, 3072 streams, k_gc_roundtrip per launch;
// r5 g5, two runs each): 0 11348 ms, 1 12727, 2 11210-11215 (the default), 3 11582-11590
#ifndef RIC_GC_UCOND
#define RIC_GC_UCOND 2
#endif
// RIC_GC_GEOFAST: the geometric models' per-value scalar work trimmed (both
// coders): k + 1 and the remainder mask kept with k, the frequency update
// without its 16-bit mask and the re-index test as one unsigned compare (the
// frequency stays in [1, 4096] and the thresholds below 4096, so both are
// the reference's 16-bit arithmetic): launch 9.94 -> 9.77 s, two
// interleaved pairs (profiles/r06_geofast_ab_b*.log).  Splitting the
// decoder's empty-run path from the unary one as well was 3.8 % slower (the
// compiler then copies the window registers on the fast path).
#ifndef RIC_GC_GEOFAST
#define RIC_GC_GEOFAST 1
#endif
// RIC_GC_OUTPIN: launch 9.73 -> 9.44 s, two interleaved pairs
// (profiles/r06_outpin_ab_b*.log)
// RIC_GC_VADDR: the decoder's store position (ctz of the reversed mask) and
// address on the VALU, three scalar ops per value fewer: launch 9.46 -> 9.34 s
// (profiles/r06_vaddr_ab_b*.log)
#ifndef RIC_GC_VADDR
#define RIC_GC_VADDR 1
#endif
#ifndef RIC_GC_OUTPIN
#define RIC_GC_OUTPIN 1
#endif
// RIC_GC_SIGREV: the decoder walks a full block's significant positions by
// the lowest set bit of the bit-reversed mask
#ifndef RIC_GC_SIGREV
#define RIC_GC_SIGREV 1
#endif
// RIC_GC_NVGPR: the coder kernels' VGPR budget as amdgpu_num_vgpr takes it
// on gfx950 (half the unified VGPR + AGPR count: 44 = 88 VGPRs; 0 = none).
// Three coder waves of 96 VGPRs left a SIMD 224 of its 512 and RCCL's kernel
// (ncclDevKernel_Generic_1) wants 248 per wave: a send / receive issued
// during a launch waited until the launch's first coder waves retired.  At
// 88 three coder waves leave exactly 248 (one spilled dword per kernel).
#ifndef RIC_GC_NVGPR
#define RIC_GC_NVGPR 44
#endif
#if RIC_GC_NVGPR
#define GC_KATTR __attribute__((amdgpu_waves_per_eu(1, 5), amdgpu_num_vgpr(RIC_GC_NVGPR)))
#else
#define GC_KATTR
#endif

namespace ric {

#include "huff_tables.inc"

namespace {

using namespace tables;

#define GC_DI __device__ __forceinline__
// global-address-space views (plain loads/stores, not flat ones that also
// count against the LDS counter)
#define GAS __attribute__((address_space(1)))
template <typename T> GC_DI const GAS T* gld(const T* p) { return (const GAS T*)p; }
template <typename T> GC_DI GAS T* gst(T* p) { return (GAS T*)p; }
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

GC_DI uint32_t lane_id() { return __lane_id(); }
// a branch operand of the decoder, wave-uniform in fact (RIC_GC_UCOND)
GC_DI uint32_t ru(uint32_t x)
{
#if RIC_GC_UCOND
	return __builtin_amdgcn_readfirstlane(x);
#else
	return x;
#endif
}
// RIC_GC_UCOND 2: the raw-bit reader's state pinned to VGPRs (the VALU does
// the bit reads while the scalar unit runs the range decoder and the models)
GC_DI uint32_t vv(uint32_t x)
{
#if RIC_GC_UCOND >= 2
	asm volatile("" : "+v"(x));
#endif
	return x;
}
// RIC_GC_EFIFO: the encoder's raw-bit FIFO word in VGPRs (its shifts on the
// VALU; the bit count and every branch stay scalar).  Measured (r5 g6, one C3
// serving step of 3072 streams): 10955 against 11409 ms per launch (-4.0 %)
#ifndef RIC_GC_EFIFO
#define RIC_GC_EFIFO 1
#endif
GC_DI uint64_t vf(uint64_t x)
{
#if RIC_GC_EFIFO
	asm volatile("" : "+v"(x));
#endif
	return x;
}
GC_DI uint32_t ev(uint32_t x)
{
#if RIC_GC_EVALU
	asm volatile("" : "+v"(x));
#endif
	return x;
}
GC_DI uint32_t eu(uint32_t x)
{
#if RIC_GC_EVALU
	return __builtin_amdgcn_readfirstlane(x);
#else
	return x;
#endif
}
// RIC_GC_UCOND 4: 2 and the decoder's byte window in VGPRs (the raw-bit
// reader's fills on the VALU; the range decoder reads its bytes back by lane 0)
GC_DI uint64_t vw(uint64_t x)
{
#if RIC_GC_UCOND == 4
	asm volatile("" : "+v"(x));
#endif
	return x;
}
// RIC_GC_UCOND 3: the range decoder's state in VGPRs as well (its bin
// arithmetic on the VALU), the decoded bin read back from lane 0 for the
// models, which stay on the scalar unit
GC_DI uint32_t vr(uint32_t x)
{
#if RIC_GC_UCOND == 3
	asm volatile("" : "+v"(x));
#endif
	return x;
}
// a wave-uniform value kept in a VGPR (the compiler would give it an SGPR)
GC_DI uint32_t to_vgpr(uint32_t x) { uint32_t r; asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "s"(x)); return r; }
// RIC_GC_ECOLD: the encoder's cold fields (the output address, its capacity,
// the .ric header words) in VGPRs: they are read once per chunk or once per
// stream, and as SGPRs they pushed the walk's hot values into spill lanes.
// Measured (one C3 serving step of 3072 streams, two A/B pairs): 10948 / 10956
// against 11005 / 11019 ms per launch (-0.5 %)
#ifndef RIC_GC_ECOLD
#define RIC_GC_ECOLD 1
#endif
GC_DI uint32_t vc(uint32_t x)
{
#if RIC_GC_ECOLD
	asm volatile("" : "+v"(x));
#endif
	return x;
}
// RIC_GC_PCOLD: a band walk's per-band pointers and limits (the band, its
// records, the compacted value stream, the yield flag) in VGPRs: the lanes
// use them once per chunk of 64 blocks, and as SGPRs they stay live through
// the block loop, where the coder's hot scalars then spill.  Measured (one
// C3 serving step of 3072 streams, two A/B pairs): 10932 / 10915 against
// 10966 / 10929 ms per launch (SGPR spill slots 137 -> 108)
#ifndef RIC_GC_PCOLD
#define RIC_GC_PCOLD 1
#endif
template <typename T> GC_DI T* vcp(T* p)
{
#if RIC_GC_PCOLD
	uint64_t x = (uint64_t)p;
	asm volatile("" : "+v"(x));
	return (T*)x;
#else
	return p;
#endif
}
GC_DI uint32_t vcu(uint32_t x)
{
#if RIC_GC_PCOLD
	asm volatile("" : "+v"(x));
#endif
	return x;
}
// lane arrays: element i of a per-wave array held in lane i of a VGPR
GC_DI uint32_t lget(uint32_t a, uint32_t i) { return __builtin_amdgcn_readlane(a, i); }
GC_DI uint32_t lset(uint32_t a, uint32_t i, uint32_t x) { return lane_id() == i ? x : a; }

// ---------------------------------------------------------------- tables
// Per-lane constants of the models, built once per wave.
struct GTabs {
	uint32_t geo_ks;     // lane i < 25: kGeoK[i] | kGeoShift[i] << 8
	uint32_t geo_thr;    // lane s in 1..10: kGeoThres[s - 1] | kGeoThres[s] << 16
	uint32_t bit_thr;    // lane s in 0..9: kBitThres[s] | kBitThres[s + 1] << 16
	uint32_t e16;        // enumDecode<16> table: lane k in 1..8 its offset (sum of C(16, j), j < k), lane 16 + k C(16, k),
	                     // lane 32 + k CnkLen | CnkLost << 8 of (16, k) (the code part's lengths: enum16 needs no cnk[])
	GC_DI void init()
	{
		const uint32_t l = lane_id();
		{
			uint32_t c = 1, off = 0, ck = 0;                 // C(16, j) for j = 0, 1, ...
			for (uint32_t j = 1; j <= 8; j++) {
				c = c * (17 - j) / j;
				if (j == (l & 15)) ck = c;
				if (j < (l & 15)) off += c;
			}
			e16 = l < 16 ? off : ck;
			if (l >= 33 && l <= 40) e16 = (uint32_t)kCnkLen[15][l - 33] | (uint32_t)kCnkLost[15][l - 33] << 8;
		}
		geo_ks = l < 25 ? (uint32_t)kGeoK[l] | (uint32_t)kGeoShift[l] << 8 : 0;
		geo_thr = (l >= 1 && l <= 10) ? (uint32_t)kGeoThres[l - 1] | (uint32_t)kGeoThres[l] << 16 : 0;
		bit_thr = l <= 9 ? (uint32_t)kBitThres[l] | (uint32_t)kBitThres[l + 1] << 16 : 0;
	}
};

// Issue priority by progress (GEncArgs::prio).  The SIMDs pick among their
// waves by priority, then by age, so with equal priorities the oldest coder
// wave of a SIMD runs ahead and its waves finish one after another, the last
// ones alone on their SIMD (the slowest way to run them).  A wave lowers its
// priority as it advances -- encode up to the finest level's H band 3, the rest
// of the encode 2, then the decode 1 and 0 -- so the waves of a SIMD keep
// level with each other.
// prio 2 (the default) keeps the encode and the decode's coarse levels at 3
// and steps down at the decode's finest V, H and D bands (2, 1, 0): the last
// step, where the waves of a SIMD finish by age again, is the shortest.
template <int P> GC_DI void set_prio(int on) { if (on) __builtin_amdgcn_s_setprio(P); }
// the priority a wave takes at band b (of nb, coding order) of its last plane
GC_DI void prio_band(int mode, bool dec, int b, int nb)
{
	if (mode == 1) {                                   // encode 3 / 2, decode 1 / 0, stepping at the finest H band
		if (b == nb - 2) { if (dec) set_prio<0>(1); else set_prio<2>(1); }
	} else if (mode == 2 && dec) {
		if (b == nb - 3) set_prio<2>(1);
		else if (b == nb - 2) set_prio<1>(1);
		else if (b == nb - 1) set_prio<0>(1);
	} else if (mode == 3 && dec) {                     // 2 at H, 1 at D, 0 half-way through D (tree_dec)
		if (b == nb - 2) set_prio<2>(1);
		else if (b == nb - 1) set_prio<1>(1);
	}
}

// prio 4: by rank among the coder waves of the same SIMD.  Waves record
// their progress (chunks of 64 blocks coded, encode then decode) in a device
// table with one row per SIMD, one word per wave slot; at every chunk a wave
// reads its SIMD's row and takes priority 3 if no other coder wave of this
// launch on its SIMD is behind it, 2 if one is, 1 if two are, 0 beyond.  The
// wave furthest behind always issues first, so the waves of a SIMD finish
// together instead of one after another by age (modes 1-3 level them only at
// band steps: a C3 step's 3072 waves ended in three tiers, 9.25 / 10.0 /
// 10.9 s, the SIMDs holding two, then one wave for the last 1.7 s).
// Row = XCC_ID, SE, SH, CU, SIMD (13 bits), word = wave slot (4 bits); a word
// is tag << 20 | progress, the tag being the launch's (12 bits, top bit set),
// so words left by other launches are ignored and no reset is needed.
constexpr uint32_t kLevelRows = 1u << 13;
__device__ uint32_t g_level[kLevelRows * 16];
// mode 5: the same ranks one priority lower (2, 1, 0), below the level
// kernels' producer waves (priority 2) that run beside the coder
__shared__ uint32_t g_lv[3];          // progress, table word, tag << 20 | top priority (0: mode off)
GC_DI void level_init(int mode, uint32_t tag)
{
	if (mode != 4 && mode != 5) { g_lv[2] = 0; return; }
	const uint32_t hw = __builtin_amdgcn_s_getreg(0xF804), xcc = __builtin_amdgcn_s_getreg(0xF814);
	const uint32_t row = (xcc & 7u) << 10 | ((hw >> 13) & 7u) << 7 | ((hw >> 12) & 1u) << 6 | ((hw >> 8) & 15u) << 2 |
	                     ((hw >> 4) & 3u);
	g_lv[0] = 0;
	g_lv[1] = row << 4 | (hw & 15u);
	g_lv[2] = ((tag & 0x7FFu) | 0x800u) << 20 | (mode == 4 ? 3u : 2u);
}
// the table word of this wave posted (its progress advanced by a chunk) and
// its SIMD's row loaded: the row is used at the next chunk (level_apply), so
// the load's round trip overlaps the chunk's coding
GC_DI uint32_t level_post()
{
	const uint32_t tw = g_lv[2], tg = tw & 0xFFF00000u;
	if (!tw) return 0u;
	const uint32_t p = (g_lv[0] + 1) & 0xFFFFFu;
	const uint32_t me = g_lv[1], l = lane_id();
	g_lv[0] = p;
	if (l == 0) __hip_atomic_store(g_level + me, tg | p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	uint32_t v = 0;
	if (l < 16 && l != (me & 15u)) v = __hip_atomic_load(g_level + (me & ~15u) + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	return v;
}
// the priority from the row loaded at the last level_post, against the
// progress posted with it
GC_DI void level_apply(uint32_t v)
{
	const uint32_t tw = g_lv[2], tg = tw & 0xFFF00000u;
	if (!tw) return;
	const uint32_t p = g_lv[0];
	const uint32_t behind = (uint32_t)__builtin_popcountll(__ballot((v & 0xFFF00000u) == tg && (v & 0xFFFFFu) < p));
	const int pr = (int)(tw & 3u) - (int)behind;
	if (pr >= 3) __builtin_amdgcn_s_setprio(3);
	else if (pr == 2) __builtin_amdgcn_s_setprio(2);
	else if (pr == 1) __builtin_amdgcn_s_setprio(1);
	else __builtin_amdgcn_s_setprio(0);
}
GC_DI void level_step(bool last = false)
{
	const uint32_t tw = g_lv[2], tg = tw & 0xFFF00000u;
	if (!tw) return;
	const uint32_t p = last ? 0xFFFFFu : (g_lv[0] + 1) & 0xFFFFFu;
	const uint32_t me = g_lv[1], l = lane_id();
	g_lv[0] = p;
	if (l == 0) __hip_atomic_store(g_level + me, tg | p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	if (last) return;
	uint32_t v = 0;
	if (l < 16 && l != (me & 15u)) v = __hip_atomic_load(g_level + (me & ~15u) + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	const uint32_t behind = (uint32_t)__builtin_popcountll(__ballot((v & 0xFFF00000u) == tg && (v & 0xFFFFFu) < p));
	const int pr = (int)(tw & 3u) - (int)behind;
	if (pr >= 3) __builtin_amdgcn_s_setprio(3);
	else if (pr == 2) __builtin_amdgcn_s_setprio(2);
	else if (pr == 1) __builtin_amdgcn_s_setprio(1);
	else __builtin_amdgcn_s_setprio(0);
}

// Yielding to the level kernels (GEncArgs::yield): while the batch stream
// runs the host-coded frames' level kernels it raises a flag in device memory;
// a coder wave that finds it raised at a chunk boundary sleeps (at most ~0.25
// ms per check, so a flag left raised only slows the coder), leaving the CU's
// issue slots to the level kernel's waves.
// RIC_GC_YCHK: blocks between two checks of the yield flag (a power of two
// <= 64; 64: once per chunk)
#ifndef RIC_GC_YCHK
#define RIC_GC_YCHK 64
#endif
GC_DI void coder_yield(const uint32_t* flag)
{
	if (!flag) return;
	for (int n = 0; n < 64 && __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); n++)
		__builtin_amdgcn_s_sleep(127);
}

// A band walk's per-chunk synchronisation -- the yield flag and the level
// table -- loaded one chunk ahead (RIC_GC_SYNC_AHEAD, default on): the loads
// issued at chunk c are consumed at chunk c + 1, so their round trip overlaps
// the chunk's coding instead of stalling the wave at every chunk start.  A
// flag seen raised is then polled until it falls (coder_yield).
#ifndef RIC_GC_SYNC_AHEAD
#define RIC_GC_SYNC_AHEAD 1
#endif
struct ChunkSync {
	uint32_t yv = 0, lv = 0;
	bool have = false;
	GC_DI void step(const uint32_t* yield)
	{
#if RIC_GC_SYNC_AHEAD
		if (have) {
			if (yv) coder_yield(yield);
			level_apply(lv);
		}
		yv = yield ? __hip_atomic_load(yield, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
		lv = level_post();
		have = true;
#else
		coder_yield(yield);
		level_step();
#endif
	}
};

// diagnostics (GEncArgs::ts): the wave's start and end (s_memrealtime, 100
// MHz), and where it ran: HW_ID (wave, SIMD, CU, SE) | XCC_ID << 32
GC_DI void ts_put(uint64_t* ts, int f, uint64_t t_start)
{
	const uint64_t hw = (uint64_t)__builtin_amdgcn_s_getreg(0xF804) | (uint64_t)__builtin_amdgcn_s_getreg(0xF814) << 32;
	GAS uint64_t* o = gst(ts) + 4 * (size_t)f;
	o[0] = t_start;
	o[1] = __builtin_amdgcn_s_memrealtime();
	o[2] = hw;
}

// ------------------------------------------------------------ the encoder
// Coded bytes go to a ring in LDS and leave for HBM in 1 KiB pieces (all 64
// lanes, 16-byte stores) once no reservation slot points into them: single
// byte stores would each hold the vector-memory counter the walk's prefetch
// loads are waited on with.
// Two ring sizes, one kernel each: 8 KiB for lossless streams (a chunk of 64
// blocks of wide int coefficients can write ~4 KiB), 4 KiB for lossy ones,
// whose chunks write well under 3 KiB: a 4 KiB ring keeps the wave's LDS at
// ~9 KiB like the decoder's, so the level kernels still fit beside many
// coder waves on a CU.  A chunk that overruns its ring is flagged either way.
constexpr uint32_t kFlush = 1024;
__shared__ __attribute__((aligned(16))) uint8_t g_ring8[8192];
__shared__ __attribute__((aligned(16))) uint8_t g_ring4[4096];
template <uint32_t R> GC_DI uint8_t* ring_base();
template <> GC_DI uint8_t* ring_base<8192>() { return g_ring8; }
template <> GC_DI uint8_t* ring_base<4096>() { return g_ring4; }
__shared__ uint16_t g_huff[16 * 16 + 17 * 17];  // kHuff_HIGH rows, then kHuff_LOW rows
__shared__ uint32_t g_coef[64 * 16];             // the current chunk's coefficients, 16 per block

// CMuxCodec encoder state.  Byte positions are offsets from `out`; the four
// reservation slots of the carry-less coder (last[], muxcodec.cpp:63-74) are a
// FIFO q0..q3: normalize_enc writes the front one and appends p.
template <uint32_t kRing>
struct GEnc {
	uint32_t out_lo, out_hi;         // the stream's address (vc)
	uint32_t cap;                    // (vc)
	uint32_t range, low, ebits;
	uint64_t ebuf;
	uint32_t p, reserved;            // reserved == 0: none (offset 0 is never a slot)
	uint32_t q0, q1, q2, q3;
	uint32_t ovf;                    // 1: past cap, 2: ring overrun
	uint32_t flushed;                // bytes [0, flushed) are in HBM
	uint32_t hdr0, hdr1, hdr2;       // the 9-byte .ric header (ric.cpp:142-152)

	// every lane writes the same byte (no exec-mask change per byte); the
	// capacity is checked where bytes leave the ring (maybe_flush / end)
	GC_DI void put(uint32_t slot, uint32_t v) { ring_base<kRing>()[slot & (kRing - 1)] = (uint8_t)v; }
	// copy ring bytes [flushed, upto) (upto a multiple of 16, or the end) to HBM
	GC_DI void flush_to(uint32_t upto)
	{
		if (flushed == 0 && upto > 0) {
			// the header overwrites the coder's two leading bytes (out + 7, + 8)
			if (lane_id() == 0) {
				uint32_t* r = (uint32_t*)ring_base<kRing>();
				r[0] = hdr0; r[1] = hdr1;
				ring_base<kRing>()[8] = (uint8_t)hdr2;
			}
		}
		const uint32_t l = lane_id();
		uint8_t* out = (uint8_t*)(((uint64_t)out_hi << 32) | out_lo);
		for (uint32_t b = flushed; b < upto; b += 64 * 16) {
			const uint32_t o = b + l * 16;
			if (o < upto && o + 16 <= cap) {
				const u32x4 v = *(const u32x4*)(ring_base<kRing>() + (o & (kRing - 1)));
				*gst((u32x4*)(out + o)) = v;
			}
		}
		flushed = upto;
	}
	// Called between chunks of blocks (never inside the block walk: a vector
	// store in that loop makes the compiler drain every load in flight before
	// it).  The ring must have held every byte since the last call: a chunk
	// that wrote more than the ring holds (a pathological stream) is flagged.
	GC_DI void maybe_flush()
	{
		if (p - flushed > kRing - 64) ovf |= 2;
		if (p > cap) ovf |= 1;
		uint32_t lw = reserved ? (reserved < q0 ? reserved : q0) : q0;
		if (lw - flushed >= kFlush) {
			lw &= ~(kFlush - 1);
			flush_to(lw);
		}
	}
	GC_DI void raw_byte(uint32_t b)
	{
		const uint32_t slot = reserved ? reserved : p;
		p += reserved ? 0u : 1u;
		reserved = 0;
		put(slot, b);
	}
	GC_DI void drain()                                   // emptyBuffer, muxcodec.cpp:536-548
	{
#pragma clang loop vectorize(disable) unroll(disable)
		while (ebits >= 8) {
			ebits -= 8;
			raw_byte((uint32_t)(ebuf >> ebits) & 255u);
		}
	}
	GC_DI void norm()                                    // normalize_enc, muxcodec.cpp:63-74
	{
		drain();                                         // flushBuffer<false>: complete bytes,
		if (ebits > 0 && !reserved) reserved = p++;      // then reserve the partial one
		uint32_t it = 0;
		do {
			put(q0, low >> 24);
#if RIC_GC_ELOW_V
			range = __builtin_amdgcn_readfirstlane(((low + range - 1) ^ low) >= 0x01000000u ? (0u - low) & 4095u : range);
#elif RIC_GC_EVALU
			range = ev(((low + range - 1) ^ low) >= 0x01000000u ? (0u - low) & 4095u : range);
#else
			if (((low + range - 1) ^ low) >= 0x01000000u) range = (0u - low) & 4095u;
#endif
			q0 = q1; q1 = q2; q2 = q3; q3 = p++;
			range = ev(range << 8);
			low = ev(low << 8);
			// a zero range would spin here forever (never on a valid stream;
			// a wave that never ends takes the whole GPU down): stop and flag
			if (__builtin_expect(++it > 4, 0)) { ovf |= 4; range = ev(1u << 16); }
		} while (eu(range) <= 4096u);
	}
	GC_DI void bin(uint32_t freq, uint32_t bit)         // codeBin, muxcodec.h:156-163
	{
		if (__builtin_expect(eu(range) <= 4096u, 0)) norm();
		const uint32_t t = (range * freq) >> 12;
		low = ev(low + (t & (0u - bit)));
		range = ev(t + ((range - 2 * t) & (0u - bit)));
	}
	GC_DI void bits(uint32_t v, uint32_t len)           // bitsCode, 64-bit FIFO (entropy.h)
	{
		if (__builtin_expect(ebits + len > 64, 0)) drain();
		ebuf = vf((ebuf << len) | v);
		ebits += len;
	}
	GC_DI void init(uint8_t* o, uint32_t c, uint32_t base)   // init_encoder at out + base
	{
		out_lo = vc((uint32_t)(uintptr_t)o); out_hi = vc((uint32_t)((uintptr_t)o >> 32)); cap = vc(c);
#if RIC_GC_ELOW_V || RIC_GC_EVALU
		low = to_vgpr(0u);                               // (experiment: the coder's low on the VALU)
#else
		low = 0;
#endif
		range = ev(1u << 16);
		ebits = 0; ebuf = 0;
		reserved = 0;
		q0 = base; q1 = base + 1; q2 = base + 2; q3 = base + 3;
		p = base + 4;
		ovf = c < base + 4 ? 1u : 0u;
		flushed = 0;
	}
	GC_DI uint32_t end()                                 // endCoding, muxcodec.cpp:87-106
	{
		drain();
		if (ebits > 0) {                                 // flushBuffer<true>: the last partial byte
			raw_byte((uint32_t)(ebuf << (8 - ebits)) & 255u);
			ebits = 0;
		}
		if (range <= 4096u) norm();
		const uint32_t last_out = 0x200 | 'W';
		if ((low & 4095u) > (last_out & 4095u)) low += 4096u;
		low = (low & ~4095u) | (last_out & 4095u);
		put(q0, low >> 24);
		put(q1, (low >> 16) & 255u);
		put(q2, (low >> 8) & 255u);
		put(q3, low & 255u);
		if (p > cap) ovf |= 1;
		if (!ovf) flush_to((p + 15) & ~15u);
		return p;
	}
};

// CBitCodec (16 contexts): lane c = freq | shift << 16 | mps << 24
struct GBit {
	uint32_t st;
	GC_DI void init() { st = 2048u; }
	template <typename E>
	GC_DI void code(E& e, const GTabs& T, uint32_t sym, uint32_t c)   // bitcodec.h:52-60, 81-92
	{
		const uint32_t v = lget(st, c);
		uint32_t freq = v & 0xFFFFu, sh = (v >> 16) & 0xFFu, mps = v >> 24;
		const uint32_t s = sym ^ mps;
		e.bin(freq, s ^ 1);
		freq = (freq + (s << (9 - sh)) - (freq >> (3 + sh))) & 0xFFFFu;
		const uint32_t th = lget(T.bit_thr, sh), t0 = th & 0xFFFFu, t1 = th >> 16;
		if (__builtin_expect(((freq - t1) & 0xFFFFu) > t0 - t1, 0)) {
			if (freq > t0) {
				if (sh == 0) { mps ^= 1; freq = 4096u - freq; sh = 1; }
				else sh--;
			} else if (sh < 9) sh++;
		}
		st = lset(st, c, freq | sh << 16 | mps << 24);
	}
};

// One CGeomCodec context in scalars (geomcodec.h:41-57, 88-97): freq, idx.
// The idx-dependent parameters (k, shift, the shift's thresholds) are read
// from the lane tables when the context is loaded and again only when idx
// moves, not per coded value.
// The idx-dependent values the per-value step uses are kept ready-made: the
// adaptation shift 3 + s, the low threshold t0 and the span t1 - t0 of the
// re-index test, so that test costs one subtract, mask and compare per value.
struct GGeoCtx {
	uint32_t freq, idx, k, s3, t0, span, k1, km;
	GC_DI void params(const GTabs& T)
	{
		const uint32_t ks = lget(T.geo_ks, idx), s = ks >> 8;
		const uint32_t thr = lget(T.geo_thr, s);
		k = ks & 0xFFu; s3 = s + 3; t0 = thr & 0xFFFFu; span = (thr >> 16) - t0;
		k1 = k + 1; km = (1u << k) - 1u;
	}
	GC_DI void load(uint32_t arr, uint32_t c, const GTabs& T) { const uint32_t v = lget(arr, c); freq = v & 0xFFFFu; idx = v >> 16; params(T); }
	GC_DI uint32_t packed() const { return freq | idx << 16; }
	// magnitude - 1 (unary + k raw bits) then, if SIGNED, one raw sign bit:
	// the remainder and the sign as one chunk
	template <bool SIGNED, typename E>
	GC_DI void code(E& e, const GTabs& T, uint32_t sym, uint32_t sign)
	{
		const uint32_t f = freq;
		uint32_t fr = freq;
		const uint32_t run = sym >> k;
		if (__builtin_expect(run != 0, 0)) {             // most runs are empty: fall through
			if (__builtin_expect(run > (1u << 20), 0)) e.ovf |= 4;   // not a coefficient of this path
			else
				for (uint32_t l = run; l > 0; l--) {
					e.bin(f, 1);
					fr -= fr >> s3;
				}
		}
		e.bin(f, 0);
#if RIC_GC_GEOFAST
		if (SIGNED) e.bits(((sym & km) << 1) | sign, k1);
		else if (k > 0) e.bits(sym & km, k);
		fr = fr + ((4096u - fr) >> s3);
		if (__builtin_expect(fr - t0 > span, 0)) {
#else
		if (SIGNED) e.bits(((sym & ((1u << k) - 1)) << 1) | sign, k + 1);
		else if (k > 0) e.bits(sym & ((1u << k) - 1), k);
		fr = (fr + ((4096u - fr) >> s3)) & 0xFFFFu;
		if (__builtin_expect(((fr - t0) & 0xFFFFu) > span, 0)) {
#endif
			if (fr < t0) { if (idx < 24) idx++; }
			else if (idx > 0) idx--;
			if (idx >= 9) fr = 2048;
			params(T);
		}
		freq = fr;
	}
};

GC_DI uint32_t geo_init_lane(const uint8_t* kinit)          // setCtx, geomcodec.cpp:31-41
{
	const uint32_t c = lane_id() & 15;
	const uint32_t idx = kinit[c];
	const uint32_t f = idx >= 9 ? 2048u : (uint32_t)((kGeoThres[idx - 1] + kGeoThres[idx]) >> 1);
	return f | idx << 16;
}

// taboo code, n = 2 (initTaboo / tabooCode, muxcodec.cpp:113-129, 210-240):
// nb[] is the Fibonacci run 1, 1, 2, 3, ...; sum[] its prefix sums.
GC_DI void taboo_lanes(uint32_t& nbl, uint32_t& suml)   // lane i < 32: nb[i], sum[i]
{
	const uint32_t l = lane_id();
	uint32_t fa = 1, fb = 1, sm = 0;
	for (uint32_t i = 0; i < 32; i++) {
		const uint32_t cur = i < 2 ? 1u : fa + fb;
		if (i >= 2) { fa = fb; fb = cur; }
		sm += cur;
		if (i == l) break;
	}
	nbl = l < 2 ? 1u : fb;
	suml = sm;
}
template <typename E>
GC_DI void taboo_code(E& e, uint32_t nbv)
{
	uint32_t nbl, suml;
	taboo_lanes(nbl, suml);
	const uint32_t nt = 2;
	int i = 0, len;
	uint32_t r = 0, nb = nbv;
	while (lget(suml, (uint32_t)i) <= nb) i++;
	if (i == 0) { e.bits(0, nt); return; }
	len = i; i--;
	nb -= lget(suml, (uint32_t)i);
	while (i > (int)nt) {
		const uint32_t k = (uint32_t)i - nt + 1;
		uint32_t cnt = lget(nbl, k), j = 0;
		while (nb >= cnt) { j++; cnt += lget(nbl, k + j); }
		nb -= cnt - lget(nbl, k + j);
		j = nt - j;
		r = (r << j) | 1;
		i -= (int)j;
	}
	if (i == (int)nt) nb++;
	r = ((((r << i) | (nb & ((1u << i) - 1))) << 1) | 1) << nt;
	e.bits(r, (uint32_t)len + nt);
}

// CBandCodec::pred<encode> (LL DPCM), bandcodec.cpp:62-104.  The residuals and
// contexts of a 64-coefficient run of a row are computed by the lanes; the
// scalar walk codes them in order.
template <typename C, typename E>
GC_DI void pred_enc(E& e, const GTabs& T, const GBandDesc& B, const char* arena)
{
	static constexpr uint8_t ginit[16] = {9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,15};
	const GAS C* c = gld((const C*)(arena + B.off));
	const long st = B.pitch;
	const int dx = B.dx, dy = B.dy;
	uint32_t geo = geo_init_lane(ginit);
	const uint32_t l = lane_id();
	for (int j = 0; j < dy; j++) {
		const GAS C* row = c + (long)j * st;
		for (int x0 = 0; x0 < dx; x0 += 64) {
			const int i = x0 + (int)l;
			uint32_t sym = 0, ctx = 15;
			if (i < dx) {
				const int cur = row[i];
				if (j == 0) {
					sym = i == 0 ? (uint32_t)s2u(cur) : (uint32_t)s2u(cur - row[i - 1]);
				} else if (i == 0) {
					sym = (uint32_t)s2u(cur - row[-st]);
				} else {
					const int w = row[i - 1], n = row[i - st], nw = row[i - 1 - st];
					const int a = w - nw, bb = n - nw;
					int var = bitlen((uint32_t)((a < 0 ? -a : a) + (bb < 0 ? -bb : bb)));
					if (var > 15) var = 15;
					ctx = (uint32_t)var;
					sym = (uint32_t)s2u(cur - w - n + nw);
				}
			}
			const int nx = dx - x0 < 64 ? dx - x0 : 64;
			for (int q = 0; q < nx; q++) {
				const uint32_t s = lget(sym, (uint32_t)q);
				if (j == 0 && x0 + q == 0) { taboo_code(e, s); continue; }
				const uint32_t cx = lget(ctx, (uint32_t)q);
				GGeoCtx g;
				g.load(geo, cx, T);
				g.code<false>(e, T, s, 0);
				geo = lset(geo, cx, g.packed());
			}
			e.maybe_flush();
		}
	}
}

// The lanes' fetch of one group of 4 blocks (scan positions s0..s0+3): lane
// 16 j + i gets coefficient i of block j, i in the block's own raster order
// over its w x h corner (the record's mask bits).  One aligned dword load per
// lane whatever the band type (no type-divergent loads into one register): a
// short band's value is the half selected by bit g of *half, taken when the
// chunk is staged (unpack_coef).
GC_DI uint32_t fetch_group(const char* band, int is_int, long st, int dx, int dy, int nblk, int s0, int g,
                           uint32_t& half)
{
	const int l = (int)lane_id();
	const int s = s0 + (l >> 4), i = l & 15;
	uint32_t v = 0;
	if (s < nblk) {
		int bx, by;
		scan_block(s, dx, dy, bx, by);
		const int w = dx - bx * 4 < 4 ? dx - bx * 4 : 4, h = dy - by * 4 < 4 ? dy - by * 4 : 4;
		if (i < w * h) {
			const int r = w == 4 ? i >> 2 : i / w, q = i - r * w;
			const long e = (long)(by * 4 + r) * st + bx * 4 + q;
			const long byte = is_int ? e * 4 : e * 2;
			v = *gld((const uint32_t*)(band + (byte & ~3l)));
			half |= (uint32_t)((byte >> 1) & 1) << g;
		}
	}
	return v;
}
GC_DI uint32_t unpack_coef(uint32_t v, int is_int, uint32_t half, int g)
{
	return is_int ? v : (v >> (((half >> g) & 1) * 16)) & 0xFFFFu;
}

// The lanes' fetch of the records of scan positions s0..s0+63.
struct RecChunk {
	uint32_t lo, hi, pin;
};
GC_DI RecChunk fetch_recs(const uint64_t* rec, const uint8_t* pin, int dx, int dy, int nblk, int s0)
{
	const int s = s0 + (int)lane_id();
	RecChunk r{0, 0, 0};
	if (s < nblk) {
		int bx, by;
		scan_block(s, dx, dy, bx, by);
		const long k = (long)by * ((dx + 3) >> 2) + bx;
		const uint64_t v = gld(rec)[k];
		r.lo = (uint32_t)v; r.hi = (uint32_t)(v >> 32);
		r.pin = pin ? gld(pin)[k] : 0u;
	}
	return r;
}

// The coefficients of one block: unary + raw remainder + sign each, one
// geometric context (CGeomCodec::code, geomcodec.h:41-57; block_enum's
// coefficient loop, bandcodec.cpp:392-401).
// rank: lane k of cv holds the k-th coefficient of the mask (a compacted
// pool's value stream), else lane i the coefficient at bit i
template <typename E>
GC_DI void code_coefs(E& e, const GTabs& T, uint32_t& geo, uint32_t gc, uint32_t mask, uint32_t cv, uint32_t cb,
                      bool rank = false)
{
	GGeoCtx g;
	g.load(geo, gc, T);
	uint32_t k = 0;
	while (mask) {
		const uint32_t i = (uint32_t)__builtin_ctz(mask);
		mask &= mask - 1;
		const uint32_t u = lget(cv, rank ? k++ : cb + i);
		g.code<true>(e, T, (u >> 1) - 1, u & 1);
	}
	geo = lset(geo, gc, g.packed());
}

// lane-exclusive prefix sum over the wave of popcount(m) (m: 16 bits), and
// the total: per bit, a ballot and the lane's count of lower lanes that have it
// (mbcnt) -- a few registers, no shuffles
GC_DI uint32_t wave_excl_popc(uint32_t m, uint32_t& total)
{
	uint32_t o = 0, t = 0;
	RIC_UNROLL
	for (int b = 0; b < 16; b++) {
		const uint64_t bb = __ballot((m >> b) & 1u);
		o += __builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u));
		t += (uint32_t)__builtin_popcountll(bb);
	}
	total = t;
	return o;
}

// a compacted pool's value stream: the 64 lanes' loads of values v0 .. v0 +
// 1023 (zero-extended, as unpack_coef gives a short band's value), none at
// or past vcap
GC_DI void fetch_cvals(const int16_t* cv, uint32_t v0, uint32_t vcap, uint32_t (&cn)[16])
{
	const uint32_t l = lane_id();
	RIC_UNROLL
	for (int g = 0; g < 16; g++) {
		const uint32_t i = v0 + (uint32_t)g * 64 + l;
		cn[g] = i < vcap ? (uint32_t)(uint16_t)gld(cv)[i] : 0u;
	}
}

// CBandCodec::tree<encode> over the GPU block records (encoder.cpp
// tree_rec_fast; bandcodec.cpp:484-589 with block_enum :346-478).  high: the
// finest level (HIGH tables); par: the band has a parent level.
// cvals (a compacted pool's band, B.cmp): the plane's value stream, vrun the
// band's first value (advanced past the band's values on return)
template <typename E>
GC_DI void tree_enc(E& e, const GTabs& T, const GBandDesc& B, const char* arena, const uint32_t* yield,
                    const int16_t* cvals = nullptr, uint32_t vcap = 0, uint32_t* vrun = nullptr)
{
	const bool high = B.high, par = B.has_pin;
	const uint64_t* rec = vcp((const uint64_t*)(arena + B.rec_off));
	const uint8_t* pin = par ? vcp((const uint8_t*)(arena + B.pin_off)) : nullptr;
	const char* band = vcp(arena + B.off);
	yield = vcp(yield);
	const int is_int = B.is_int;
	const long st = B.pitch;
	const int dx = B.dx, dy = B.dy;
	const int nblk = ((dx + 3) >> 2) * ((dy + 3) >> 2);
	const uint32_t l = lane_id();
	// CGeomCodec init {5,9,9,...,10,10,10,11} (bandcodec.cpp:487)
	const uint32_t gidx = l == 0 ? 5u : (l < 12 ? 9u : (l < 15 ? 10u : 11u));
	uint32_t geo = (gidx >= 9 ? 2048u : (uint32_t)((kGeoThres[gidx - 1] + kGeoThres[gidx]) >> 1)) | gidx << 16;
	GBit tree, bord;
	tree.init(); bord.init();
	// k_mean init 2,3,4,5,8,11,13,14,15,... << 10 (bandcodec.cpp:488-489)
	uint32_t kmean = l < 8 ? (uint32_t)((l < 4 ? l + 2 : (l == 4 ? 8 : (l == 5 ? 11 : (l == 6 ? 13 : 14)))) << 10)
	                       : 15u << 10;
	const uint32_t hbase = high ? 0u : 256u, hrow = high ? 16u : 17u;
	const uint32_t hoff = high ? 0xFFFFFFFFu : 0u;      // HIGH tables index k - 1
	// Chunks of 64 blocks in scan order.  The loads of chunk c + 1 (records,
	// 16 groups of 4 blocks' coefficients) are issued when chunk c starts and
	// consumed a whole chunk later, in one wait; chunk c's coefficients then
	// sit in LDS (g_coef), one 16-lane row per block.
	// A compacted band (cvals): chunk c's values are the stream's next n_c (the
	// popcounts of its blocks' record masks, propagated blocks included, as
	// k_cmp_write lays them out); the 1024 values from chunk c + 1's first are
	// loaded when chunk c starts, block j's at g_coef[boff_j ..].
	const bool cmp = cvals != nullptr;
	if (cmp) { cvals = vcp(cvals); vcap = vcu(vcap); }
	uint32_t vpos = cmp ? *vrun : 0u, boff = 0;
	RecChunk rn = fetch_recs(rec, pin, dx, dy, nblk, 0);
	uint32_t cn[16], half = 0;
	if (cmp) fetch_cvals(cvals, vpos, vcap, cn);
	else {
		RIC_UNROLL
		for (int g = 0; g < 16; g++) cn[g] = fetch_group(band, is_int, st, dx, dy, nblk, 4 * g, g, half);
	}
	ChunkSync cs;
	for (int s0 = 0; s0 < nblk; s0 += 64) {
		cs.step(yield);
		const RecChunk rc = rn;
		RIC_UNROLL
		for (int g = 0; g < 16; g++) g_coef[g * 64 + l] = cmp ? cn[g] : unpack_coef(cn[g], is_int, half, g);
		if (cmp) {
			uint32_t nc;
			boff = wave_excl_popc(BlockRec::mask((uint64_t)rc.lo | (uint64_t)rc.hi << 32), nc);
			vpos += nc;
		}
		if (s0 + 64 < nblk) {
			rn = fetch_recs(rec, pin, dx, dy, nblk, s0 + 64);
			half = 0;
			if (cmp) fetch_cvals(cvals, vpos, vcap, cn);
			else {
				RIC_UNROLL
				for (int g = 0; g < 16; g++) cn[g] = fetch_group(band, is_int, st, dx, dy, nblk, s0 + 64 + 4 * g, g, half);
			}
		}
		const int nj = nblk - s0 < 64 ? nblk - s0 : 64;
		for (int j = 0; j < nj; j++) {
			if (RIC_GC_YCHK < 64 && j && !(j & (RIC_GC_YCHK - 1))) coder_yield(yield);
			const uint32_t li = (uint32_t)j;
			const uint64_t r = (uint64_t)lget(rc.lo, li) | (uint64_t)lget(rc.hi, li) << 32;
			const uint32_t ins = BlockRec::insig(r);
			const uint32_t mask = BlockRec::mask(r);
			if (BlockRec::edge(r)) {
				bord.code(e, T, ins, 0);
				if (ins) continue;
				e.bits(BlockRec::raw(r), BlockRec::rawlen(r));
				const uint32_t cv = g_coef[(cmp ? lget(boff, li) : (uint32_t)j * 16) + (l & 15)];
				code_coefs(e, T, geo, BlockRec::gctx(r), mask, cv, 0, cmp);
			} else {
				uint32_t ctx = 15;
				if (par) {
					const uint32_t pi = lget(rc.pin, li);
					if (BlockRec::pin_prop(pi)) continue;
					ctx = BlockRec::pin_ctx(pi);
				}
				tree.code(e, T, ins, ctx);
				if (ins) continue;
				const uint32_t cv = g_coef[(cmp ? lget(boff, li) : (uint32_t)j * 16) + (l & 15)];
				const uint32_t k = BlockRec::k(r);
				const uint32_t km = lget(kmean, ctx);
				const uint32_t idx = (km + (1u << 9)) >> 10;
				const uint32_t h = g_huff[hbase + idx * hrow + k + hoff];
				const uint32_t rl = BlockRec::rawlen(r);
				e.bits(((h >> 5) << rl) | BlockRec::raw(r), (h & 31) + rl);
				code_coefs(e, T, geo, k - 1, mask, cv, 0, cmp);
				const uint32_t kk = high ? k - 1 : k;
				kmean = lset(kmean, ctx, (km + (kk << 7) - (km >> 3)) & 0xFFFFu);
			}
		}
		e.maybe_flush();
	}
	if (cmp) *vrun = vpos;
}

// One frame's stream per workgroup (one wave): the reference's CompressImage
// coding order (src/ric/ric.cpp:157-176 -> CWavelet2D::CodeBand,
// src/lib/wavelet2d.cpp:150-177): the coarsest LL, then every level coarse to
// fine, V, H, D.  The .ric file goes to out + f * ostride: the 9-byte header
// (ric.cpp:142-152) then the payload; the coder buffer starts at out + 7 and
// the header overwrites its two dropped leading bytes (as ric_codec).
GC_DI void load_huff()
{
	for (int i = (int)threadIdx.x; i < 16 * 16 + 17 * 17; i += 64)
		g_huff[i] = i < 256 ? kHuff_HIGH[i >> 4][i & 15] : kHuff_LOW[(i - 256) / 17][(i - 256) % 17];
	__syncthreads();
}

// frame f's whole stream; *end: the coder's end offset (file length 9 + end -
// 9), the status: 0 ok, 1 capacity, 2 a fused level kernel's ring timeout, 3
// the LDS ring overran / a guard, 4 the frame's level-0 values exceed a
// compacted pool's capacity (nothing coded: the caller codes it elsewhere)
template <uint32_t RING>
GC_DI uint32_t enc_frame(const GEncArgs& a, int f, uint32_t& end_out)
{
	const char* arena = a.arena + (size_t)f * a.astride;
	uint8_t* out = a.out + (size_t)f * a.ostride;
	int32_t status = 0;
	for (int p = 0; p < a.nplanes; p++) status |= *gld((const int32_t*)(arena + p * a.pstride + a.status_off));
	status = __builtin_amdgcn_readfirstlane(status);
	// not coded: over a compacted pool's capacity, or its compaction gave up
	// (kCmpOverCap, kCmpLookback): the host takes the frame
	if (status & (4 | 8)) { end_out = 0; return 4; }
	GTabs T;
	T.init();
	GEnc<RING> e;
	e.init(out, (uint32_t)a.cap, 7);
	e.hdr0 = vc('R' | 'U' << 8 | 'D' << 16 | (uint32_t)'2' << 24);
	e.hdr1 = vc((uint32_t)(a.w & 0xFFFF) | (uint32_t)(a.h & 0xFFFF) << 16);
	e.hdr2 = vc((uint32_t)((a.q & 31) | ((a.nplanes == 3) << 5) | ((a.trans & 3) << 6)));
	for (int p = 0; p < a.nplanes; p++) {               // Y, Co, Cg into the one stream (ric.cpp:157-176)
		const char* pa = arena + p * a.pstride;
		if (a.ll.is_int) pred_enc<int32_t>(e, T, a.ll, pa);
		else pred_enc<int16_t>(e, T, a.ll, pa);
		const int16_t* cvals = a.cmp_rel ? (const int16_t*)(pa + a.cmp_rel + a.cvals_off) : nullptr;
		uint32_t vrun = 0;                               // the compacted bands' running value index
		for (int b = 0; b < a.nb; b++) {
			if (p + 1 == a.nplanes) prio_band(a.prio, false, b, a.nb);
			if (a.b[b].cmp && cvals) tree_enc(e, T, a.b[b], pa, a.yield, cvals, a.cvcap, &vrun);
			else tree_enc(e, T, a.b[b], pa, a.yield);
		}
	}
	const uint32_t end = e.end();
	uint32_t rc = 0;
	if (status) rc = 2;                                  // a fused kernel's ring timeout
	else if (e.ovf & 6) rc = 3;                          // the LDS ring overran (pathological stream) / guard
	else if (e.ovf) rc = 1;
	end_out = end;
	return rc;
}

// The posted result of frame f (host-visible memory the caller polls while
// the launch runs): posted[2 f] = the coder's end offset, posted[2 f + 1] =
// status | 0x100 | tag << 12.  The tag is the launch's (a 20-bit counter the
// caller keeps): a word left from an earlier launch over the same frames never
// carries it, so the caller needs no reset between launches.  The stream's
// stores reach memory (system scope: the host's copy engine reads it) before
// the words that announce it.
GC_DI void post_result(uint32_t* posted, uint32_t tag, int f, uint32_t rc, uint32_t end)
{
	if (!posted) return;
	__threadfence_system();
	if (lane_id() == 0) {
		__hip_atomic_store(posted + 2 * f, rc ? 0u : end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		__hip_atomic_store(posted + 2 * f + 1, rc | 0x100u | tag << 12, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
	}
}

template <uint32_t RING>
__global__ void __launch_bounds__(64) GC_KATTR k_gc_encode(const GEncArgs* __restrict__ ap, uint32_t* posted, uint32_t tag)
{
	const GEncArgs& a = *ap;
	const int f = blockIdx.x;
	const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
	set_prio<3>(a.prio);
	level_init(a.prio, tag);
	load_huff();
	uint32_t end;
	const uint32_t rc = enc_frame<RING>(a, f, end);
	level_step(true);
	if (lane_id() == 0) {
		gst(a.res)[2 * f] = rc ? 0u : end;               // file length = 9 + (end - 7) - 2
		gst(a.res)[2 * f + 1] = rc;
		if (a.ts) ts_put(a.ts, f, t_start);
	}
	post_result(posted, tag, f, rc, end);
}


// ============================================================ the decoder
// CMuxCodec decoder over a .ric file in HBM.  The reference decodes from a
// copy of the payload with two zero bytes in front and zero padding behind
// (src/ric/ric.cpp:203-205): virtual byte x is 0 for x < 2 or x >= 2 + n, else
// file byte x + 7.  The file is staged into an LDS ring ahead of the walk
// (1 KiB per 64-lane load, refilled between chunks of blocks); a chunk that
// reads past what was staged (a pathological stream) is flagged.
constexpr uint32_t kDRing = 4096;
constexpr uint32_t kDAhead = 2048;     // bytes staged past the read position at each refill
constexpr uint32_t kDMargin = 512;     // staged bytes kept ahead of a block / a unary run's bin
// The decoder's LDS is the lossy encoder's: its byte ring is the encoder's 4
// KiB ring and its chunk of decoded blocks the encoder's coefficient chunk, so a
// wave that encodes and then decodes (k_gc_roundtrip) holds 9.3 KiB, as either.
#define g_dring g_ring4
#define g_blk ((int32_t*)g_coef)
static_assert(kDRing == sizeof(g_ring4), "the decoder's ring is the lossy encoder's");

// enumDecode<16> patterns for k = 1..8 (filled once per device by
// launch_gc_decode): g_enum16[offset of k + code], the offsets in GTabs::e16
// Constant memory: the index is wave-uniform, so the load is a scalar one
// (s_load_dword through the scalar cache, counted on lgkmcnt), which does not
// wait on the walk's vector prefetch loads the way a vector load would.
constexpr int kEnum16N = 39202;
__constant__ uint32_t g_enum16[(kEnum16N + 1) / 2];       // two patterns per word, low half first

struct GDec {
	// Staging-only values, held in VGPRs (the lanes use them; the scalar walk
	// never does): the file's address, the payload size n (ric.cpp: at most
	// W*H), the file bytes that may be loaded.  SGPRs are the scarce resource.
	uint32_t vfile_lo, vfile_hi, vn, vflen;
	uint32_t range, low, code, nbits, buffer;
	uint32_t p, limit;
	uint32_t ovf;                      // 1: read past the end (RIC_E_STREAM), 2: ring overrun
	uint32_t st_hi;                    // file bytes [.., st_hi) are in the ring
	u32x4 stage;
	uint64_t win;                      // file bytes [wf, wf + 8)
	uint32_t wf, nxt;

	// The bytes around the read position in registers: file bytes [wf, wf + 8)
	// (wf a multiple of 4, p + 7 in [wf, wf + 4)), the next dword read from the
	// LDS ring one step ahead.  The read position only moves forward (huffDecode
	// moves it by at most 2, never back: it is entered with nbits < 8).
	// big-endian: file byte wf + o is bits 56 - 8 o of win (the byte swap is one
	// VALU op on the dword read from LDS)
	GC_DI uint32_t rd_dword(uint32_t f) const { return __builtin_bswap32(*(const uint32_t*)(g_dring + (f & (kDRing - 1)))); }
	// The window only moves inside what is staged: ensure() keeps at least
	// kDMargin staged bytes ahead before every block (and LL value) and before
	// every bin of a unary run, the one place a block can read without bound;
	// outside runs a block reads < 256 bytes (16 values x (a bin's <= 4
	// normalisation bytes + <= 25 raw bits), the tree bit, k, the enum code).
	GC_DI void wadvance()
	{
		win = vw((win << 32) | nxt);
		wf += 4;
		nxt = rd_dword(wf + 8);
	}
	// x + 7 in [wf, wf + 8).  The ring holds the virtual stream: the two bytes
	// in front and everything past the payload are zeroed when staged.
	GC_DI uint32_t byte(uint32_t x) const { return ru((uint32_t)(win >> (56 - ((x + 7) - wf) * 8)) & 255u); }
	GC_DI uint32_t next()
	{
		const uint32_t b = byte(p);
		if (p < limit) p++; else ovf |= 1;
		if (ru(p + 7 - wf) >= 4u) wadvance();
		return b;
	}
	GC_DI u32x4 load_kib(uint32_t off) const
	{
		const uint32_t o = off + lane_id() * 16;
		u32x4 v = {0, 0, 0, 0};
		if (o + 16 <= vflen) v = *gld((const u32x4*)((((uint64_t)vfile_hi << 32) | vfile_lo) + o));
		// virtual bytes past the payload read as 0 (ric.cpp's zero padding):
		// file bytes from n + 9 on
		const uint32_t end = vn + 9;
		RIC_UNROLL
		for (int i = 0; i < 4; i++) {
			const uint32_t b = o + 4 * (uint32_t)i;
			const uint32_t keep = end <= b ? 0u : (end - b >= 4 ? 4u : end - b);
			v[i] &= keep >= 4 ? 0xFFFFFFFFu : (1u << (8 * keep)) - 1u;
		}
		return v;
	}
	GC_DI void put_kib(uint32_t off, const u32x4& v)
	{
		*(u32x4*)(g_dring + ((off + lane_id() * 16) & (kDRing - 1))) = v;
	}
	// stage file bytes up to kDAhead past the read position (the KiB at st_hi
	// is in flight in `stage`)
	GC_DI void stage_now()
	{
		put_kib(st_hi, stage);
		st_hi += 1024;
		while (st_hi < p + 7 + kDAhead) {
			const u32x4 v = load_kib(st_hi);
			put_kib(st_hi, v);
			st_hi += 1024;
		}
		stage = load_kib(st_hi);
	}
	// between chunks: the bytes a chunk may read are staged; flags a chunk
	// that read past them
	// (pend == st_hi: the next KiB is in flight.)  Staging only advances with
	// the read position, so the ring always keeps the bytes just behind it.
	GC_DI void ensure()
	{
		if (__builtin_expect((int)ru(st_hi - (p + 7 + kDMargin)) < 0, 0)) stage_now();
	}
	GC_DI void refill()
	{
		if (st_hi >= p + 7 + kDAhead) return;
		stage_now();
	}
	// f: the file, len its size, cap the bytes readable at f (a multiple of 16)
	GC_DI void init(const uint8_t* f, uint32_t len, uint32_t cap, uint32_t npay)
	{
		uint32_t fl = (len + 15) & ~15u;
		if (fl > cap) fl = cap;
		vfile_lo = to_vgpr((uint32_t)(uintptr_t)f);
		vfile_hi = to_vgpr((uint32_t)((uintptr_t)f >> 32));
		vn = to_vgpr(npay);
		vflen = to_vgpr(fl);
		st_hi = 0;
		for (uint32_t off = 0; off < 2 * 1024 + 1024; off += 1024) { put_kib(off, load_kib(off)); st_hi = off + 1024; }
		g_dring[7 + (lane_id() & 1)] = 0;                // virtual bytes 0, 1 (file 7, 8: the header's tail)
		stage = load_kib(st_hi);
		limit = npay + 2 + 65536 - 16;
		range = 1u << 16;
		nbits = 0; buffer = 0; ovf = 0;
		wf = 8;
		win = (uint64_t)rd_dword(8) << 32 | rd_dword(12);
		nxt = rd_dword(16);
		code = low = (byte(2) << 8) | byte(3);
		p = 4;
	}
	GC_DI void norm()                                    // normalize_dec, muxcodec.cpp:76-85
	{
		uint32_t it = 0;
		do {
			if (((code - low + range - 1) ^ (code - low)) >= 0x01000000u) range = (low - code) & 4095u;
			const uint32_t b = next();
			low = vr((low << 8) | b);
			code = vr((code << 8) | b);
			range = vr(range << 8);
			if (__builtin_expect(++it > 4, 0)) { ovf |= 1; range = 1u << 16; }   // corrupt stream: no spin
		} while (ru(range) <= 4096u);
	}
	GC_DI uint32_t bit(uint32_t freq)                    // getBit, muxcodec.h:205-213
	{
		if (__builtin_expect(ru(range) <= 4096u, 0)) norm();
		const uint32_t t = (range * freq) >> 12;
		// low < t as arithmetic (a bool-to-int on the scalar unit would take a
		// round trip through a VGPR)
		const uint32_t lt = (uint32_t)(((uint64_t)low - (uint64_t)t) >> 63);
		const uint32_t tst = lt - 1u;
		low = vr(low - (t & tst));
		range = vr(t + ((range - 2 * t) & tst));
#if RIC_GC_UCOND == 3
		return ru(1u - lt);
#else
		return 1u - lt;
#endif
	}
	GC_DI void fill(uint32_t len)                        // fillBuffer, muxcodec.cpp:572-579
	{
		// the nb bytes fillBuffer reads one at a time, taken from the window at
		// once (nb <= 4: len <= 26; the window holds >= 5 bytes at the read
		// position; bytes past the payload are the ring's zeros).  One straight
		// path, no byte loop: a corrupt stream that runs to the read limit stops
		// there and is flagged, as next() does.
		const uint32_t nb = (len - nbits + 7) >> 3;
		const uint32_t o = p + 7 - wf;
		const uint32_t v = (uint32_t)((win << (8 * o)) >> (64 - 8 * nb));
		buffer = vv((uint32_t)(((uint64_t)buffer << (8 * nb)) | v));
		nbits = vv(nbits + 8 * nb);
		p += nb;
		if (__builtin_expect(p > limit, 0)) { p = limit; ovf |= 1; }
		if (ru(p + 7 - wf) >= 4u) wadvance();
	}
	GC_DI uint32_t bits(uint32_t len)                    // bitsDecode, muxcodec.h:233-239
	{
		if ((int)ru(nbits - len) < 0) fill(len);
		nbits = vv(nbits - len);
		return (buffer >> nbits) & ((1u << len) - 1);
	}
	// the same with the mask (1 << len) - 1 given
	GC_DI uint32_t bits_m(uint32_t len, uint32_t mask)
	{
		if ((int)ru(nbits - len) < 0) fill(len);
		nbits = vv(nbits - len);
		return (buffer >> nbits) & mask;
	}
	// huffDecode (muxcodec.h:241-276): lane s tests code s of the table row
	// (hrow: (code << 5) | len per lane, 0 past the row); the first match wins
	GC_DI uint32_t huff(uint32_t hrow, uint32_t nsym)
	{
		const uint32_t c = (((buffer << 16) | (byte(p) << 8) | byte(p + 1)) >> nbits) & 0xFFFFu;
		const uint32_t l = lane_id();
		const uint32_t len_l = hrow & 31u;
		const bool hit = l < nsym && len_l > 0 && (c >> (16 - len_l)) == (hrow >> 5);
		const uint64_t m = __ballot(hit);
		uint32_t sym, len;
		if (m) { sym = (uint32_t)__builtin_ctzll(m); len = lget(len_l, sym); }
		else { sym = 0; len = lget(len_l, 0); }
		p -= (uint32_t)((int)(nbits - len) >> 3);
		if (p > limit) { p = limit; ovf |= 1; }
		if (nbits < len) buffer = byte(p - 1);
		nbits = (nbits - len) & 7;
		while (ru(p + 7 - wf) >= 4u) wadvance();
		return sym;
	}
	// enum_code's code part (muxcodec.cpp:391-393); cnk lane i = (n-1)*8 + k-1:
	// CnkLen | CnkLost << 8, in two lane arrays
	GC_DI uint32_t enum_code(const uint32_t (&cnk)[2], uint32_t k, uint32_t nmax)
	{
		const uint32_t i = (nmax - 1) * 8 + (k - 1);
		const uint32_t e = i < 64 ? lget(cnk[0], i) : lget(cnk[1], i - 64);
		const uint32_t lost = e >> 8;
		uint32_t c = bits((e & 255u) - 1);
		if (c >= lost) c = ((c << 1) | bits(1)) - lost;
		return c;
	}
	// enumDecode (muxcodec.cpp:381-405); binom lane (r - 1) * 16 + n = C(n, r)
	GC_DI uint32_t enum_n(const uint32_t (&cnk)[2], const uint32_t (&binom)[2], uint32_t k, uint32_t nmax, bool guard16)
	{
		int n = (int)nmax - 1;
		uint32_t out = 0;
		if (k > ((nmax + 1) >> 1)) { k = nmax - k; out = (1u << nmax) - 1; }
		int row = (int)k - 1;
		uint32_t c = enum_code(cnk, k, nmax);
		if (guard16) {
			// the host's table decode (decoder.cpp enum16) reads code 0 for a
			// code >= C(16, k) (corrupt streams only); C(16, k) = C(15, k) + C(15, k - 1)
			const uint32_t i1 = (k - 1) * 16 + 15, i0 = (k - 2) * 16 + 15;
			const uint32_t a1 = i1 < 64 ? lget(binom[0], i1) : lget(binom[1], i1 - 64);
			const uint32_t a0 = k < 2 ? 1u : (i0 < 64 ? lget(binom[0], i0) : lget(binom[1], i0 - 64));
			if (c >= a1 + a0) c = 0;
		}
		// the reference scans n downwards and takes each n with C(n, row + 1) <= c:
		// per row that is the largest such n, found by the lanes at once (lane
		// 16 (row & 3) + j of binom[row >> 2] holds C(j, row + 1); C(0, r) = 0, so
		// some lane always qualifies while n >= 0)
		const uint32_t l = lane_id();
		while (row >= 0 && n >= 0) {
			const uint32_t vrow = row < 4 ? binom[0] : binom[1];
			const bool ok = (l >> 4) == ((uint32_t)row & 3u) && (l & 15u) <= (uint32_t)n && vrow <= c;
			const uint64_t m = __ballot(ok);
			const uint32_t idx = 63u - (uint32_t)__builtin_clzll(m);
			const uint32_t nn = idx & 15u;
			out ^= 1u << nn;
			c -= lget(vrow, idx);
			row--;
			n = (int)nn - 1;
		}
		return out;
	}
	// enumDecode<16> by table (the host decoder's decoder.cpp enum16): the
	// pattern of (k, code) for k <= 8, complemented above 8.  One load from a
	// 78 KB table in HBM (L2 / scalar-cache resident) instead of k ballot rows.
	// etab: the table (GDecArgs::etab); the offset of k's patterns and C(16,
	// k) come from the lane table T.e16
	GC_DI uint32_t enum16(const uint32_t (&cnk)[2], const GTabs& T, const uint32_t* etab, uint32_t k)
	{
		const bool comp = k > 8;
		const uint32_t kk = comp ? 16 - k : k;
		const uint32_t off = lget(T.e16, kk), lim = lget(T.e16, 16 + kk);
		// enum_code(cnk, kk, 16) with the lengths from T.e16 (cnk[], two lane
		// arrays used only by the edge blocks, is then not live across the
		// block walk: at 88 VGPRs it was spilled to scratch and reloaded, with
		// a full vmcnt wait, for every full block)
		const uint32_t e = lget(T.e16, 32 + kk);
		const uint32_t lost = e >> 8;
		uint32_t c = bits((e & 255u) - 1);
		if (c >= lost) c = ((c << 1) | bits(1)) - lost;
		if (c >= lim) c = 0;                                 // the host reads code 0 past C(16, k) (corrupt streams)
		const uint32_t i = off + c;
		// RIC_GC_UNIFORM: the pattern made wave-uniform (a global-address-space
		// load + readfirstlane).  Read through the generic pointer (the default)
		// the compiler counts it as divergent, and the decoder state the
		// coefficient loop touches lives in VGPRs with exec-mask branches: about
		// half the decoder's instructions go to the VALU instead of the scalar
		// unit.  Measured (C3 serving step, 2816 streams, k_gc_roundtrip per
		// stream): divergent 1313 M SALU + 1323 M VALU, 11.94 s per launch;
		// uniform 2229 M SALU + 366 M VALU, 13.02 s.  With ~3 coder waves per
		// SIMD the scalar unit is the shared port: the balanced mix issues more.
#if RIC_GC_UNIFORM
		const uint32_t m = (__builtin_amdgcn_readfirstlane(*gld(etab + (i >> 1))) >> ((i & 1) * 16)) & 0xFFFFu;
#else
		const uint32_t m = (etab[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu;
#endif
		return comp ? ~m & 0xFFFFu : m;
	}
	GC_DI uint32_t max_dec(uint32_t max)                 // maxDecode, muxcodec.cpp:526-534
	{
		uint32_t value = 0;
		const uint32_t len = (uint32_t)bitlen(max), lost = (1u << len) - max - 1;
		if (len > 1) value = bits(len - 1);
		if (value >= lost) value = ((value << 1) | bits(1)) - lost;
		return value;
	}
	GC_DI uint32_t taboo()                               // tabooDecode, muxcodec.cpp:242-280
	{
		uint32_t nbl, suml;
		taboo_lanes(nbl, suml);
		const uint32_t nt = 2;
		int i, l = nt;
		uint32_t nb = 0;
		if (nbits < nt) fill(nt);
		uint32_t t = ((1u << nt) - 1) << (nbits - nt);
		while ((~buffer & t) != t) {
			l++;
			if (l > (int)nbits) { fill((uint32_t)l); t <<= 8; }
			t >>= 1;
			if (l > 25) { ovf |= 1; return 0; }
		}
		nbits -= (uint32_t)l;
		const uint32_t cd = buffer >> (nbits + nt + 1);
		i = l - (int)nt;
		if (i > 0) { i--; nb += lget(suml, (uint32_t)i); }
		while (i > (int)nt) {
			uint32_t j = 1;
			while (j < (uint32_t)i && ((cd >> (i - (int)j)) & 1) == 0) j++;
			nb += lget(suml, (uint32_t)(i - (int)j)) - lget(suml, (uint32_t)(i - (int)nt));
			i -= (int)j;
		}
		if (i == (int)nt) nb -= 1;
		nb += cd & ((1u << i) - 1);
		return nb;
	}
};

struct GBitD {                                          // CBitCodec::decode, bitcodec.h:62-70
	uint32_t st;
	GC_DI void init() { st = 2048u; }
	GC_DI uint32_t decode(GDec& d, const GTabs& T, uint32_t c)
	{
		const uint32_t v = lget(st, c);
		uint32_t freq = v & 0xFFFFu, sh = (v >> 16) & 0xFFu, mps = v >> 24;
		uint32_t sym = d.bit(freq) ^ 1;
		freq = (freq + (sym << (9 - sh)) - (freq >> (3 + sh))) & 0xFFFFu;
		sym ^= mps;
		const uint32_t th = lget(T.bit_thr, sh), t0 = th & 0xFFFFu, t1 = th >> 16;
		if (__builtin_expect((int)ru((t0 - t1) - ((freq - t1) & 0xFFFFu)) < 0, 0)) {
			if (freq > t0) {
				if (sh == 0) { mps ^= 1; freq = 4096u - freq; sh = 1; }
				else sh--;
			} else if (sh < 9) sh++;
		}
		st = lset(st, c, freq | sh << 16 | mps << 24);
		return sym;
	}
};

struct GGeoD {                                          // one CGeomCodec context in scalars (as GGeoCtx)
	uint32_t freq, idx, k, s3, t0, span, k1, kmask;
	GC_DI void params(const GTabs& T)
	{
		const uint32_t ks = lget(T.geo_ks, idx), s = ks >> 8;
		const uint32_t thr = lget(T.geo_thr, s);
		k = ks & 0xFFu; s3 = s + 3; t0 = thr & 0xFFFFu; span = (thr >> 16) - t0;
		k1 = k + 1; kmask = (2u << k) - 1u;
	}
	GC_DI void load(uint32_t arr, uint32_t c, const GTabs& T) { const uint32_t v = lget(arr, c); freq = v & 0xFFFFu; idx = v >> 16; params(T); }
	GC_DI uint32_t packed() const { return freq | idx << 16; }
	// SIGNED: magnitude - 1 then the raw sign (decoder.cpp GeoReg::decode_signed);
	// else the plain geometric value (GeoM::decode).  lmax: the unary guard.
	template <bool SIGNED>
	GC_DI int decode(GDec& d, const GTabs& T, uint32_t lmax)
	{
		const uint32_t f = freq;
		uint32_t fr = freq, l = 0;
		int out;
#if RIC_GC_GEOFAST
		if (__builtin_expect(ru(d.bit(f)), 0)) {         // most runs are empty: fall through
			do {
				fr -= fr >> s3;
				if (++l > lmax) break;
				d.ensure();
			} while (ru(d.bit(f)));
		}
		if (SIGNED) {
			const uint32_t v = d.bits_m(k1, kmask);
			const int mag = (int)((l << k) | (v >> 1)) + 1;
			out = (v & 1) ? -mag : mag;
		} else {
			if (k > 0) l = (l << k) | d.bits(k);
			out = (int)l;
		}
#if RIC_GC_OUTPIN
		// the value is formed here, before the re-index branch may redefine k
		// (else the compiler sinks it past the branch and copies k and its
		// mask twice per value to merge them)
		asm volatile("" : "+v"(out));
#endif
		fr = fr + ((4096u - fr) >> s3);
		if (__builtin_expect(fr - t0 > span, 0)) {
#else
		if (__builtin_expect(ru(d.bit(f)), 0)) {         // most runs are empty: fall through
			do {
				fr -= fr >> s3;
				if (++l > lmax) break;
				d.ensure();
			} while (ru(d.bit(f)));
		}
		if (SIGNED) {
			const uint32_t v = d.bits(k + 1);
			const int mag = (int)((l << k) | (v >> 1)) + 1;
			out = (v & 1) ? -mag : mag;
		} else {
			if (k > 0) l = (l << k) | d.bits(k);
			out = (int)l;
		}
		fr = (fr + ((4096u - fr) >> s3)) & 0xFFFFu;
		if (__builtin_expect((int)ru(span - ((fr - t0) & 0xFFFFu)) < 0, 0)) {
#endif
			if (fr < t0) { if (idx < 24) idx++; }
			else if (idx > 0) idx--;
			if (idx >= 9) fr = 2048;
			params(T);
		}
		freq = fr;
		return out;
	}
};

GC_DI int trunc_c(int is_int, int v) { return is_int ? v : (int)(int16_t)v; }
GC_DI int ldc(const char* band, int is_int, long e)
{
	return is_int ? (int)gld((const int32_t*)band)[e] : (int)gld((const int16_t*)band)[e];
}
GC_DI void stc(char* band, int is_int, long e, int v)
{
	if (is_int) gst((int32_t*)band)[e] = v;
	else gst((int16_t*)band)[e] = (int16_t)v;
}

// CBandCodec::pred<decode> (LL DPCM), bandcodec.cpp:62-104: the previous row
// comes in 64-column runs through the lanes; a run of decoded values is stored
// by the lanes at its end.
GC_DI void pred_dec(GDec& d, const GTabs& T, const GBandDesc& B, char* arena)
{
	static constexpr uint8_t ginit[16] = {9,10,11,12,13,14,15,16,17,18,19,20,21,22,23,15};
	char* c = arena + B.off;
	const long st = B.pitch;
	const int dx = B.dx, dy = B.dy, is_int = B.is_int;
	uint32_t geo = geo_init_lane(ginit);
	const uint32_t l = lane_id();
	for (int j = 0; j < dy; j++) {
		int left = 0, upleft = 0;
		for (int x0 = 0; x0 < dx; x0 += 64) {
			__threadfence();                          // the previous row's stores
			const int i = x0 + (int)l;
			const int up = (j > 0 && i < dx) ? ldc(c, is_int, (long)(j - 1) * st + i) : 0;
			uint32_t cur = 0;
			const int nx = dx - x0 < 64 ? dx - x0 : 64;
			for (int q = 0; q < nx; q++) {
				const int x = x0 + q;
				int v;
				d.ensure();
				if (j == 0 && x == 0) {
					v = trunc_c(is_int, u2s((int)d.taboo()));
				} else {
					uint32_t ctx = 15;
					int pred;
					const int u = (int)lget((uint32_t)up, (uint32_t)q);
					if (j == 0) pred = left;
					else if (x == 0) pred = u;
					else {
						const int a = left - upleft, bb = u - upleft;
						int var = bitlen((uint32_t)((a < 0 ? -a : a) + (bb < 0 ? -bb : bb)));
						ctx = (uint32_t)(var > 15 ? 15 : var);
						pred = left + u - upleft;
					}
					GGeoD g;
					g.load(geo, ctx, T);
					const int r = g.decode<false>(d, T, 1u << 20);
					geo = lset(geo, ctx, g.packed());
					v = trunc_c(is_int, pred + u2s(r));
					upleft = u;
				}
				if (j > 0 && x == 0) upleft = (int)lget((uint32_t)up, 0);
				left = v;
				cur = lset(cur, (uint32_t)q, (uint32_t)v);
			}
			if (i < dx) stc(c, is_int, (long)j * st + i, (int)cur);
			d.refill();
		}
	}
	__threadfence();
}

// Per block of a chunk (lane j = scan position s0 + j): what the parent band
// and the geometry say, computed by the lanes before the walk.
//  bits 0-4 tree context, 5 full (not an edge block), 6 propagated (parent
//  anchor holds INSIGNIF), 7 clear the parent anchor, 8-9 w - 1, 10-11 h - 1
GC_DI uint32_t block_info(const GBandDesc& B, const GBandDesc* P, const char* arena, int nblk, int s, int& bx, int& by)
{
	bx = by = 0;
	if (s >= nblk) return 0;
	scan_block(s, B.dx, B.dy, bx, by);
	const int w = B.dx - bx * 4 < 4 ? B.dx - bx * 4 : 4, h = B.dy - by * 4 < 4 ? B.dy - by * 4 : 4;
	const bool full = w == 4 && by * 4 + 4 <= B.dy;
	uint32_t info = (uint32_t)(w - 1) << 8 | (uint32_t)(h - 1) << 10 | (full ? 1u << 5 : 0u);
	uint32_t ctx = 15;
	if (P) {
		const char* pb = arena + P->off;
		const long pst = P->pitch;
		const int px = bx * 2, py = by * 2;
		if (full) {
			const int a = ldc(pb, P->is_int, (long)py * pst + px);
			if (a == kInsignif) {
				info |= 1u << 6 | 1u << 7;
			} else {
				// maxLen<2, decode> (bandcodec.cpp:324-344)
				int mx = 0, mn = 0;
				for (int jj = 0; jj < 2; jj++)
					for (int ii = 0; ii < 2; ii++) {
						const int v = ldc(pb, P->is_int, (long)(py + jj) * pst + px + ii);
						mx = v > mx ? v : mx;
						mn = v < mn ? v : mn;
					}
				mn = trunc_c(P->is_int, -mn);
				ctx = (uint32_t)bitlen((uint32_t)(mn > mx ? mn : mx));
			}
		} else if (px < P->dx && (by * 4 + 4 <= B.dy || py < P->dy)) {
			if (ldc(pb, P->is_int, (long)py * pst + px) == kInsignif) info |= 1u << 7;
		}
	}
	return info | (ctx & 31u);
}

// CBandCodec::tree<decode> (bandcodec.cpp:484-589; decoder.cpp tree_dec):
// chunks of 64 blocks in scan order; each chunk's values are built in LDS and
// stored by the lanes (every position of every block, so no Clear() pass), the
// parent anchors the chunk consumed are cleared by the lanes too.
// cblk (a compacted pool's band, B.cmp): the plane's compact block; the
// chunk's blocks go there as masks + values (vpos: the plane's values so far,
// advanced past the band's), at most vcap values (a stream that decodes more,
// a corrupt one, is flagged)
template <bool ETAB>
GC_DI void tree_dec(GDec& d, const GTabs& T, const GBandDesc& B, const GBandDesc* P, char* arena,
                    const uint32_t (&cnk)[2], const uint32_t (&binom)[2], const uint32_t* etab, const uint32_t* yield,
                    bool prio_half = false, char* cblk = nullptr, uint32_t cvals_off = 0, uint32_t vcap = 0,
                    uint32_t* vpos = nullptr)
{
	const bool high = B.high;
	arena = vcp(arena);
	yield = vcp(yield);
	if (cblk) { cblk = vcp(cblk); cvals_off = vcu(cvals_off); vcap = vcu(vcap); }
	char* band = arena + B.off;
	const int is_int = B.is_int;
	const long st = B.pitch;
	const int dx = B.dx, dy = B.dy;
	const int nblk = ((dx + 3) >> 2) * ((dy + 3) >> 2);
	const uint32_t l = lane_id();
	const int mval = high ? 0 : kInsignif;             // the INSIGNIF mark, where the band has children
	const uint32_t gidx = l == 0 ? 5u : (l < 12 ? 9u : (l < 15 ? 10u : 11u));
	uint32_t geo = (gidx >= 9 ? 2048u : (uint32_t)((kGeoThres[gidx - 1] + kGeoThres[gidx]) >> 1)) | gidx << 16;
	GBitD tree, bord;
	tree.init(); bord.init();
	uint32_t kmean = l < 8 ? (uint32_t)((l < 4 ? l + 2 : (l == 4 ? 8 : (l == 5 ? 11 : (l == 6 ? 13 : 14)))) << 10)
	                       : 15u << 10;
	const uint32_t hbase = high ? 0u : 256u, hn = high ? 16u : 17u;
	const uint32_t lmax = is_int ? (1u << 20) : (1u << 15);
	const int s_half = prio_half ? (nblk / 2) & ~63 : -1;
	uint32_t cnt_band = 0;                              // (compacted) the band's values so far
	ChunkSync csy;
	for (int s0 = 0; s0 < nblk; s0 += 64) {
		csy.step(yield);
		if (s0 == s_half) set_prio<0>(1);
		int bx, by;
		const uint32_t info = block_info(B, P, arena, nblk, s0 + (int)l, bx, by);
		// the chunk's blocks: zeros, and the marks of the propagated ones
		RIC_UNROLL
		for (int i = 0; i < 16; i++) g_blk[l * 16 + i] = 0;
		if ((info >> 6) & 1) {
			g_blk[l * 16 + 0] = mval; g_blk[l * 16 + 2] = mval; g_blk[l * 16 + 8] = mval; g_blk[l * 16 + 10] = mval;
		}
		__threadfence_block();
		const int nj = nblk - s0 < 64 ? nblk - s0 : 64;
		for (int j = 0; j < nj; j++) {
			if (RIC_GC_YCHK < 64 && j && !(j & (RIC_GC_YCHK - 1))) coder_yield(yield);
			const uint32_t in = lget(info, (uint32_t)j);
			const uint32_t ob = (uint32_t)j * 16;
			d.ensure();
			if ((in >> 5) & 1) {
				if ((in >> 6) & 1) continue;                   // propagated
				const uint32_t ctx = in & 31u;
				if (ru(tree.decode(d, T, ctx))) {
					g_blk[ob + 0] = mval; g_blk[ob + 2] = mval; g_blk[ob + 8] = mval; g_blk[ob + 10] = mval;
					continue;
				}
				const uint32_t km = lget(kmean, ctx);
				const uint32_t idx = (km + (1u << 9)) >> 10;
				const uint32_t hrow = l < hn ? (uint32_t)g_huff[hbase + idx * hn + l] : 0u;
				const uint32_t k = d.huff(hrow, hn) + (high ? 1u : 0u);
				if (high || k != 0) {
					uint32_t sig = ru(k == 16 ? 0xFFFFu : ETAB ? d.enum16(cnk, T, etab, k) : d.enum_n(cnk, binom, k, 16, true));
					GGeoD g;
					g.load(geo, k - 1, T);
#if RIC_GC_SIGREV
					// bit i = raster i (one bit reverse per block): the values in
					// raster order by the lowest set bit, two scalar ops per value
					// fewer than the highest-bit walk
#if RIC_GC_VADDR
					// (the store's position found and addressed on the VALU)
					for (uint32_t rs = __builtin_bitreverse32(sig) >> 16; rs; rs &= rs - 1) {
						uint32_t rv = rs;
						asm volatile("" : "+v"(rv));
						g_blk[ob + (uint32_t)__builtin_ctz(rv)] = g.decode<true>(d, T, lmax);
					}
#else
					for (uint32_t rs = __builtin_bitreverse32(sig) >> 16; rs; rs &= rs - 1)
						g_blk[ob + (uint32_t)__builtin_ctz(rs)] = g.decode<true>(d, T, lmax);
#endif
#else
					while (sig) {
						const uint32_t b = 31u - (uint32_t)__builtin_clz(sig);      // bit 15 = raster 0
						sig &= ~(1u << b);
						g_blk[ob + 15 - b] = g.decode<true>(d, T, lmax);   // stc truncates a short band's value
					}
#endif
					geo = lset(geo, k - 1, g.packed());
				}
				const uint32_t kk = high ? k - 1 : k;
				kmean = lset(kmean, ctx, (km + (kk << 7) - (km >> 3)) & 0xFFFFu);
			} else {
				if (ru(bord.decode(d, T, 0))) continue;
				const uint32_t w = ((in >> 8) & 3) + 1, h = ((in >> 10) & 3) + 1, cnt = w * h;
				uint32_t k = high ? d.max_dec(cnt - 1) + 1 : d.max_dec(cnt);
				if (k > cnt) k = cnt;
				if (high || k != 0) {
					uint32_t sig = k != cnt ? d.enum_n(cnk, binom, k, cnt, false) : (1u << cnt) - 1;
					const uint32_t gc = kKConv2[kKConv1[cnt]][k - 1];
					GGeoD g;
					g.load(geo, gc, T);
					for (uint32_t q = 0; q < cnt; q++) {
						if (sig & (1u << (cnt - 1))) {
							const uint32_t r = w == 4 ? q >> 2 : q / w, cc = q - r * w;
							g_blk[ob + r * 4 + cc] = g.decode<true>(d, T, lmax);
						}
						sig <<= 1;
					}
					geo = lset(geo, gc, g.packed());
				}
			}
		}
		__threadfence_block();
		// the lanes store the chunk
		if (cblk) {
			// compacted: each block's mask (its non-zero positions, raster over
			// its w x h corner) and those values in that order, the blocks' values
			// back to back (k_dcmp_expand scatters them into the dense band)
			const int w = (int)((info >> 8) & 3) + 1, h = (int)((info >> 10) & 3) + 1;
			const bool in = s0 + (int)l < nblk;
			uint32_t m = 0;
			if (in)
				for (int r = 0; r < h; r++)
					for (int q = 0; q < w; q++) m |= (g_blk[l * 16 + r * 4 + q] != 0 ? 1u : 0u) << (r * w + q);
			uint32_t nc;
			const uint32_t o = wave_excl_popc(m, nc);
			const uint32_t v0 = *vpos + cnt_band;
			if (l == 0) gst((uint32_t*)(cblk + B.ccoff_off))[s0 >> 6] = cnt_band;
			if (in) {
				gst((uint16_t*)(cblk + B.cmask_off))[s0 + (int)l] = (uint16_t)m;
				GAS int16_t* vals = gst((int16_t*)(cblk + cvals_off));
				uint32_t k = v0 + o;
				for (int r = 0; r < h; r++)
					for (int q = 0; q < w; q++) {
						const int v = g_blk[l * 16 + r * 4 + q];
						if (v == 0) continue;
						if (k < vcap) vals[k] = (int16_t)v;
						k++;
					}
				if (((info >> 7) & 1) && P) stc(arena + P->off, P->is_int, (long)(by * 2) * P->pitch + bx * 2, 0);
			}
			if (v0 + nc > vcap) d.ovf |= 1;
			cnt_band += nc;
		} else if (s0 + (int)l < nblk) {
			const int w = (int)((info >> 8) & 3) + 1, h = (int)((info >> 10) & 3) + 1;
			for (int r = 0; r < h; r++)
				for (int q = 0; q < w; q++) stc(band, is_int, (long)(by * 4 + r) * st + bx * 4 + q, g_blk[l * 16 + r * 4 + q]);
			if (((info >> 7) & 1) && P) stc(arena + P->off, P->is_int, (long)(by * 2) * P->pitch + bx * 2, 0);
		}
		d.refill();
	}
	if (cblk) {
		if (lane_id() == 0) gst((uint32_t*)cblk)[B.cmp - 1] = cnt_band;     // nval[k]
		*vpos += cnt_band;
	}
	__threadfence();
}

// One frame's stream per workgroup (one wave): DecompressImage's decoding
// order (src/ric/ric.cpp:207-225 -> CWavelet2D::DecodeBand,
// src/lib/wavelet2d.cpp:179-222): the coarsest LL, then coarse to fine V, H, D.
// The bands land in the frame's arena, ready for the inverse kernels.
// frame f's stream of len bytes decoded into its arena; the result word (0
// ok, 1 the stream ran past its end, 3 | position << 4 a staging overrun)
template <bool ETAB>
GC_DI uint32_t dec_frame(const GDecArgs& a, int f, uint32_t len)
{
	char* arena = a.arena + (size_t)f * a.astride;
	const uint8_t* file = a.in + (size_t)f * a.istride;
	const uint32_t l = lane_id();
	uint32_t cnk[2], binom[2];
	for (int h = 0; h < 2; h++) {
		const uint32_t i = (uint32_t)h * 64 + l;        // (nmax - 1) * 8 + (k - 1)
		cnk[h] = (uint32_t)kCnkLen[i >> 3][i & 7] | (uint32_t)kCnkLost[i >> 3][i & 7] << 8;
		const uint32_t r = (i >> 4) + 1, nn = i & 15;   // C(nn, r)
		uint32_t cb = 1;
		if (nn < r) cb = 0;
		else for (uint32_t t = 1; t <= r; t++) cb = cb * (nn - r + t) / t;
		binom[h] = cb;
	}
	GTabs T;
	T.init();
	GDec d;
	const uint32_t npix = (uint32_t)(a.w * a.h * a.nplanes);   // ric.cpp:203-205 reads W * H * C payload bytes
	const uint32_t npay = len > 9 ? (len - 9 < npix ? len - 9 : npix) : 0u;
	d.init(file, len, (uint32_t)a.istride, npay);
	auto dump = [&](int k) {
		if (a.dbg && l == 0) {
			GAS uint32_t* o = gst(a.dbg) + (size_t)f * 2048 + (size_t)k * 8;
			o[0] = d.range; o[1] = d.low; o[2] = d.code; o[3] = d.nbits; o[4] = d.buffer; o[5] = d.p; o[6] = d.ovf; o[7] = 0xC0DE;
		}
	};
	for (int p = 0; p + 1 < a.nplanes; p++) {          // colour: Y, Co before the last plane (ric.cpp:207-225)
		char* pa = arena + p * a.pstride;
		pred_dec(d, T, a.ll, pa);
		uint32_t vpos = 0;
		for (int b = 0; b < a.nb; b++) {
			const GBandDesc& B = a.b[b];
			tree_dec<ETAB>(d, T, B, B.par >= 0 ? &a.b[B.par] : nullptr, pa, cnk, binom, a.etab, a.yield, false,
			               a.cmp_rel && B.cmp ? pa + a.cmp_rel : nullptr, a.cvals_off, a.cvcap, &vpos);
		}
	}
	arena += (a.nplanes - 1) * a.pstride;              // the last (or only) plane, with the diagnostics
	pred_dec(d, T, a.ll, arena);
	dump(0);
	if (a.dbg) {                                     // the decoded LL, row-major (first 1024 values)
		const GBandDesc& B = a.ll;
		for (int i = (int)l; i < B.dx * B.dy && i < 1024; i += 64)
			gst(a.dbg)[(size_t)f * 2048 + 1024 + i] = (uint32_t)ldc(arena + B.off, B.is_int, (long)(i / B.dx) * B.pitch + i % B.dx);
	}
	uint32_t vpos = 0;
	for (int b = 0; b < a.nb; b++) {
		const GBandDesc& B = a.b[b];
		prio_band(a.prio, true, b, a.nb);
		tree_dec<ETAB>(d, T, B, B.par >= 0 ? &a.b[B.par] : nullptr, arena, cnk, binom, a.etab, a.yield,
		               a.prio == 3 && b == a.nb - 1, a.cmp_rel && B.cmp ? arena + a.cmp_rel : nullptr, a.cvals_off, a.cvcap,
		               &vpos);
		dump(b + 1);
	}
	// status in bits 0-3; on a staging overrun, the read position (diagnostic)
	if (a.dbg && f == 0) {                           // every band, the host harness's order (finest first, D H V, LL)
		__threadfence();
		size_t o = (size_t)gridDim.x * 2048;         // after every frame's 2048-word slot block
		for (int k = 0; k <= a.nb; k++) {
			// a.b is coarse -> fine V, H, D: band i of the harness order
			const int lev = k / 3, ori = k % 3;          // harness: level lev, orientation D=0, H=1, V=2
			const GBandDesc* B = k == a.nb ? &a.ll : &a.b[a.nb - 3 - 3 * lev + (2 - ori)];
			const int cnt = B->dx * B->dy;
			for (int i = (int)l; i < cnt; i += 64)
				gst(a.dbg)[o + i] = (uint32_t)ldc(arena + B->off, B->is_int, (long)(i / B->dx) * B->pitch + i % B->dx);
			o += cnt;
		}
	}
	return d.ovf & 2 ? 3u | (d.p < (1u << 27) ? d.p << 4 : 0xFFFFFFF0u) : (d.ovf ? 1u : 0u);
}

template <bool ETAB>
__global__ void __launch_bounds__(64) GC_KATTR k_gc_decode(const GDecArgs* __restrict__ ap)
{
	const GDecArgs& a = *ap;
	const int f = blockIdx.x;
	const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
	if (a.prio == 1) set_prio<1>(1);
	else set_prio<3>(a.prio);
	level_init(a.prio, 0x7FFu);                      // (a finished wave's word reads as ahead of every wave)
	load_huff();
	const uint32_t r = dec_frame<ETAB>(a, f, gld(a.lens)[(size_t)f * a.lens_stride]);
	level_step(true);
	if (lane_id() == 0) {
		gst(a.res)[f] = r;
		if (a.ts) ts_put(a.ts, f, t_start);
	}
}

// Encode and then decode frame f's stream on one wave (lossy streams: the
// 4 KiB ring).  Once the stream is in HBM, its length and status go to
// `posted` (host memory the caller polls, so the stream can leave for the host
// while the wave decodes): posted[2 f] = the coder's end offset, posted[2 f +
// 1] = status | 0x100.  ea.res / da.res get the words k_gc_encode /
// k_gc_decode write.  A stream that failed is not decoded (result word 0).
template <bool ETAB>
__global__ void __launch_bounds__(64) GC_KATTR k_gc_roundtrip(const GEncArgs* __restrict__ eap, const GDecArgs* __restrict__ dap,
                                                    uint32_t* posted, uint32_t* posted_dec, uint32_t tag)
{
	const GEncArgs& ea = *eap;
	const GDecArgs& da = *dap;
	const int f = blockIdx.x;
	const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
	set_prio<3>(ea.prio);
	level_init(ea.prio, tag);
	load_huff();
	uint32_t end;
	const uint32_t rc = enc_frame<4096>(ea, f, end);
	if (lane_id() == 0) {
		gst(ea.res)[2 * f] = rc ? 0u : end;
		gst(ea.res)[2 * f + 1] = rc;
		if (ea.ts) ts_put(ea.ts, f, t_start);
	}
	post_result(posted, tag, f, rc, end);
	// (the fence in post_result also lets this wave's decoder read the stream back)
	__threadfence();
	const uint64_t t_dec = __builtin_amdgcn_s_memrealtime();
	if (da.prio == 1) set_prio<1>(1);
	const uint32_t r = rc ? 0u : dec_frame<ETAB>(da, f, end);
	if (lane_id() == 0) {
		gst(da.res)[f] = r;
		if (da.ts) ts_put(da.ts, f, t_dec);
	}
	// the decoded bands are the harvest's input, read by kernels the host
	// launches while this one still runs (on any XCD): written back (agent-scope
	// release) before the word that announces them.  posted_dec[f] = the decoder's
	// status (its low 7 bits; a diagnostic read position stays in res[f] only;
	// 0x80: the encode failed) | 0x100 | tag << 12
	if (posted_dec) {
		__threadfence();
		if (lane_id() == 0)
			__hip_atomic_store(posted_dec + f, (rc ? 0x80u : (r & 0x7Fu)) | 0x100u | tag << 12, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
	}
	level_step(true);                                     // (done: behind no one)
}
}  // namespace

// LDS footprint of a coder wave.  RIC_GC_LDS=<bytes> pads each coder
// workgroup's LDS allocation (static + dynamic) up to that size, which caps the
// coder waves per CU at floor(160 KiB / bytes): a CU's four SIMDs then hold at
// most one coder wave each instead of two stacking on one SIMD (the scalar
// coder issues from one wave per SIMD slot).  0 / unset: no padding.
static size_t gc_dyn_lds(const void* kernel)
{
	static const long want = [] { const char* e = getenv("RIC_GC_LDS"); return e ? atol(e) : 0L; }();
	if (want <= 0) return 0;
	hipFuncAttributes fa;
	if (hipFuncGetAttributes(&fa, kernel) != hipSuccess) return 0;
	return (size_t)want > fa.sharedSizeBytes ? (size_t)want - fa.sharedSizeBytes : 0;
}

int launch_gc_encode(const GEncArgs* dev_args, int nframes, int lossless, hipStream_t st, uint32_t* posted, uint32_t tag)
{
	if (nframes <= 0) return 0;
	if (lossless) {
		static const size_t dyn = gc_dyn_lds((const void*)k_gc_encode<8192>);
		hipLaunchKernelGGL(k_gc_encode<8192>, dim3(nframes), dim3(64), dyn, st, dev_args, posted, tag & 0xFFFFFu);
	} else {
		static const size_t dyn = gc_dyn_lds((const void*)k_gc_encode<4096>);
		hipLaunchKernelGGL(k_gc_encode<4096>, dim3(nframes), dim3(64), dyn, st, dev_args, posted, tag & 0xFFFFFu);
	}
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the enumDecode<16> table, once per device (enumCode, muxcodec.cpp:352-359:
// code = sum over set bits of C(position, rank + 1))
static int enum16_upload(hipStream_t st)
{
	// (the kernels take the table's address from GDecArgs::etab: ric_gc_enum16_table)
	static std::mutex mu;
	static uint64_t done = 0;                        // devices 0..63
	int dev = 0;
	if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
	std::lock_guard<std::mutex> g(mu);
	if (done >> dev & 1) return 0;
	uint32_t C[17][17];
	for (int n = 0; n < 17; n++)
		for (int r = 0; r < 17; r++) C[n][r] = r == 0 ? 1 : n == 0 ? 0 : C[n - 1][r - 1] + C[n - 1][r];
	uint32_t off[9] = {0};
	uint32_t n = 0;
	for (int k = 1; k <= 8; k++) { off[k] = n; n += C[16][k]; }
	if (n != (uint32_t)kEnum16N) return -1;
	std::vector<uint16_t> pat(n, 0);
	for (uint32_t b = 1; b < 65536; b++) {
		const int k = __builtin_popcount(b);
		if (k > 8) continue;
		uint32_t code = 0, row = 0;
		for (int i = 0; i < 16; i++)
			if (b & (1u << i)) { code += C[i][row + 1]; row++; }
		pat[off[k] + code] = (uint16_t)b;
	}
	pat.resize((n + 1) & ~1u, 0);
	if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_enum16), pat.data(), pat.size() * sizeof(uint16_t), 0, hipMemcpyHostToDevice, st) !=
	        hipSuccess ||
	    hipStreamSynchronize(st) != hipSuccess)
		return -1;
	done |= 1ull << dev;
	return 0;
}

// the device address of the enumDecode<16> table (GDecArgs::etab), uploaded
// on first use on the current device
const uint32_t* gc_enum16_table(hipStream_t st)
{
	if (enum16_upload(st)) return nullptr;
	void* p = nullptr;
	if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_enum16)) != hipSuccess) return nullptr;
	return (const uint32_t*)p;
}

__global__ void k_gc_flag(uint32_t* flag, uint32_t v)
{
	if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

int launch_gc_flag(uint32_t* flag, uint32_t v, hipStream_t st)
{
	hipLaunchKernelGGL(k_gc_flag, dim3(1), dim3(64), 0, st, flag, v);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_gc_roundtrip(const GEncArgs* dev_eargs, const GDecArgs* dev_dargs, uint32_t* posted, uint32_t* posted_dec,
                        uint32_t tag, int nframes, hipStream_t st)
{
	if (nframes <= 0) return 0;
	// RIC_GC_ETAB=0 and RIC_GC_LDS act here as in the separate launches
	static const bool etab = [] { const char* e = getenv("RIC_GC_ETAB"); return !e || atoi(e) != 0; }();
	if (etab) {
		if (enum16_upload(st)) return -1;
		static const size_t dyn = gc_dyn_lds((const void*)k_gc_roundtrip<true>);
		hipLaunchKernelGGL(k_gc_roundtrip<true>, dim3(nframes), dim3(64), dyn, st, dev_eargs, dev_dargs, posted, posted_dec,
		                   tag & 0xFFFFFu);
	} else {
		static const size_t dyn = gc_dyn_lds((const void*)k_gc_roundtrip<false>);
		hipLaunchKernelGGL(k_gc_roundtrip<false>, dim3(nframes), dim3(64), dyn, st, dev_eargs, dev_dargs, posted, posted_dec,
		                   tag & 0xFFFFFu);
	}
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_gc_decode(const GDecArgs* dev_args, int nframes, hipStream_t st)
{
	if (nframes <= 0) return 0;
	// RIC_GC_ETAB=0: the lane-parallel enumerative decode instead of the table
	static const bool etab = [] { const char* e = getenv("RIC_GC_ETAB"); return !e || atoi(e) != 0; }();
	if (etab) {
		if (enum16_upload(st)) return -1;
		static const size_t dyn = gc_dyn_lds((const void*)k_gc_decode<true>);
		hipLaunchKernelGGL(k_gc_decode<true>, dim3(nframes), dim3(64), dyn, st, dev_args);
	} else {
		static const size_t dyn = gc_dyn_lds((const void*)k_gc_decode<false>);
		hipLaunchKernelGGL(k_gc_decode<false>, dim3(nframes), dim3(64), dyn, st, dev_args);
	}
	return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace ric
