// device.cpp -- device memory and the stream gather's transport (include/ric_gpu.h).
//
// Device memory: callers (the Python binding, the tests, bench.py, the CLI)
// get HBM buffers from the product's own HIP runtime, so no second runtime
// (e.g. one bundled with a framework) is ever mapped into the process beside
// it.
//
// ric_comm: the path's one exchange -- the .ric streams of
// every rank to rank 0 -- over RCCL (xGMI between the GPUs of a node), one
// communicator per process, point-to-point send / receive of device buffers.
// The chunked gather protocol itself (which streams go in which round) is
// host logic in shard.py, shared with the CPU (gloo) transport of the tests.
// The reference has no multi-process path (src/ric/ric.cpp:174-176 writes one
// file per image); this is the drop-in's scale-out.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "ric_gpu.h"
#include "codec_params.h"
#include "ric_image.h"

using namespace ric;

namespace {

bool dfail(hipError_t e, const char* what)
{
	if (e == hipSuccess) return false;
	set_last_error(std::string(what) + ": " + hipGetErrorString(e));
	(void)hipGetLastError();
	return true;
}
#define DCHK(x) do { if (dfail((x), #x)) return RIC_E_HIP; } while (0)

bool nfail(ncclResult_t r, const char* what)
{
	if (r == ncclSuccess) return false;
	set_last_error(std::string(what) + ": " + ncclGetErrorString(r));
	return true;
}
#define NCHK(x) do { if (nfail((x), #x)) return RIC_E_HIP; } while (0)

int on_device(int device)
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return set_last_error("no HIP device visible"), RIC_E_HIP;
	if (device < 0 || device >= n) return RIC_E_ARG;
	DCHK(hipSetDevice(device));
	return RIC_OK;
}

// The per-device side stream of the calls below: every copy, memset and
// digest runs on it and waits only for itself.  Never the legacy null stream
// or an implicit device-wide synchronisation (hipFree, hipHostFree): the
// gather calls these while the stream coder's kernel (seconds) is in flight
// (round 4 did a hipMalloc + hipFree per digest call; hipFree waits for the
// whole device).  Scratch only grows; the first use sizes it for a gather
// chunk (kStageMin), so a step never reallocates.
constexpr size_t kStageMin = 64u << 20;
struct Aux {
	std::mutex mu;
	hipStream_t st = nullptr;
	unsigned long long* d_dig = nullptr;   // kDigestRuns words
	unsigned long long* h_dig = nullptr;   // pinned
	uint8_t* h_stage = nullptr;            // pinned staging of ric_device_pack_h2d
	size_t stage_n = 0;
};
constexpr int kMaxDev = 64;
Aux g_aux[kMaxDev];

// The side and communicator streams, at the device's greatest stream
// priority (RIC_SIDE_PRIO=0: the default priority): the runtime gives each a
// hardware queue of its own instead of one of the GPU_MAX_HW_QUEUES shared
// round robin by the process's other streams, where a packet queued behind
// the stream coder's launch would wait for it (a digest kernel queued there
// waited ~0.5 s for a 0.9 s launch; profiles/r05_gather_ops_during_launch.log)
hipError_t side_stream_create(hipStream_t* st)
{
	static const int prio = [] { const char* e = getenv("RIC_SIDE_PRIO"); return e ? atoi(e) : 1; }();
	int least = 0, greatest = 0;
	if (prio && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
		return hipStreamCreateWithPriority(st, hipStreamNonBlocking, greatest);
	return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
}

// (device already current)
int aux_ready(Aux& a)
{
	if (!a.st) DCHK(side_stream_create(&a.st));
	if (!a.d_dig) DCHK(hipMalloc(&a.d_dig, sizeof(unsigned long long) * kDigestRuns));
	if (!a.h_dig) DCHK(hipHostMalloc(&a.h_dig, sizeof(unsigned long long) * kDigestRuns, 0));
	return RIC_OK;
}

int aux_stage(Aux& a, size_t bytes)
{
	if (a.stage_n >= bytes) return RIC_OK;
	if (a.h_stage) DCHK(pinned_free(a.h_stage));   // (growth only: once per size class)
	a.h_stage = nullptr;
	a.stage_n = 0;
	const size_t n = std::max(kStageMin, (bytes + (16u << 20) - 1) / (16u << 20) * (16u << 20));
	DCHK(hipHostMalloc(&a.h_stage, n, 0));
	a.stage_n = n;
	return RIC_OK;
}

// the digest of one host byte run (the formula of launch_digest): blocks of
// 4096 bytes, whose position-weighted sum fits 32 bits (255 * 4095 * 4096 / 2)
unsigned long long host_digest(const uint8_t* p, size_t n)
{
	constexpr unsigned long long kMul = 0x9E3779B97F4A7C15ull;
	unsigned long long s1 = 0, s2 = 0;
	for (size_t k = 0; k < n; k += 4096) {
		const size_t m = std::min<size_t>(4096, n - k);
		uint32_t b1 = 0, b2 = 0;
		for (size_t j = 0; j < m; j++) {
			b1 += p[k + j];
			b2 += (uint32_t)j * p[k + j];
		}
		s1 += b1;
		s2 += b2 + (unsigned long long)k * b1;
	}
	return s2 * kMul + s1;
}

// ------------------------------------------------ frees beside a coder launch
// (codec_params.h CoderCall).  The lock is held across an immediate free, so a
// CoderCall cannot begin (and launch) between the check and the free.
std::mutex g_free_mu;
int g_coder_calls = 0;
long g_parked = 0;
std::vector<std::pair<void*, bool>> g_deferred;   // (pointer, pinned)

hipError_t free_now(void* p, bool pinned) { return pinned ? hipHostFree(p) : hipFree(p); }

hipError_t free_or_park(void* p, bool pinned)
{
	if (!p) return hipSuccess;
	// RIC_PARK_FREES=0: free at once (the A/B of tests/test_gpu_zz_concurrency.py)
	static const bool park = [] { const char* e = getenv("RIC_PARK_FREES"); return !e || atoi(e) != 0; }();
	std::lock_guard<std::mutex> g(g_free_mu);
	if (park && g_coder_calls > 0) {
		g_deferred.emplace_back(p, pinned);
		g_parked++;
		return hipSuccess;
	}
	return free_now(p, pinned);
}

}  // namespace

namespace ric {

CoderCall::CoderCall()
{
	std::lock_guard<std::mutex> g(g_free_mu);
	g_coder_calls++;
}

CoderCall::~CoderCall()
{
	std::lock_guard<std::mutex> g(g_free_mu);
	if (--g_coder_calls > 0) return;
	for (auto& d : g_deferred) (void)free_now(d.first, d.second);
	g_deferred.clear();
}

hipError_t dev_free(void* p) { return free_or_park(p, false); }
hipError_t pinned_free(void* p) { return free_or_park(p, true); }

long deferred_frees()
{
	std::lock_guard<std::mutex> g(g_free_mu);
	return g_parked;
}

}  // namespace ric

struct ric_comm {
	ncclComm_t comm = nullptr;
	hipStream_t st = nullptr;
	int device = 0, nranks = 1, rank = 0;
	double* d_red = nullptr;                        // allreduce scratch
	int red_n = 0;
};

extern "C" {

int ric_device_alloc(int device, size_t bytes, void** out)
{
	if (!out) return RIC_E_ARG;
	*out = nullptr;
	if (int rc = on_device(device)) return rc;
	if (bytes == 0) bytes = 16;
	const hipError_t e = hipMalloc(out, bytes);
	if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
		(void)hipGetLastError();
		set_last_error("hipMalloc: out of device memory (" + std::to_string(bytes) + " bytes)");
		*out = nullptr;
		return RIC_E_CAPACITY;
	}
	DCHK(e);
	return RIC_OK;
}

int ric_device_free(void* p)
{
	if (p) DCHK(dev_free(p));
	return RIC_OK;
}

int ric_host_alloc(size_t bytes, void** out)
{
	if (!out) return RIC_E_ARG;
	*out = nullptr;
	DCHK(hipHostMalloc(out, bytes ? bytes : 16, 0));
	return RIC_OK;
}

int ric_host_free(void* p)
{
	if (p) DCHK(pinned_free(p));
	return RIC_OK;
}

int ric_device_copy(int device, void* dst, const void* src, size_t bytes, int kind)
{
	if ((!dst || !src) && bytes) return RIC_E_ARG;
	if (kind != RIC_COPY_H2D && kind != RIC_COPY_D2H && kind != RIC_COPY_D2D) return RIC_E_ARG;
	if (!bytes) return RIC_OK;
	if (int rc = on_device(device)) return rc;
	const hipMemcpyKind k = kind == RIC_COPY_H2D ? hipMemcpyHostToDevice
	                        : kind == RIC_COPY_D2H ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice;
	Aux& a = g_aux[device % kMaxDev];
	std::lock_guard<std::mutex> g(a.mu);
	if (int rc = aux_ready(a)) return rc;
	DCHK(hipMemcpyAsync(dst, src, bytes, k, a.st));
	DCHK(hipStreamSynchronize(a.st));
	return RIC_OK;
}

int ric_device_memset(int device, void* p, int value, size_t bytes)
{
	if (!p && bytes) return RIC_E_ARG;
	if (!bytes) return RIC_OK;
	if (int rc = on_device(device)) return rc;
	Aux& a = g_aux[device % kMaxDev];
	std::lock_guard<std::mutex> g(a.mu);
	if (int rc = aux_ready(a)) return rc;
	DCHK(hipMemsetAsync(p, value, bytes, a.st));
	DCHK(hipStreamSynchronize(a.st));
	return RIC_OK;
}

int ric_device_sync(int device)
{
	if (int rc = on_device(device)) return rc;
	DCHK(hipDeviceSynchronize());
	return RIC_OK;
}

int ric_device_digests(int device, const uint8_t* base, int n, const size_t* off, const size_t* len,
                       unsigned long long* host_out)
{
	if (n < 0 || (n && (!base || !off || !len || !host_out))) return RIC_E_ARG;
	if (!n) return RIC_OK;
	if (int rc = on_device(device)) return rc;
	Aux& a = g_aux[device % kMaxDev];
	std::lock_guard<std::mutex> g(a.mu);
	if (int rc = aux_ready(a)) return rc;
	for (int i0 = 0; i0 < n; i0 += kDigestRuns) {
		const int m = std::min(kDigestRuns, n - i0);
		DCHK(hipMemsetAsync(a.d_dig, 0, sizeof(unsigned long long) * (size_t)m, a.st));
		launch_digests(base, off + i0, len + i0, m, a.d_dig, a.st);
		DCHK(hipGetLastError());
		DCHK(hipMemcpyAsync(a.h_dig, a.d_dig, sizeof(unsigned long long) * (size_t)m, hipMemcpyDeviceToHost, a.st));
		DCHK(hipStreamSynchronize(a.st));
		memcpy(host_out + i0, a.h_dig, sizeof(unsigned long long) * (size_t)m);
	}
	return RIC_OK;
}

int ric_host_digests(const uint8_t* base, int n, const size_t* off, const size_t* len, unsigned long long* out)
{
	if (n < 0 || (n && (!base || !off || !len || !out))) return RIC_E_ARG;
	for (int i = 0; i < n; i++) out[i] = host_digest(base + off[i], len[i]);
	return RIC_OK;
}

int ric_device_pack_h2d(int device, uint8_t* dst, int n, const uint8_t* const* src, const size_t* len, const size_t* off,
                        unsigned long long* dig_out)
{
	if (n < 0 || (n && (!dst || !src || !len || !off))) return RIC_E_ARG;
	size_t total = 0;
	for (int i = 0; i < n; i++) {
		if (len[i] && !src[i]) return RIC_E_ARG;
		total = std::max(total, off[i] + len[i]);
	}
	if (!n) return RIC_OK;
	if (int rc = on_device(device)) return rc;
	Aux& a = g_aux[device % kMaxDev];
	std::lock_guard<std::mutex> g(a.mu);
	if (int rc = aux_ready(a)) return rc;
	if (int rc = aux_stage(a, total)) return rc;
	// the runs into pinned staging (the gaps zeroed: the payload is shipped
	// whole), each run's digest taken from its source on the way
	size_t at = 0;
	std::vector<int> ord(n);
	for (int i = 0; i < n; i++) ord[i] = i;
	std::sort(ord.begin(), ord.end(), [&](int x, int y) { return off[x] < off[y]; });
	for (int i : ord) {
		if (off[i] > at) memset(a.h_stage + at, 0, off[i] - at);
		memcpy(a.h_stage + off[i], src[i], len[i]);
		if (dig_out) dig_out[i] = host_digest(src[i], len[i]);
		at = std::max(at, off[i] + len[i]);
	}
	DCHK(hipMemcpyAsync(dst, a.h_stage, total, hipMemcpyHostToDevice, a.st));
	DCHK(hipStreamSynchronize(a.st));
	return RIC_OK;
}

// ------------------------------------------------------------------ ric_comm
int ric_comm_unique_id(uint8_t* id, size_t len)
{
	if (!id || len < NCCL_UNIQUE_ID_BYTES) return RIC_E_ARG;
	ncclUniqueId u;
	NCHK(ncclGetUniqueId(&u));
	memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
	return RIC_OK;
}

int ric_comm_create(ric_comm** out, const uint8_t* id, int nranks, int rank, int device)
{
	if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return RIC_E_ARG;
	*out = nullptr;
	if (int rc = on_device(device)) return rc;
	ric_comm* c = new ric_comm;
	c->device = device; c->nranks = nranks; c->rank = rank;
	ncclUniqueId u;
	memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
	if (dfail(side_stream_create(&c->st), "hipStreamCreate") ||
	    nfail(ncclCommInitRank(&c->comm, nranks, u, rank), "ncclCommInitRank")) {
		ric_comm_destroy(c);
		return RIC_E_HIP;
	}
	*out = c;
	return RIC_OK;
}

void ric_comm_destroy(ric_comm* c)
{
	if (!c) return;
	(void)hipSetDevice(c->device);
	if (c->st) (void)hipStreamSynchronize(c->st);
	if (c->comm) (void)ncclCommDestroy(c->comm);
	if (c->d_red) (void)dev_free(c->d_red);
	if (c->st) (void)hipStreamDestroy(c->st);
	delete c;
}

int ric_comm_allreduce_f64(ric_comm* c, double* vals, int n, int op)
{
	if (!c || !vals || n < 1 || op < 0 || op > 2) return RIC_E_ARG;
	DCHK(hipSetDevice(c->device));
	if (c->red_n < n) {
		if (c->d_red) DCHK(dev_free(c->d_red));
		c->d_red = nullptr;
		DCHK(hipMalloc(&c->d_red, sizeof(double) * (size_t)n));
		c->red_n = n;
	}
	DCHK(hipMemcpyAsync(c->d_red, vals, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, c->st));
	const ncclRedOp_t o = op == RIC_RED_SUM ? ncclSum : op == RIC_RED_MAX ? ncclMax : ncclMin;
	NCHK(ncclAllReduce(c->d_red, c->d_red, (size_t)n, ncclFloat64, o, c->comm, c->st));
	DCHK(hipMemcpyAsync(vals, c->d_red, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, c->st));
	DCHK(hipStreamSynchronize(c->st));
	return RIC_OK;
}

int ric_comm_sendrecv(ric_comm* c, int nops, const int* peer, const int* is_send, void* const* buf, const size_t* bytes)
{
	if (!c || nops < 0 || (nops && (!peer || !is_send || !buf || !bytes))) return RIC_E_ARG;
	for (int i = 0; i < nops; i++)
		if (peer[i] < 0 || peer[i] >= c->nranks || (bytes[i] && !buf[i])) return RIC_E_ARG;
	if (!nops) return RIC_OK;
	DCHK(hipSetDevice(c->device));
	NCHK(ncclGroupStart());
	ncclResult_t r = ncclSuccess;
	for (int i = 0; i < nops && r == ncclSuccess; i++) {
		if (!bytes[i]) continue;
		r = is_send[i] ? ncclSend(buf[i], bytes[i], ncclUint8, peer[i], c->comm, c->st)
		               : ncclRecv(buf[i], bytes[i], ncclUint8, peer[i], c->comm, c->st);
	}
	const ncclResult_t r2 = ncclGroupEnd();
	if (nfail(r, "ncclSend/ncclRecv") || nfail(r2, "ncclGroupEnd")) return RIC_E_HIP;
	DCHK(hipStreamSynchronize(c->st));
	return RIC_OK;
}

}  // extern "C"
