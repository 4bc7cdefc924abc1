// sdz_runtime.cpp -- the C ABI of libsdz.so (include/sdz.h): argument checks,
// device scratch pools, kernel-timing events and the host-copy convenience paths.
// No codec runs on the CPU here: every entry point launches the HIP kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "sdz_internal.h"
#include "runtime.h"

#define FB_SLOT_BYTES (64 + 2048)            // k_deflate.hip FB_SLOT: a record-path block slot

using namespace sdz;

namespace sdz {
namespace rt {

thread_local std::string g_err;
// bumped by every device allocation or free of the pools: free_hbm()'s cached value is stale then
static std::atomic<unsigned> g_hbm_epoch{0};
std::recursive_mutex g_dev_mu[kMaxDev];
Pool g_host;
Pinned g_pinned;
Pinned g_plan_pinned;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(SDZ_API_HIP_ERROR, std::string(what) + ": " + hipGetErrorString(e));
}

int ensure_device() {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(SDZ_API_NO_DEVICE, "no HIP device available (libsdz has no CPU codec path)");
    return SDZ_API_OK;
}

int cur_device(int* d) {
    HIPCHK(hipGetDevice(d));
    if (*d < 0 || *d >= kMaxDev) return fail(SDZ_API_BAD_ARG, "device index out of range");
    return SDZ_API_OK;
}

namespace {
struct DeferredEv {
    hipEvent_t ev;
    hipStream_t s;
    bool* pending;
};
thread_local int t_defer_depth = 0;
thread_local bool t_defer_synced = false;
thread_local hipStream_t t_defer_s = nullptr;
thread_local std::vector<DeferredEv> t_deferred;
// record a queued event now (a get() of its slot)
void defer_take(hipEvent_t ev) {
    for (size_t i = 0; i < t_deferred.size(); ++i)
        if (t_deferred[i].ev == ev) {
            (void)hipEventRecord(ev, t_deferred[i].s);
            t_deferred.erase(t_deferred.begin() + (long)i);
            return;
        }
}
bool defer_put(hipEvent_t ev, hipStream_t s, bool* pending) {
    if (!t_defer_depth || s != t_defer_s) return false;
    defer_take(ev);                                   // (one entry per event: the later use wins)
    t_deferred.push_back({ev, s, pending});
    return true;
}
}  // namespace

DeferScope::DeferScope(hipStream_t s) {
    if (t_defer_depth++ == 0) {
        t_defer_s = s;
        t_defer_synced = false;
    }
}
DeferScope::~DeferScope() {
    if (--t_defer_depth) return;
    if (t_defer_synced) {
        for (const DeferredEv& d : t_deferred) *d.pending = false;
        t_deferred.clear();
    } else {
        flush();
    }
}
void DeferScope::flush() {
    for (const DeferredEv& d : t_deferred) (void)hipEventRecord(d.ev, d.s);
    t_deferred.clear();
}
void DeferScope::synced() { t_defer_synced = true; }

int Pool::get(size_t bytes, hipStream_t s, void** out, Slot** slot) {
    int d = 0;
    if (int rc = cur_device(&d)) return rc;
    Slot& S = slots[d];
    if (!S.ev) HIPCHK(hipEventCreateWithFlags(&S.ev, hipEventDisableTiming));
    if (S.pending) defer_take(S.ev);
    if (S.p && S.cap < bytes) {
        if (S.pending) HIPCHK(hipEventSynchronize(S.ev));
        HIPCHK(hipFree(S.p));
        S.p = nullptr;
        S.cap = 0;
        S.pending = false;
        g_hbm_epoch.fetch_add(1);
    }
    if (!S.p) {
        size_t want = std::max(bytes, (size_t)1 << 20);
        g_hbm_epoch.fetch_add(1);
        hipError_t e = hipMalloc(&S.p, want);
        if (e != hipSuccess) { S.p = nullptr; return hip_fail(e, "hipMalloc(scratch)"); }
        S.cap = want;
    }
    if (S.pending) HIPCHK(hipStreamWaitEvent(s, S.ev, 0));
    // SDZ_POISON=1 (development aid): every get() hands out its bytes as 0xA5, so a kernel that reads
    // pool memory it has not written in this call reads the same wrong value from the first call on
    static const bool poison = getenv("SDZ_POISON") && *getenv("SDZ_POISON") == '1';
    if (poison) HIPCHK(hipMemsetAsync(S.p, 0xA5, bytes, s));
    *slot = &S;
    *out = S.p;
    return SDZ_API_OK;
}

int Pool::done(Slot* S, hipStream_t s) {
    S->pending = true;
    if (defer_put(S->ev, s, &S->pending)) return SDZ_API_OK;
    HIPCHK(hipEventRecord(S->ev, s));
    return SDZ_API_OK;
}

int Pinned::get(size_t bytes, void** out, bool wait, hipStream_t busy) {
    int d = 0;
    if (int rc = cur_device(&d)) return rc;
    if (pending[d] && (wait || cap[d] < bytes)) {
        defer_take(ev[d]);
        HIPCHK(hipEventSynchronize(ev[d]));
        pending[d] = false;
    }
    if (cap[d] < bytes) {
        // (busy: the caller's own copies from the old buffer may still be in flight on that stream,
        // not yet covered by a done() event)
        if (p[d] && busy) HIPCHK(hipStreamSynchronize(busy));
        if (p[d]) HIPCHK(hipHostFree(p[d]));
        p[d] = nullptr;
        cap[d] = 0;
        const size_t want = std::max(bytes, (size_t)1 << 20);
        HIPCHK(hipHostMalloc(&p[d], want, hipHostMallocDefault));
        cap[d] = want;
    }
    *out = p[d];
    return SDZ_API_OK;
}

thread_local hipEvent_t g_ev0 = nullptr, g_ev1 = nullptr;
thread_local bool g_ev_pending = false;
thread_local float g_extra_ms = 0.f;    // GPU time of the last call outside g_ev0..g_ev1 (split pre-pass)
int g_timing = 0;

void timing_begin(hipStream_t s) {
    if (!g_timing) return;
    g_extra_ms = 0.f;
    if (!g_ev0) { hipEventCreate(&g_ev0); hipEventCreate(&g_ev1); }
    hipEventRecord(g_ev0, s);
}
void timing_end(hipStream_t s) {
    if (!g_timing) return;
    hipEventRecord(g_ev1, s);
    g_ev_pending = true;
}

uint32_t* pinned_words() {
    struct W {
        uint32_t* p = nullptr;
        ~W() { if (p) (void)hipHostFree(p); }
    };
    static thread_local W w;
    if (!w.p && hipHostMalloc((void**)&w.p, 64, hipHostMallocDefault) != hipSuccess) w.p = nullptr;
    return w.p;
}

int Pinned::done(hipStream_t s) {
    int d = 0;
    if (int rc = cur_device(&d)) return rc;
    if (!ev[d]) HIPCHK(hipEventCreateWithFlags(&ev[d], hipEventDisableTiming));
    pending[d] = true;
    if (defer_put(ev[d], s, &pending[d])) return SDZ_API_OK;
    HIPCHK(hipEventRecord(ev[d], s));
    return SDZ_API_OK;
}

}  // namespace rt
uint32_t* rt_pinned_words() { return rt::pinned_words(); }
}  // namespace sdz

using namespace sdz::rt;

namespace {

thread_local float g_last_ms = 0.f;
thread_local float g_breakdown[3] = { 0.f, 0.f, 0.f };   // decode / resolve / finalize of the last inflate

Pool g_inflate_scratch, g_deflate_state, g_tmp, g_stage, g_split, g_find;
// g_tmp layout: [0, 64) a device max / sum, [64, 128) the dictionary's adler32 (DICTID),
// [128, 256) small results, then the file name
constexpr size_t kTmpMax = 0, kTmpDictId = 64, kTmpFname = 256;
constexpr uint64_t kInflaterOutCap = 4ull << 20;   // sdz_inflater: output slot per device call
constexpr uint64_t kLzSmallMax = 1024;              // deflate L4-9: inputs up to this size take the lane parse
constexpr uint64_t kSideMin = 4ull << 20;           // deflate: the input checksum on the side stream from this total
constexpr uint64_t kDeflaterRedo = 8;             // sdz_deflater: record mode while redone bytes <= 8 x input
constexpr uint64_t kDeflaterRedoFloor = 64ull << 20;  //   + 64 MiB, then serial
constexpr size_t kInflaterOnePassMin = 32u << 10;  // sdz_inflater: a first append this long tries the one-pass path
constexpr bool kMatch4Default = false;           // deflate levels 4-9: the 4-byte chain search (SDZ_MATCH4)

const char* const kZmsg[ZM_COUNT] = {
    "",
    "invalid gzip id",
    "unknown compression method",
    "invalid window size",
    "incorrect header check",
    "need dictionary",
    "invalid block type",
    "invalid stored block lengths",
    "too many length or distance symbols",
    "invalid bit length repeat",
    "oversubscribed dynamic bit lengths tree",
    "incomplete dynamic bit lengths tree",
    "oversubscribed literal/length tree",
    "incomplete literal/length tree",
    "oversubscribed distance tree",
    "incomplete distance tree",
    "empty distance tree with lengths",
    "invalid distance code",
    "invalid literal/length code",
};

// one-shot device checksum of a device buffer, blocking (the host checksum entry points)
int device_checksum(const uint8_t* d_buf, uint64_t len, int kind, int32_t seed, int32_t* out,
                    hipStream_t s) {
    void* tmp = nullptr;
    int32_t res = 0;
    {
        PoolUse use(g_tmp, s);
        if (int rc = use.get(kTmpFname, &tmp)) return rc;
        int32_t* d_res = (int32_t*)((uint8_t*)tmp + kTmpDictId);
        launch_checksum_one(d_buf, len, kind, seed, d_res, s);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(&res, d_res, sizeof res, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    *out = res;
    return SDZ_API_OK;
}

}  // namespace

extern "C" {

const char* sdz_last_error(void) { return sdz::rt::g_err.c_str(); }
int sdz_version(void) { return SDZ_ABI_VERSION; }

int sdz_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int sdz_set_device(int device) {
    HIPCHK(hipSetDevice(device));
    return SDZ_API_OK;
}

const char* sdz_zmsg(int32_t code) { return (code >= 0 && code < ZM_COUNT) ? kZmsg[code] : ""; }

void* sdz_device_alloc(uint64_t bytes) {
    if (ensure_device()) return nullptr;
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 1);
    if (e != hipSuccess) { hip_fail(e, "hipMalloc"); return nullptr; }
    return p;
}
void sdz_device_free(void* ptr) { if (ptr) hipFree(ptr); }
int sdz_copy_to_device(void* dst, const void* src, uint64_t bytes) {
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return SDZ_API_OK;
}
int sdz_copy_to_host(void* dst, const void* src, uint64_t bytes) {
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return SDZ_API_OK;
}
int sdz_memset_device(void* dst, int value, uint64_t bytes) {
    HIPCHK(hipMemset(dst, value, bytes));
    return SDZ_API_OK;
}
int sdz_copy_device_to_device(void* dst, const void* src, uint64_t bytes) {
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToDevice));
    return SDZ_API_OK;
}
int sdz_sync(void* stream) {
    if (stream) { HIPCHK(hipStreamSynchronize((hipStream_t)stream)); }
    else { HIPCHK(hipDeviceSynchronize()); }
    return SDZ_API_OK;
}
void* sdz_stream_create(void) {
    if (ensure_device()) return nullptr;
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e != hipSuccess) { hip_fail(e, "hipStreamCreate"); return nullptr; }
    return (void*)s;
}
int sdz_stream_destroy(void* stream) {
    if (!stream) return fail(SDZ_API_BAD_ARG, "sdz_stream_destroy: null stream");
    HIPCHK(hipStreamDestroy((hipStream_t)stream));
    return SDZ_API_OK;
}
int sdz_set_timing(int enabled) { g_timing = enabled; return SDZ_API_OK; }
int sdz_last_kernel_breakdown(float* ms3) {
    if (!ms3) return fail(SDZ_API_BAD_ARG, "sdz_last_kernel_breakdown: null pointer");
    ms3[0] = g_breakdown[0]; ms3[1] = g_breakdown[1]; ms3[2] = g_breakdown[2];
    return SDZ_API_OK;
}
float sdz_last_kernel_ms(void) {
    if (g_ev_pending) {
        hipEventSynchronize(g_ev1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, g_ev0, g_ev1);
        g_last_ms = ms + g_extra_ms;
        g_ev_pending = false;
    }
    return g_last_ms;
}

// ----------------------------------------------------------------- inflate

}  // extern "C"

namespace {

// Free HBM of the current device, for sizing scratch: hipMemGetInfo is a driver query (tens of
// microseconds, a visible share of a small call's latency), so its value is kept per device for
// up to 50 ms; the pools this library grows in between are a small part of 288 GB.
size_t free_hbm() {
    static std::mutex mu;
    static size_t val[kMaxDev] = {};
    static double at[kMaxDev] = {};
    static unsigned ep[kMaxDev] = {};
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= kMaxDev) d = 0;
    const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    const unsigned e = g_hbm_epoch.load();
    std::lock_guard<std::mutex> lk(mu);
    // re-read after 50 ms, or once a pool of this process allocated or freed since (another
    // process's allocations are seen within the 50 ms)
    if (val[d] == 0 || t - at[d] > 50.0 || ep[d] != e) {
        size_t f = 0, tot = 0;
        val[d] = hipMemGetInfo(&f, &tot) == hipSuccess ? f : 16ull << 30;
        at[d] = t;
        ep[d] = e;
    }
    return val[d];
}

// Scratch of one inflate call: per-stream code lengths, then (one-shot) decode and resolve
// state, the token ring (round_tokens per stream; C2's streams finish in one round),
// ntok / flags / the active counter, and `extra` bytes for the caller (incremental staging).
// Fills the round machinery of `a`; returns the extra region or an error via rc.
int inflate_scratch(InflateArgs& a, uint32_t n, bool own_state, size_t extra, hipStream_t s,
                    PoolUse& use, uint8_t** extra_out) {
    const uint64_t dsb = inflate_dsave_bytes(), rsb = inflate_rsave_bytes();
    // tokens per stream per round: as many as a quarter of free HBM (at most 32 GiB) allows,
    // up to 128 Ki; SDZ_ROUND_TOKENS overrides
    const size_t mem_free = free_hbm();
    uint64_t budget = std::min<uint64_t>(32ull << 30, mem_free / 4);
    // the wave decoder's provisional slots (below) come out of the same quarter
    const uint64_t wdp_bytes = own_state && a.wave ? (uint64_t)n * kWdProvTokens * 4 : 0;
    budget = budget > 2 * wdp_bytes ? budget - wdp_bytes : budget / 2;
    uint64_t want = 1u << 17;
    if (const char* e = getenv("SDZ_ROUND_TOKENS")) want = strtoull(e, nullptr, 10);
    uint32_t T = (uint32_t)std::min<uint64_t>(want, std::max<uint64_t>(1024, budget / (4ull * n)));
    T = std::max<uint32_t>(64, T & ~31u);
    const size_t off_ds = (size_t)n * kInflateScratchPerStream;
    const size_t off_rs = off_ds + (own_state ? (size_t)n * dsb : 0);
    const size_t off_tk = (off_rs + (own_state ? (size_t)n * rsb : 0) + 255) & ~(size_t)255;
    const size_t off_nt = off_tk + (size_t)n * T * 4;
    // the wave decoder's provisional tokens (one-shot calls): each lane's chunk is decoded into a
    // slot of its own there and compacted into the token ring after the iteration's join
    const bool wdp = own_state && a.wave;
    const size_t off_wp = (off_nt + (size_t)n * 8 + 256 + 255) & ~(size_t)255;
    const size_t off_ex = (off_wp + (wdp ? (size_t)n * kWdProvTokens * 4 : 0) + 255) & ~(size_t)255;
    void* scratch = nullptr;
    if (int rc = use.get(off_ex + extra, &scratch)) {
        // no room for the wave decoder's slots: the lane decoder (which needs none) takes the call
        if (!wdp || inflate_wdec_mode() == 1) return rc;
        (void)hipGetLastError();                          // (the failed hipMalloc's error)
        a.wave = 0;
        return inflate_scratch(a, n, own_state, extra, s, use, extra_out);
    }
    uint8_t* base = (uint8_t*)scratch;
    // SDZ_POISON_SCRATCH=<bits> (development aid): parts of the layout handed out as 0xA5 bytes --
    // 1 code-length scratch, 2 DSave, 4 RSave, 8 token rings, 16 ntok / flags / active, 32 wave slots
    if (const char* e = getenv("SDZ_POISON_SCRATCH")) {
        const unsigned bits = (unsigned)strtoul(e, nullptr, 0);
        const size_t part[6][2] = { { 0, off_ds }, { off_ds, own_state ? (size_t)n * dsb : 0 },
                                    { off_rs, own_state ? (size_t)n * rsb : 0 }, { off_tk, (size_t)n * T * 4 },
                                    { off_nt, (size_t)n * 8 + 256 }, { off_wp, wdp ? (size_t)n * kWdProvTokens * 4 : 0 } };
        for (int k = 0; k < 6; ++k)
            if ((bits >> k) & 1u && part[k][1]) HIPCHK(hipMemsetAsync(base + part[k][0], 0xA5, part[k][1], s));
    }
    a.scratch = base;
    if (own_state) { a.dsave = base + off_ds; a.rsave = base + off_rs; }
    a.tokens = (uint32_t*)(base + off_tk);
    a.round_tokens = T;
    a.ntok = (uint32_t*)(base + off_nt);
    a.flags = a.ntok + n;
    a.active = a.flags + n;
    a.wdprov = wdp ? (uint32_t*)(base + off_wp) : nullptr;
    if (extra_out) *extra_out = base + off_ex;
    return SDZ_API_OK;
}

// timing_started: the call's timing events were started by an earlier attempt (the wave decoder's,
// handed back with kWdRestart), whose decode time g_restart_ms is added to this run's breakdown
thread_local float g_restart_ms = 0.f;
int inflate_run(InflateArgs& a, hipStream_t s, bool timing_started = false, int (*hook)(void*) = nullptr,
                void* hook_ctx = nullptr) {
    static thread_local uint32_t host_active_pageable = 0;
    uint32_t* const pw = pinned_words();
    uint32_t& host_active = pw ? pw[0] : host_active_pageable;
    a.dbg = nullptr;
    const bool phases = getenv("SDZ_PHASE_TIMING") != nullptr;   // development aid
    if (phases) {
        HIPCHK(hipMalloc(&a.dbg, 64 * sizeof(unsigned long long)));
        HIPCHK(hipMemsetAsync(a.dbg, 0, 64 * sizeof(unsigned long long), s));
    }
    if (!timing_started) { timing_begin(s); g_restart_ms = 0.f; }
    if (int rc = run_inflate_rounds(a, s, &host_active, g_timing ? g_breakdown : nullptr, hook, hook_ctx)) {
        if (a.dbg) { (void)hipFree(a.dbg); a.dbg = nullptr; }
        if (rc == kWdRestart) {                          // the caller starts over; timing goes on
            g_restart_ms = g_timing ? g_breakdown[0] : 0.f;
            return rc;
        }
        g_restart_ms = 0.f;
        return rc > 0 ? rc : hip_fail(hipGetLastError(), "inflate rounds");
    }
    if (g_timing) g_breakdown[0] += g_restart_ms;
    g_restart_ms = 0.f;
    timing_end(s);
    if (phases) {
        unsigned long long h[64];
        HIPCHK(hipMemcpyAsync(h, a.dbg, sizeof h, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        fprintf(stderr, "sdz phases:");
        for (int k = 0; k < 32; ++k) fprintf(stderr, " %llu", h[k]);
        fprintf(stderr, "\n");
        hipFree(a.dbg);
    }
    HIPCHK(hipGetLastError());
    return SDZ_API_OK;
}

// Block-parallel decode of long streams (k_split.hip): when a batch holds streams much longer
// than its median, their block starts are found, their blocks decoded as segments (one lane
// each) and chained back in order, before the rounds; the rounds then feed their tokens to
// the resolve phase.  Which streams: those of compressed size >= a threshold t (>= 16 KiB,
// SDZ_SPLIT_MIN) chosen by split_threshold's cost model; SDZ_SPLIT_SHARE=x forces t = x times
// the batch's bytes per decoder lane, SDZ_SPLIT=0 turns splitting off.  Returns 0 with
// plan.nsplit == 0 when nothing is split.
// per device: the side stream the segments decode on (overlapping the first round's decode
// of the other streams) and its completion event
struct SideStream { hipStream_t s = nullptr; hipEvent_t ev = nullptr; };
SideStream g_side[kMaxDev];
int side_stream(SideStream** out) {
    int d = 0;
    if (int rc = cur_device(&d)) return rc;
    SideStream& S = g_side[d];
    if (!S.s) HIPCHK(hipStreamCreateWithFlags(&S.s, hipStreamNonBlocking));
    if (!S.ev) HIPCHK(hipEventCreateWithFlags(&S.ev, hipEventDisableTiming));
    *out = &S;
    return SDZ_API_OK;
}
// The first round's decode takes about
//   finder(split bytes) + max(longest unsplit stream / lane rate, longest segment / lane rate,
//                             all bytes / full-chip rate)
// (the segments decode while the unsplit streams do; a lane decodes its stream serially, and
// at 64 Ki busy lanes the chip is at its aggregate rate).  The rates are measured figures:
// ~2.5 MB/s of input per lane, ~220 GB/s of input for the chip (C2), ~130 GB/s for the
// finder (C4); segments are blocks (~30 KB on zlib output; 32 KB fitted to C4's measured
// optimum).  The threshold minimising this
// over the batch's own sizes is taken (none when splitting does not pay: a batch of equal
// streams, C2).
uint64_t split_threshold(std::vector<uint64_t> len, uint64_t split_min) {
    const double r_lane = 2.5e6, r_chip = 220e9, r_find = 130e9, seg_max = 32768;
    std::sort(len.begin(), len.end());
    uint64_t total = 0;
    for (uint64_t x : len) total += x;
    const double floor_t = (double)total / r_chip;
    const size_t n = len.size();
    double best = std::max((double)len[n - 1] / r_lane, floor_t);   // nothing split
    uint64_t thr = ~0ull;
    double suffix = 0;
    for (size_t k = n; k-- > 0;) {                       // split streams k .. n-1 (t = len[k])
        suffix += (double)len[k];
        if (len[k] < split_min) break;
        if (k > 0 && len[k - 1] == len[k]) continue;      // equal sizes split together: at the run's first
        const double unsplit = k ? (double)len[k - 1] / r_lane : 0.0;
        const double t = suffix / r_find + std::max(std::max(unsplit, seg_max / r_lane), floor_t);
        if (t < best) { best = t; thr = len[k]; }
    }
    return thr;
}

// What the split pre-pass keeps between its two halves (inflate_split_start before the
// first round, inflate_split_finish from inside it, run_inflate_rounds' hook).
struct SplitHost {
    SplitPlan plan{};
    uint32_t* split_state = nullptr;
    InflateArgs a{};                                     // the call's arguments (input, scratch)
    hipStream_t s = nullptr;
    SideStream* side = nullptr;
    std::vector<SplitInfo> sp;
    uint64_t lanes = 0;
    uint32_t ns = 0, scap = 0;
    size_t cand_bytes = 0;
    SplitInfo* d_sp1 = nullptr;
    uint64_t *d_cand1 = nullptr, *d_surv = nullptr;
    uint32_t *d_nsurv = nullptr, *d_npacked = nullptr;
    PoolUse* seg_use = nullptr;                          // the segments' pool (used on the side stream)
};

// Half 1, before the first round: which streams split (their split_state PENDING, so the
// first round's decode skips them), and the finder launched on the side stream -- it runs
// while the first round decodes the other streams.  SDZ_SPLIT=0 turns splitting off.
int inflate_split_start(const InflateArgs& a, hipStream_t s, PoolUse& find_use, SplitHost& H) {
    const uint32_t n = a.n;
    if (const char* e = getenv("SDZ_SPLIT")) if (atoi(e) == 0) return SDZ_API_OK;
    if (a.wave) return SDZ_API_OK;                       // the wave decoder is parallel inside a block
    uint64_t split_min = 16 << 10;
    if (const char* e = getenv("SDZ_SPLIT_MIN")) split_min = strtoull(e, nullptr, 10);
    std::vector<uint64_t> len(n);
    if (a.host_len) {
        std::copy(a.host_len, a.host_len + n, len.begin());
    } else {
        HIPCHK(hipMemcpyAsync(len.data(), a.in_len, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    uint64_t thr = 0;
    if (const char* e = getenv("SDZ_SPLIT_SHARE")) {
        uint64_t total = 0;
        for (uint64_t x : len) total += x;
        thr = std::max<uint64_t>(split_min, (uint64_t)(atof(e) * (double)(total / 65536)));
    } else {
        thr = split_threshold(len, split_min);
    }
    if (getenv("SDZ_SPLIT_DEBUG")) fprintf(stderr, "sdz split: threshold %llu\n", (unsigned long long)thr);
    H.sp.clear();
    H.lanes = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (len[i] < thr || len[i] > (1ull << 32)) continue;
        SplitInfo x{};
        x.sid = i;
        x.nbits = len[i] * 8;
        x.lane0 = H.lanes;
        H.lanes += (x.nbits + 31) / 32;
        H.sp.push_back(x);
    }
    if (H.sp.empty()) return SDZ_API_OK;
    const uint32_t ns = (uint32_t)H.sp.size();
    H.ns = ns;
    H.a = a;
    H.s = s;
    // the finder's scratch (filter survivors: ~0.1 % of positions on zlib output; room for
    // 0.2 %, and a stream's candidates beyond that are only lost parallelism) and the
    // per-stream split_state
    H.cand_bytes = (size_t)ns * SP_CAND_MAX * sizeof(uint64_t);
    H.scap = (uint32_t)std::min<uint64_t>(1u << 30, std::max<uint64_t>(SPLIT_FILTER_BLOCKS * 16, H.lanes * 32 / 512));
    const size_t b1 = ns * sizeof(SplitInfo) + H.cand_bytes + (size_t)H.scap * sizeof(uint64_t) +
                      SPLIT_FILTER_BLOCKS * sizeof(uint32_t) + 256 + (size_t)n * sizeof(uint32_t);
    void* p1 = nullptr;
    if (int rc = find_use.get(b1, &p1)) return rc;
    uint8_t* d1 = (uint8_t*)p1;
    H.d_sp1 = (SplitInfo*)d1;
    H.d_cand1 = (uint64_t*)(d1 + ns * sizeof(SplitInfo));
    H.d_surv = H.d_cand1 + (size_t)ns * SP_CAND_MAX;
    H.d_nsurv = (uint32_t*)(H.d_surv + H.scap);
    H.d_npacked = H.d_nsurv + SPLIT_FILTER_BLOCKS;
    H.split_state = H.d_npacked + 64;
    {
        std::vector<uint32_t> st(n, 0u);
        for (const SplitInfo& x : H.sp) st[x.sid] = SPS_PENDING;
        HIPCHK(hipMemcpyAsync(H.split_state, st.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(H.d_sp1, H.sp.data(), ns * sizeof(SplitInfo), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemsetAsync(H.d_nsurv, 0, SPLIT_FILTER_BLOCKS * sizeof(uint32_t), s));
        HIPCHK(hipStreamSynchronize(s));                 // (host vectors are copy sources)
    }
    if (int rc = side_stream(&H.side)) return rc;
    HIPCHK(hipEventRecord(H.side->ev, s));               // (the side stream sees the copies above)
    HIPCHK(hipStreamWaitEvent(H.side->s, H.side->ev, 0));
    launch_split_find(a.in, a.in_off, H.d_sp1, ns, H.d_cand1, H.lanes, H.d_surv, H.d_nsurv, H.scap, H.side->s);
    // (every candidate was a survivor: the survivor list's room holds the packed candidates)
    launch_split_pack(H.d_sp1, ns, H.d_cand1, H.d_surv, H.d_npacked, H.side->s);
    HIPCHK(hipGetLastError());
    if (getenv("SDZ_DEBUG_SYNC") && hipStreamSynchronize(H.side->s) != hipSuccess)   // (development)
        return fail(SDZ_API_HIP_ERROR, "debug sync: split finder");
    H.plan.nsplit = ns;
    return SDZ_API_OK;
}

// Half 2, from run_inflate_rounds right after the first round's decode is queued: the
// candidates come back (the host waits on the side stream only), the segments are planned
// -- the stream's start, then one per candidate; token capacity from the bits to the next
// candidate (1 token per 6 bits; a segment that fills up sends its stream to the serial
// path) -- and decoded on the side stream, one lane each, in one round; plan.ready marks
// their end (run_inflate_rounds waits for it before chaining).
int inflate_split_finish(void* ctx) {
    SplitHost& H = *(SplitHost*)ctx;
    const uint32_t ns = H.ns;
    hipStream_t ss = H.side->s;
    uint32_t npacked = 0;
    HIPCHK(hipMemcpyAsync(H.sp.data(), H.d_sp1, ns * sizeof(SplitInfo), hipMemcpyDeviceToHost, ss));
    HIPCHK(hipMemcpyAsync(&npacked, H.d_npacked, sizeof npacked, hipMemcpyDeviceToHost, ss));
    HIPCHK(hipStreamSynchronize(ss));
    std::vector<uint64_t> packed(npacked);
    if (npacked) {
        HIPCHK(hipMemcpyAsync(packed.data(), H.d_surv, npacked * sizeof(uint64_t), hipMemcpyDeviceToHost, ss));
        HIPCHK(hipStreamSynchronize(ss));
    }
    if (getenv("SDZ_SPLIT_DEBUG")) {
        std::vector<uint32_t> nsv(SPLIT_FILTER_BLOCKS);
        HIPCHK(hipMemcpyAsync(nsv.data(), H.d_nsurv, nsv.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, ss));
        HIPCHK(hipStreamSynchronize(ss));
        uint64_t tsv = 0, tc = 0, over = 0, full = 0;
        for (uint32_t x : nsv) { tsv += x; full += x == H.scap / SPLIT_FILTER_BLOCKS; }
        for (const SplitInfo& x : H.sp) { tc += x.ncand; over += x.ncand > SP_CAND_MAX; }
        fprintf(stderr, "sdz split: %u streams, %llu bits, %llu survivors (%llu full regions of %u), "
                "%llu candidates, %llu streams over the cap\n", ns, (unsigned long long)(H.lanes * 32),
                (unsigned long long)tsv, (unsigned long long)full, H.scap / SPLIT_FILTER_BLOCKS,
                (unsigned long long)tc, (unsigned long long)over);
    }
    std::vector<SegInfo> seg;
    uint64_t tok = 0;
    uint32_t chain = 0;
    for (uint32_t k = 0; k < ns; ++k) {
        SplitInfo& x = H.sp[k];
        const uint32_t nc = std::min<uint32_t>(x.ncand, SP_CAND_MAX);
        const uint64_t* c = packed.data() + x.cand0;
        x.skip0 = nc && c[0] == 0 ? 1 : 0;
        x.seg0 = (uint32_t)seg.size();
        x.chain0 = chain;
        const bool use = x.ncand <= SP_CAND_MAX;
        const uint32_t m = use ? 1 + nc - x.skip0 : 1;
        x.nseg = m;
        chain += m;
        for (uint32_t j = 0; j < m; ++j) {
            const uint64_t b = j == 0 ? 0 : c[j - 1 + x.skip0];
            const uint64_t e = j + 1 < m ? c[j + x.skip0] : x.nbits;
            SegInfo g{};
            g.bit = b;
            g.tok = tok;
            g.cap = (uint32_t)std::min<uint64_t>(((e - b) / 6 + 1024 + 31) & ~31ull, 1u << 30);
            g.split = k;
            g.stream = x.sid;
            tok += g.cap;
            seg.push_back(g);
        }
    }
    const uint32_t nseg = (uint32_t)seg.size();
    const uint64_t dsb = inflate_dsave_bytes();
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t o = 0;
    const size_t o_sp = o; o = al(o + ns * sizeof(SplitInfo));
    const size_t o_seg = o; o = al(o + nseg * sizeof(SegInfo));
    const size_t o_cand = o; o = al(o + H.cand_bytes);
    const size_t o_chain = o; o = al(o + chain * sizeof(uint32_t));
    const size_t o_ctok = o; o = al(o + chain * sizeof(uint64_t));
    const size_t o_segD = o; o = al(o + nseg * dsb);
    const size_t o_lens = o; o = al(o + nseg * kInflateScratchPerStream);
    const size_t o_nt = o; o = al(o + (2 * (size_t)nseg + 1) * sizeof(uint32_t));
    const size_t o_tok = o; o = al(o + tok * sizeof(uint32_t));
    void* base = nullptr;
    if (int rc = H.seg_use->get(o, &base)) return rc;   // (ordered on the side stream)
    uint8_t* B = (uint8_t*)base;
    H.plan.nseg = nseg;
    H.plan.sp = (SplitInfo*)(B + o_sp);
    H.plan.seg = (SegInfo*)(B + o_seg);
    H.plan.cand = (uint64_t*)(B + o_cand);
    H.plan.chain = (uint32_t*)(B + o_chain);
    H.plan.chain_tok = (uint64_t*)(B + o_ctok);
    H.plan.segtok = (uint32_t*)(B + o_tok);
    HIPCHK(hipMemcpyAsync(H.plan.sp, H.sp.data(), ns * sizeof(SplitInfo), hipMemcpyHostToDevice, ss));
    HIPCHK(hipMemcpyAsync(H.plan.seg, seg.data(), nseg * sizeof(SegInfo), hipMemcpyHostToDevice, ss));
    HIPCHK(hipMemcpyAsync(H.plan.cand, H.d_cand1, H.cand_bytes, hipMemcpyDeviceToDevice, ss));
    HIPCHK(hipStreamSynchronize(ss));                    // (host vectors are copy sources)
    InflateArgs g = H.a;
    g.n = nseg;
    g.dsave = B + o_segD;
    g.scratch = B + o_lens;
    g.ntok = (uint32_t*)(B + o_nt);
    g.flags = g.ntok + nseg;
    g.active = g.flags + nseg;
    g.split_plan = nullptr;
    g.split_state = nullptr;
    g.segmode = 1;
    g.seg = H.plan.seg;
    g.spinfo = H.plan.sp;
    g.cand = H.plan.cand;
    g.segtok = H.plan.segtok;
    launch_seg_decode(g, ss);
    HIPCHK(hipGetLastError());
    if (getenv("SDZ_DEBUG_SYNC") && hipStreamSynchronize(ss) != hipSuccess)            // (development)
        return fail(SDZ_API_HIP_ERROR, "debug sync: segment decode");
    HIPCHK(hipEventRecord(H.side->ev, ss));
    H.plan.segD = g.dsave;
    H.plan.ready = (void*)H.side->ev;
    return SDZ_API_OK;
}

// incremental-mode state slab: DSave[n] | RSave[n] | window[n][32 KiB] | carry[n][CARRY]
struct IStateLayout {
    size_t ds, rs, win, carry, bytes;
    explicit IStateLayout(uint32_t n) {
        ds = 0;
        rs = ((size_t)n * inflate_dsave_bytes() + 255) & ~(size_t)255;
        win = (rs + (size_t)n * inflate_rsave_bytes() + 255) & ~(size_t)255;
        carry = win + (size_t)n * IS_WIN;
        bytes = carry + (size_t)n * SDZ_INFLATE_CARRY;
    }
};
int inflate_append_impl(void* state, const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                        uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap, sdz_inflate_record* rec,
                        uint32_t n, int32_t format, const uint8_t* dict, uint32_t dict_len,
                        const uint64_t* in_total_hint, hipStream_t s);

}  // namespace

extern "C" {

int sdz_inflate_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                             uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap,
                             sdz_inflate_record* rec, uint32_t n, int32_t format,
                             const uint8_t* dict, uint32_t dict_len, void* stream) {
    return rt::inflate_batch_device(in, in_off, in_len, out, out_off, out_cap, rec, n, format, dict, dict_len, stream,
                                    nullptr, nullptr);
}
}  // extern "C"

// host_len / host_cap (optional): the lengths and output capacities on the host too (the
// host-buffer path): no length read-back for the split plan, and when every stream's output
// fits one round's tokens (a token is >= 1 output byte), no active-count read-back either
int rt::inflate_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint8_t* out,
                             const uint64_t* out_off, const uint64_t* out_cap, sdz_inflate_record* rec, uint32_t n,
                             int32_t format, const uint8_t* dict, uint32_t dict_len, void* stream,
                             const uint64_t* host_len, const uint64_t* host_cap, bool host_no_gzip) {
    if (int rc = ensure_device()) return rc;
    if (n == 0) return SDZ_API_OK;
    if (!in || !in_off || !in_len || !out || !out_off || !out_cap || !rec)
        return fail(SDZ_API_BAD_ARG, "sdz_inflate_batch_device: null pointer");
    if (format < SDZ_FMT_AUTO || format > SDZ_FMT_CONTAINER)
        return fail(SDZ_API_BAD_ARG, "sdz_inflate_batch_device: bad format");
    hipStream_t s = (hipStream_t)stream;
    DevLock lk;
    if (lk.rc) return lk.rc;
    InflateArgs a{};
    PoolUse tmp_use(g_tmp, s);
    void* tmp = nullptr;
    if (int rc = tmp_use.get(kTmpFname, &tmp)) return rc;
    if (dict) {                                         // DICTID on the device: no host sync
        int32_t* d_id = (int32_t*)((uint8_t*)tmp + kTmpDictId);
        launch_checksum_one(dict, dict_len, 0, 1, d_id, s);
        a.dict_adler_dev = d_id;
    }
    PoolUse use(g_inflate_scratch, s);
    a.wave = inflate_wave_policy(n, host_len, in_len, s) ? 1u : 0u;
    if (int rc = inflate_scratch(a, n, true, 0, s, use, nullptr)) return rc;
    a.in = in; a.in_off = in_off; a.in_len = in_len;
    a.out = out; a.out_off = out_off; a.out_cap = out_cap;
    a.rec = rec;
    a.dict = dict; a.dict_len = dict_len; a.dict_adler = 1;
    a.n = n; a.format = format;
    a.streaming = 0; a.window = nullptr; a.carry = nullptr;
    a.split_plan = nullptr; a.split_state = nullptr; a.segmode = 0;
    a.host_len = host_len;
    a.one_round = 0;
    a.host_cap_max = 0;
    a.no_gzip = host_no_gzip ? 1u : 0u;
    if (host_len && host_cap) {
        bool one = true;
        uint64_t mx = 1;
        for (uint32_t i = 0; i < n; ++i) {
            one = one && host_cap[i] + 16 <= a.round_tokens && host_len[i] <= (1ull << 28);
            mx = std::max<uint64_t>(mx, host_cap[i]);
        }
        a.one_round = one ? 1u : 0u;
        a.host_cap_max = mx;
    }
    bool restarted = false;
    if (a.wave) {
        const int rw = inflate_run(a, s, false, nullptr, nullptr);
        if (rw != kWdRestart) return rw;
        a.wave = 0;                                       // many small blocks: lane decoder + split
        restarted = true;
    }
    PoolUse find_use(g_find, s);
    SplitHost sh;
    if (int rc = inflate_split_start(a, s, find_use, sh)) return rc;
    // the segments' pool is used on the side stream (its reuse waits there)
    PoolUse split_use(g_split, sh.side ? sh.side->s : s);
    sh.seg_use = &split_use;
    if (sh.plan.nsplit) { a.split_plan = &sh.plan; a.split_state = sh.split_state; }
    int rc = inflate_run(a, s, restarted, sh.plan.nsplit ? inflate_split_finish : nullptr, &sh);
    if (sh.plan.nsplit) {
        // every exit: the main stream waits for the side stream's work, and the side stream
        // (where the segments' pool is released) for the main stream's rounds
        (void)hipEventRecord(sh.side->ev, sh.side->s);
        (void)hipStreamWaitEvent(s, sh.side->ev, 0);
        (void)hipEventRecord(sh.side->ev, s);
        (void)hipStreamWaitEvent(sh.side->s, sh.side->ev, 0);
    }
    return rc;
}

extern "C" {

uint64_t sdz_inflate_state_bytes(uint32_t n) { return IStateLayout(n).bytes; }

int sdz_inflate_state_reset_device(void* state, uint32_t n, void* stream) {
    if (int rc = ensure_device()) return rc;
    if (n == 0) return SDZ_API_OK;
    if (!state) return fail(SDZ_API_BAD_ARG, "sdz_inflate_state_reset_device: null state");
    IStateLayout L(n);
    launch_istate_reset((uint8_t*)state + L.ds, (uint8_t*)state + L.rs, n, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return SDZ_API_OK;
}

int sdz_inflate_append_batch_device(void* state, const uint8_t* in, const uint64_t* in_off,
                                    const uint64_t* in_len, uint8_t* out, const uint64_t* out_off,
                                    const uint64_t* out_cap, sdz_inflate_record* rec, uint32_t n,
                                    int32_t format, const uint8_t* dict, uint32_t dict_len,
                                    void* stream) {
    if (int rc = ensure_device()) return rc;
    if (n == 0) return SDZ_API_OK;
    if (!state || !in || !in_off || !in_len || !out || !out_off || !out_cap || !rec)
        return fail(SDZ_API_BAD_ARG, "sdz_inflate_append_batch_device: null pointer");
    if (format != SDZ_FMT_RAW && format != SDZ_FMT_CONTAINER)
        return fail(SDZ_API_BAD_ARG, "sdz_inflate_append_batch_device: format must be RAW or CONTAINER");
    return inflate_append_impl(state, in, in_off, in_len, out, out_off, out_cap, rec, n, format, dict, dict_len,
                               nullptr, (hipStream_t)stream);
}

}  // extern "C"

namespace {
// The incremental call.  Staging: carry ++ chunk per stream, each stream its own slot of
// SDZ_INFLATE_CARRY + in_len + 64 bytes (k_stage_slots: prefix sums on the device), so one
// long chunk does not size every stream's slot.  The total comes from the host when the
// caller knows it (in_total_hint: sdz_inflater_append), else from one device sum.
int inflate_append_impl(void* state, const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                        uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap, sdz_inflate_record* rec,
                        uint32_t n, int32_t format, const uint8_t* dict, uint32_t dict_len,
                        const uint64_t* in_total_hint, hipStream_t s) {
    DevLock lk;
    if (lk.rc) return lk.rc;
    IStateLayout SL(n);
    InflateArgs a{};
    PoolUse tmp_use(g_tmp, s);
    void* tmp = nullptr;
    if (int rc = tmp_use.get(kTmpFname, &tmp)) return rc;
    uint64_t total = 0;
    if (in_total_hint) total = *in_total_hint;
    else if (device_sum_u64(in_len, n, (unsigned long long*)((uint8_t*)tmp + kTmpMax), &total, s))
        return hip_fail(hipGetLastError(), "inflate append: input sizes");
    if (dict) {
        int32_t* d_id = (int32_t*)((uint8_t*)tmp + kTmpDictId);
        launch_checksum_one(dict, dict_len, 0, 1, d_id, s);
        a.dict_adler_dev = d_id;
    }
    a.dsave = (uint8_t*)state + SL.ds;
    a.rsave = (uint8_t*)state + SL.rs;
    a.window = (uint8_t*)state + SL.win;
    a.carry = (uint8_t*)state + SL.carry;
    a.streaming = 1;
    a.n = n; a.format = format;
    a.dict = dict; a.dict_len = dict_len; a.dict_adler = 1;
    // (256-aligned: the slot offsets and lengths follow it as u64 arrays)
    const size_t stage_bytes = ((size_t)n * (SDZ_INFLATE_CARRY + 64 + 255) + total + 256 + 255) & ~(size_t)255;
    PoolUse use(g_inflate_scratch, s);
    uint8_t* ex = nullptr;
    if (int rc = inflate_scratch(a, n, false, stage_bytes + 16 * (size_t)n + 64, s, use, &ex)) return rc;
    uint8_t* stage = ex;
    uint64_t* st_off = (uint64_t*)(ex + stage_bytes);
    uint64_t* st_len = st_off + n;
    launch_istate_stage(a, in, in_off, in_len, stage, st_off, st_len, s);
    if (getenv("SDZ_CHECK_STAGE")) {                    // development aid: staged runs inside the region
        std::vector<uint64_t> o(n), l(n);
        HIPCHK(hipMemcpyAsync(o.data(), st_off, n * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(l.data(), st_len, n * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        fprintf(stderr, "sdz stage: n %u total %llu stage_bytes %zu base %p ex %p T %u st0 %llu/%llu\n", n,
                (unsigned long long)total, stage_bytes, (void*)a.scratch, (void*)ex, a.round_tokens,
                (unsigned long long)o[0], (unsigned long long)l[0]);
        for (uint32_t i = 0; i < n; ++i)
            if (o[i] + l[i] + 64 > stage_bytes) return fail(SDZ_API_BAD_ARG, "stage check: stream " + std::to_string(i));
        if (getenv("SDZ_CHECK_STAGE")[0] == 's') return fail(SDZ_API_BAD_ARG, "stage check: stopped before decode");
    }
    a.in = stage; a.in_off = st_off; a.in_len = st_len;
    a.out = out; a.out_off = out_off; a.out_cap = out_cap;
    a.rec = rec;
    return inflate_run(a, s);
}
}  // namespace

extern "C" {

// ----------------------------------------------------------------- deflate

uint64_t sdz_deflate_bound(uint64_t in_len, int32_t format, uint32_t fname_len) {
    // stored-block worst case (5 bytes per <= 16383-symbol block at most) + trees + container
    uint64_t blocks = in_len / 16000 + 2;
    uint64_t b = in_len + blocks * 5 + in_len / 8 + 1024;
    if (format == SDZ_DEFLATE_ZLIB) b += 10;              // 78 20 + DICTID with a dictionary
    if (format == SDZ_DEFLATE_GZIP) b += 18 + fname_len + 1;
    return (b + 7) & ~7ull;
}

int sdz_deflate_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                             uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap,
                             sdz_deflate_record* rec, uint32_t n, int32_t level, int32_t format,
                             const uint8_t* fname, uint32_t fname_len, uint32_t mtime,
                             const uint8_t* dict, uint32_t dict_len, void* stream) {
    return rt::deflate_batch_device(in, in_off, in_len, out, out_off, out_cap, rec, n, level, format, fname, fname_len,
                                    mtime, dict, dict_len, stream, nullptr);
}
}  // extern "C"

// host_len (optional): the n input lengths on the host too (the host-buffer path knows
// them), which spares the plan's device-to-host read and its wait
int rt::deflate_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint8_t* out,
                             const uint64_t* out_off, const uint64_t* out_cap, sdz_deflate_record* rec, uint32_t n,
                             int32_t level, int32_t format, const uint8_t* fname, uint32_t fname_len, uint32_t mtime,
                             const uint8_t* dict, uint32_t dict_len, void* stream, const uint64_t* host_len,
                             uint32_t noflush, const int32_t* cks_in, const DeflateExt* ext) {
    if (int rc = ensure_device()) return rc;
    if (n == 0) return SDZ_API_OK;
    if (level < 1 || level > 9) return fail(SDZ_API_BAD_ARG, "level must be between 1 and 9, inclusive");
    if (format < SDZ_DEFLATE_RAW || format > SDZ_DEFLATE_GZIP)
        return fail(SDZ_API_BAD_ARG, "container must be one of `raw`, `deflate`, `gzip`");
    if (!in || !in_off || !in_len || !out || !out_off || !out_cap || !rec)
        return fail(SDZ_API_BAD_ARG, "sdz_deflate_batch_device: null pointer");
    if (dict && format != SDZ_DEFLATE_ZLIB)
        return fail(SDZ_API_BAD_ARG, "Can only provide a dictionary for `deflate` containers.");
    hipStream_t s = (hipStream_t)stream;
    DevLock lk;
    if (lk.rc) return lk.rc;
    // per-stream state slabs: process in sub-batches so the pool stays bounded
    const uint64_t slab = deflate_state_bytes();
    const size_t mem_free = free_hbm();
    void* tmp = nullptr;
    PoolUse tmp_use(g_tmp, s);
    if (int rc = tmp_use.get(kTmpFname + fname_len + 64, &tmp)) return rc;
    int32_t* d_dictid = nullptr;
    if (dict) {                                   // DICTID on the device: no host sync
        d_dictid = (int32_t*)((uint8_t*)tmp + kTmpDictId);
        launch_checksum_one(dict, dict_len, 0, 1, d_dictid, s);
    }
    // Record path (inputs up to kDeflateRecMax = 1 GiB, no dictionary -- it moves the
    // window): hash chains and match records per position found in parallel before the
    // parse (k_deflate.hip).  The host plans it from the input sizes: each stream's record /
    // link range, block slots, chain units and match segments, cut into sub-batches that
    // fit half of free HBM.  Streams off the path run the serial kernel.
    // Levels 1-3 take it with the segment-parallel parse only (their chains need its rounds of
    // inserted positions, k_deflate.hip): for streams over 256 KiB, or batches up to 64 MiB --
    // a large batch of short streams keeps every lane of the serial kernel busy, which beats
    // the rounds (C3 shape at L1: 0.80 s serial, 6.8 s in rounds).
    const bool fastlv = level <= 3;
    const bool lz_on = !getenv("SDZ_SERIAL_PARSE");
    const bool recpath = (!fastlv || lz_on) && !dict;
    std::vector<uint64_t> len(recpath ? n : 0);
    if (recpath && host_len) {
        std::copy(host_len, host_len + n, len.begin());
    } else if (recpath) {
        HIPCHK(hipMemcpyAsync(len.data(), in_len, (size_t)n * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    uint64_t tot_all = 0;
    for (uint32_t i = 0; i < (recpath ? n : 0); ++i)
        if (len[i] > 0 && len[i] <= kDeflateRecMax) tot_all += len[i];
    auto on_path = [&](uint32_t i) {
        if (!recpath || len[i] == 0 || len[i] > kDeflateRecMax) return false;
        return !fastlv || len[i] > (256u << 10) || tot_all <= (64ull << 20);
    };
    // the parse of levels 4-9: segment-parallel (k_lz_*, segments of 2^lz_shift positions,
    // shorter when the batch is small so one long stream still spreads over many lanes) unless
    // a lane per stream finishes first -- it runs as long as the longest stream (~0.6 us per
    // byte), the segments as long as the whole batch (~13.5 ms per GiB): C3 38.6 vs 58 ms
    uint32_t lz_shift = 0;
    if (recpath && lz_on) {
        uint64_t tot = 0, mx = 0;
        for (uint32_t i = 0; i < n; ++i)
            if (on_path(i)) { tot += len[i]; mx = std::max<uint64_t>(mx, len[i]); }
        lz_shift = 9;
        while (lz_shift < 12 && (tot >> (lz_shift + 1)) >= 65536) ++lz_shift;
        // small batches (one buffer of a few hundred KB): down to 128-position segments while
        // there are fewer than 4,096 (deflate(paradiselost.txt) L6: 2^9 1.33 ms, 2^8 1.27,
        // 2^7 1.23, 2^6 1.27)
        if (!fastlv) while (lz_shift > 7 && (tot >> lz_shift) < 4096) --lz_shift;
        if (fastlv) lz_shift = std::max(7u, lz_shift - 2);      // deflate_fast: its state is the position alone
        else if (tot >= (mx << 15) && !noflush && !ext) lz_shift = 0;
        // a few short inputs (the drop-in's deflate() of a small buffer): one parse launch in
        // place of the segment parse's seven, which set such a call's latency; SDZ_LZ_SMALL
        // overrides the byte limit
        uint64_t lz_small = kLzSmallMax;
        if (const char* e = getenv("SDZ_LZ_SMALL")) lz_small = strtoull(e, nullptr, 10);
        if (!fastlv && !noflush && !ext && n <= 256 && mx <= lz_small) lz_shift = 0;
        if (const char* e = getenv("SDZ_LZ_SHIFT"))            // tests: segment size 2^6 .. 2^16
            lz_shift = (uint32_t)std::min(16, std::max(6, atoi(e)));
    }
    // (NO_FLUSH: steps up to lookahead MIN_LOOKAHEAD only, as k_deflate.hip's lz_seg)
    auto lz_segs = [&](uint64_t l) -> uint64_t {
        if (noflush) l = l >= 262 ? l - 261 : 0;
        return lz_shift ? (l + (1ull << lz_shift) - 1) >> lz_shift : 0;
    };
    // levels 4-9 search over 4-byte chains (k_dfl_link4 / k_dfl_match4; SDZ_MATCH4=1 / 0 overrides the default);
    // a Deflater keeps its own records and links between calls and stays on k_dfl_match
    const char* m4e = getenv("SDZ_MATCH4");
    const bool m4_on = m4e ? m4e[0] == '1' : kMatch4Default;
    const bool match4 = recpath && !ext && level >= 4 && m4_on;
    // a stream's first three match segments in one workgroup (not for a Deflater: its list skips
    // the segments final from earlier calls); SDZ_SEG_MERGE=0 turns it off
    const char* sme = getenv("SDZ_SEG_MERGE");
    const bool seg_merge = recpath && !ext && !(sme && sme[0] == '0');
    // k_dfl_match segment size: 16 Ki positions, or for a call whose segments would not fill the
    // chip (one buffer of a few hundred KB: ~30 workgroups on 256 CUs) the power of two >= 2 Ki
    // that gives ~256 of them (each stages its own 32 KiB of history); SDZ_PM_SEG=N forces it
    uint32_t pm_seg = 16384;
    if (recpath && !ext && !match4) {
        const uint64_t want = tot_all / 256;
        while (pm_seg > 2048 && pm_seg / 2 >= want) pm_seg /= 2;
        if (const char* e = getenv("SDZ_PM_SEG")) {
            const uint32_t v = (uint32_t)atoi(e);
            if (v >= 1024 && v <= 16384 && (v & (v - 1)) == 0) pm_seg = v;
        }
    }
    // per position: record 8, link 2, parse words 8 + 4 + 3 bitmaps, 4-byte link 4; per segment 28
    const uint64_t kPosBytes = (lz_shift ? 8 + 2 + 8 + 4 + 1 : 8 + 2) + (match4 ? 4 : 0);
    auto rec_cost = [&](uint32_t i) -> uint64_t {
        if (!on_path(i)) return 0;
        const uint64_t p = (len[i] + 63) & ~63ull;
        return p * kPosBytes + lz_segs(len[i]) * 44 + deflate_rec_blocks(len[i]) * FB_SLOT_BYTES + 64;
    };
    const uint64_t budget = std::max<uint64_t>(1ull << 30, mem_free / 2);
    // sub-batches [cb[j], cb[j + 1])
    std::vector<uint32_t> cb{ 0 };
    {
        uint64_t acc = 0;
        const uint32_t cap = recpath ? 65536u
                                     : (uint32_t)std::max<uint64_t>(1024, std::min<uint64_t>(65536, budget / slab));
        for (uint32_t i = 0; i < n; ++i) {
            const uint64_t c = slab + rec_cost(i) + 64;
            if (i > cb.back() && (acc + c > budget || i - cb.back() >= cap)) { cb.push_back(i); acc = 0; }
            acc += c;
        }
        cb.push_back(n);
    }
    // pool: the largest sub-batch's slabs, record buffers, block slots and plan arrays
    uint64_t pool_bytes = 0;
    for (size_t j = 0; j + 1 < cb.size(); ++j) {
        uint64_t sb = 0, pos = 0, blk = 0, units = 0, segs = 0;
        for (uint32_t i = cb[j]; i < cb[j + 1]; ++i) {
            sb += slab;
            if (on_path(i)) {
                pos += (len[i] + 63) & ~63ull;
                blk += deflate_rec_blocks(len[i]);
                units += deflate_chain_units(len[i]) + deflate_match_segs(len[i], pm_seg);
                segs += lz_segs(len[i]);
            }
        }
        const uint64_t m = cb[j + 1] - cb[j];
        const uint64_t b = sb + pos * kPosBytes + blk * FB_SLOT_BYTES + m * 16 + 8 * (m + 1) + 4 * (m + 1) + 4 * units +
                           (lz_shift ? 4 * (m + 1) + 8 * m + 44 * segs + 24 * 256 : 0) + 4096;
        pool_bytes = std::max(pool_bytes, b);
    }
    void* state = nullptr;
    PoolUse state_use(g_deflate_state, s);
    if (int rc = state_use.get(pool_bytes, &state)) return rc;
    uint8_t* d_fname = nullptr;
    if (fname_len) {
        d_fname = (uint8_t*)tmp + kTmpFname;
        HIPCHK(hipMemcpyAsync(d_fname, fname, fname_len, hipMemcpyHostToDevice, s));
    }
    unsigned long long* dbg = nullptr;
    const bool phases = getenv("SDZ_PHASE_TIMING") != nullptr;   // development aid
    if (phases) {
        HIPCHK(hipMalloc(&dbg, 64 * sizeof(unsigned long long)));
        HIPCHK(hipMemsetAsync(dbg, 0, 64 * sizeof(unsigned long long), s));
    }
    SideStream* side = nullptr;                   // the record path's input checksum runs there
    // (a small call keeps it on its own stream: the fork's event round trips cost more than the
    // overlap saves)
    if (recpath && tot_all >= kSideMin && side_stream(&side) != SDZ_API_OK) side = nullptr;
    timing_begin(s);
    for (size_t j = 0; j + 1 < cb.size(); ++j) {
        const uint32_t b = cb[j], m = cb[j + 1] - cb[j];
        DeflateArgs a{};
        a.dbg = dbg;
        a.in = in; a.in_off = in_off + b; a.in_len = in_len + b;
        a.out = out; a.out_off = out_off + b; a.out_cap = out_cap + b;
        a.rec = rec + b; a.state = (uint8_t*)state;
        a.fast = 0;
        a.dict = dict; a.dict_len = dict_len; a.dict_adler = 1; a.dict_adler_dev = d_dictid;
        a.fname = d_fname; a.fname_len = fname_len; a.mtime = mtime;
        a.n = m; a.level = level; a.format = format;
        a.noflush = noflush; a.cks_in = cks_in;
        if (recpath) {
            // the plan: rp0 / tb0 (m + 1 each), then the unit lists
            std::vector<uint64_t> rp0(m + 1);
            std::vector<uint32_t> tb0(m + 1), units;
            uint64_t pos = 0;
            uint32_t blk = 0, nbmax = 0, nm = 0;
            for (uint32_t k = 0; k < m; ++k) {
                const uint32_t i = b + k;
                tb0[k] = blk;
                if (!on_path(i)) { rp0[k] = ~0ull; continue; }
                rp0[k] = pos;
                pos += (len[i] + 63) & ~63ull;
                const uint32_t nb = (uint32_t)deflate_rec_blocks(len[i]);
                blk += nb;
                nbmax = std::max(nbmax, nb);
                const uint32_t ms = deflate_match_segs(len[i], pm_seg);
                for (uint32_t u = 0; u < ms; ++u) {
                    if (ext && (uint64_t)(u + 1) * 16384 <= ext->rec_from) continue;   // final from earlier calls
                    if (seg_merge && u > 0) continue;    // (second pass below)
                    units.push_back(k << kRecUnitShift | u);
                    ++nm;
                }
            }
            // seg_merge: every stream's segment 0 (covering segments 0-2) first, then segments 3..
            for (uint32_t k = 0; seg_merge && k < m; ++k) {
                if (rp0[k] == ~0ull) continue;
                const uint32_t ms = deflate_match_segs(len[b + k], pm_seg);
                for (uint32_t u = 3; u < ms; ++u) { units.push_back(k << kRecUnitShift | u); ++nm; }
            }
            rp0[m] = pos;
            tb0[m] = blk;
            const uint32_t nmseg = nm;
            for (uint32_t k = 0; k < m; ++k) {
                if (rp0[k] == ~0ull) continue;
                const uint32_t cu = deflate_chain_units(len[b + k]);
                for (uint32_t u = 0; u < cu; ++u) {
                    if (ext && 65536ull + (uint64_t)u * 32768 <= ext->pv_from) continue;
                    units.push_back(k << kRecUnitShift | u);
                }
            }
            // parse segments: sg0 (m + 1), then the stream of each segment
            std::vector<uint32_t> lzs;
            if (lz_shift) {
                lzs.resize(m + 1);
                for (uint32_t k = 0; k < m; ++k) {
                    lzs[k] = (uint32_t)(lzs.size() - (m + 1));
                    if (rp0[k] == ~0ull) continue;
                    const uint64_t K = lz_segs(len[b + k]);
                    for (uint64_t q = 0; q < K; ++q) lzs.push_back(k);
                }
                lzs[m] = (uint32_t)(lzs.size() - (m + 1));
            }
            const uint32_t nlseg = lz_shift ? lzs[m] : 0;
            uint8_t* B = (uint8_t*)state;
            size_t o = (size_t)m * slab;
            auto take = [&](size_t bytes) { uint8_t* p = B + o; o += (bytes + 255) & ~(size_t)255; return p; };
            if (ext) {                                    // a Deflater's own records and links
                a.rec_buf = ext->rec;
                a.qoff = ext->rec_cap;                    // (its quarter words sit past its capacity)
                a.pv_buf = ext->pv;
                a.sym_buf = (uint32_t*)take((size_t)pos * 8);
            } else {
                a.rec_buf = (uint64_t*)take((size_t)pos * 8);
                a.qoff = pos;                             // records [0, pos), quarter words [pos, 2 pos) (u32)
                a.pv_buf = (uint16_t*)take((size_t)pos * 2);
                a.sym_buf = (uint32_t*)a.rec_buf;
                if (match4) a.l4_buf = (uint32_t*)take((size_t)pos * 4);
            }
            a.blk = take((size_t)blk * FB_SLOT_BYTES);
            a.cks = (int32_t*)take((size_t)m * 4);
            // the plan arrays in one region, laid out as in the pinned staging (one copy, below)
            const size_t pb = rp0.size() * 8 + tb0.size() * 4 + units.size() * 4 + lzs.size() * 4;
            uint8_t* d_plan = take(pb);
            uint64_t* d_rp0 = (uint64_t*)d_plan;
            uint32_t* d_tb0 = (uint32_t*)(d_plan + rp0.size() * 8);
            uint32_t* d_units = d_tb0 + tb0.size();
            uint32_t* d_lzs = d_units + units.size();
            if (lz_shift) {
                a.lz_shift = lz_shift;
                a.nlseg = nlseg;
                a.lz_sg0 = d_lzs;
                a.lz_seg = d_lzs + (m + 1);
                a.lz_w = (uint64_t*)take((size_t)pos * 8);
                a.lz_s2 = (uint32_t*)take((size_t)pos * 4);
                a.lz_v1 = (uint64_t*)take((size_t)pos / 8);
                a.lz_e1 = (uint64_t*)take((size_t)pos / 8);
                a.lz_e2 = (uint64_t*)take((size_t)pos / 8);
                a.lz_end = (uint64_t*)take((size_t)nlseg * 8);
                a.lz_carry = (uint64_t*)take((size_t)nlseg * 8);
                a.lz_c = (uint32_t*)take((size_t)nlseg * 4);
                a.lz_cnt = (uint32_t*)take((size_t)nlseg * 4);
                a.lz_fin = (uint32_t*)take((size_t)m * 4);
                if (level <= 3) {
                    a.lz_e1 = a.lz_v1;                  // deflate_fast emits a symbol at every step
                    a.lz_i = (uint64_t*)take((size_t)pos / 8);
                    a.lz_i1 = (uint64_t*)take((size_t)pos / 8);
                    a.lz_i2 = (uint64_t*)take((size_t)pos / 8);
                    a.lz_act = (uint32_t*)take((size_t)m * 4);
                    a.lz_nact = (uint32_t*)take(4);
                    a.fz_rc = (uint32_t*)take((size_t)nlseg * 4);
                    a.fz_chg = (uint32_t*)take((size_t)nlseg * 4);
                    a.fz_fx = (uint32_t*)take((size_t)nlseg * 4);
                }
            }
            if (o > pool_bytes) return fail(SDZ_API_OOM, "deflate: record plan exceeds its pool");
            // plan -> device through the pinned staging buffer (one copy, waited for below)
            void* pin = nullptr;
            if (int rc = g_plan_pinned.get(pb + 64, &pin)) return rc;
            uint8_t* P = (uint8_t*)pin;
            std::memcpy(P, rp0.data(), rp0.size() * 8);
            std::memcpy(P + rp0.size() * 8, tb0.data(), tb0.size() * 4);
            uint8_t* Pu = P + rp0.size() * 8 + tb0.size() * 4;
            if (!units.empty()) std::memcpy(Pu, units.data(), units.size() * 4);
            uint8_t* Pl = Pu + units.size() * 4;
            if (!lzs.empty()) std::memcpy(Pl, lzs.data(), lzs.size() * 4);
            HIPCHK(hipMemcpyAsync(d_plan, P, pb, hipMemcpyHostToDevice, s));
            a.rp0 = d_rp0; a.tb0 = d_tb0;
            a.mseg = d_units; a.nmseg = nmseg;
            a.seg_merge = seg_merge ? 1u : 0u;
            a.pm_seg = pm_seg;
            a.cunit = d_units + nmseg; a.ncunit = (uint32_t)units.size() - nmseg;
            a.nbmax = nbmax;
            a.wide = m <= 256 ? 1u : 0u;                // few streams: the LDS-staged parse
            // the last positions' searches in k_dfl_match's LDS window (its plain walk only: a
            // Deflater's segment list skips final segments, the 4-byte chains have their own)
            a.tail_in_match = !ext && !match4 && !noflush && !getenv("SDZ_TAIL_HBM") ? 1u : 0u;
            if (int rc = g_plan_pinned.done(s)) return rc;   // (the next get() waits for the plan copies)
            launch_deflate(a, s, side ? side->s : nullptr, side ? side->ev : nullptr);
        } else {
            launch_deflate(a, s, nullptr, nullptr);
        }
    }
    timing_end(s);
    if (phases) {
        unsigned long long h[64];
        HIPCHK(hipMemcpyAsync(h, dbg, sizeof h, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        fprintf(stderr, "sdz deflate phases:");
        for (int k = 0; k < 32; ++k) fprintf(stderr, " %llu", h[k]);
        fprintf(stderr, "\n");
        hipFree(dbg);
    }
    HIPCHK(hipGetLastError());
    return SDZ_API_OK;
}
extern "C" {

// ----------------------------------------------------------------- checksums

int sdz_adler32_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                             const int32_t* seed, int32_t* result, uint32_t n, void* stream) {
    if (int rc = ensure_device()) return rc;
    launch_checksum(in, in_off, in_len, seed, result, n, 0, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return SDZ_API_OK;
}

int sdz_crc32_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                           const int32_t* seed, int32_t* result, uint32_t n, void* stream) {
    if (int rc = ensure_device()) return rc;
    launch_checksum(in, in_off, in_len, seed, result, n, 1, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return SDZ_API_OK;
}

// host buffer -> staging pool -> k_checksum; every failure is reported (never a silent 0)
static int host_checksum(const uint8_t* buf, size_t len, int32_t seed, int kind, int32_t* out) {
    if (int rc = ensure_device()) return rc;
    if (!out || (!buf && len)) return fail(SDZ_API_BAD_ARG, "checksum: null pointer");
    DevLock lk;
    if (lk.rc) return lk.rc;
    hipStream_t s = nullptr;
    void* d = nullptr;
    PoolUse use(g_stage, s);
    if (int rc = use.get(len + 64, &d)) return rc;
    if (len) HIPCHK(hipMemcpyAsync(d, buf, len, hipMemcpyHostToDevice, s));
    return device_checksum((const uint8_t*)d, len, kind, seed, out, s);
}

int sdz_adler32_checked(const uint8_t* buf, size_t len, int32_t seed, int32_t* result) {
    return host_checksum(buf, len, seed, 0, result);
}
int sdz_crc32_checked(const uint8_t* buf, size_t len, int32_t seed, int32_t* result) {
    return host_checksum(buf, len, seed, 1, result);
}
int32_t sdz_adler32(const uint8_t* buf, size_t len, int32_t seed) {
    int32_t r = 0;
    return sdz_adler32_checked(buf, len, seed, &r) == SDZ_API_OK ? r : 0;
}
int32_t sdz_crc32(const uint8_t* buf, size_t len, int32_t seed) {
    int32_t r = 0;
    return sdz_crc32_checked(buf, len, seed, &r) == SDZ_API_OK ? r : 0;
}

// ------------------------------------------------------------ incremental deflate

uint64_t sdz_deflate_state_bytes(uint32_t n) { return (uint64_t)n * deflate_state_bytes(); }

uint64_t sdz_deflate_append_bound(uint64_t in_len, int32_t format, uint32_t fname_len) {
    // blocks flushed by one call: this call's input at <= 31 bits per 3-byte match / 9 bits per
    // literal (static trees; dynamic and stored are only chosen when smaller), plus the block
    // pending from earlier calls (<= 16,383 symbols), header and trailer
    return in_len + in_len / 3 + (128u << 10) + 64 + (format == SDZ_DEFLATE_GZIP ? fname_len + 1 : 0);
}

int sdz_deflate_state_reset_device(void* state, uint32_t n, void* stream) {
    if (int rc = ensure_device()) return rc;
    if (n == 0) return SDZ_API_OK;
    if (!state) return fail(SDZ_API_BAD_ARG, "sdz_deflate_state_reset_device: null state");
    launch_deflate_reset((uint8_t*)state, n, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return SDZ_API_OK;
}

int sdz_deflate_append_batch_device(void* state, const uint8_t* in, const uint64_t* in_off,
                                    const uint64_t* in_len, uint8_t* out, const uint64_t* out_off,
                                    const uint64_t* out_cap, sdz_deflate_record* rec, uint32_t n,
                                    int32_t level, int32_t format, const uint8_t* fname,
                                    uint32_t fname_len, uint32_t mtime, const uint8_t* dict,
                                    uint32_t dict_len, int32_t finish, void* stream) {
    if (int rc = ensure_device()) return rc;
    if (n == 0) return SDZ_API_OK;
    if (level < 1 || level > 9) return fail(SDZ_API_BAD_ARG, "level must be between 1 and 9, inclusive");
    if (format < SDZ_DEFLATE_RAW || format > SDZ_DEFLATE_GZIP)
        return fail(SDZ_API_BAD_ARG, "container must be one of `raw`, `deflate`, `gzip`");
    if (!state || !in || !in_off || !in_len || !out || !out_off || !out_cap || !rec)
        return fail(SDZ_API_BAD_ARG, "sdz_deflate_append_batch_device: null pointer");
    if (dict && format != SDZ_DEFLATE_ZLIB)
        return fail(SDZ_API_BAD_ARG, "Can only provide a dictionary for `deflate` containers.");
    hipStream_t s = (hipStream_t)stream;
    DevLock lk;
    if (lk.rc) return lk.rc;
    void* tmp = nullptr;
    PoolUse tmp_use(g_tmp, s);
    if (int rc = tmp_use.get(kTmpFname + fname_len + 64, &tmp)) return rc;
    int32_t* d_dictid = nullptr;
    if (dict) {                                   // DICTID on the device: no host sync
        d_dictid = (int32_t*)((uint8_t*)tmp + kTmpDictId);
        launch_checksum_one(dict, dict_len, 0, 1, d_dictid, s);
    }
    uint8_t* d_fname = nullptr;
    if (fname_len) {
        d_fname = (uint8_t*)tmp + kTmpFname;
        HIPCHK(hipMemcpyAsync(d_fname, fname, fname_len, hipMemcpyHostToDevice, s));
    }
    DeflateArgs a{};
    a.in = in; a.in_off = in_off; a.in_len = in_len;
    a.out = out; a.out_off = out_off; a.out_cap = out_cap;
    a.rec = rec; a.state = (uint8_t*)state;
    a.dict = dict; a.dict_len = dict_len; a.dict_adler = 1; a.dict_adler_dev = d_dictid;
    a.fname = d_fname; a.fname_len = fname_len; a.mtime = mtime;
    a.n = n; a.level = level; a.format = format;
    timing_begin(s);
    launch_deflate_stream(a, finish ? 1u : 0u, s);
    timing_end(s);
    HIPCHK(hipGetLastError());
    if (fname_len) HIPCHK(hipStreamSynchronize(s));     // (the host file name was a copy source)
    return SDZ_API_OK;
}

// ---------------------------------------------------------- fast (not bit-exact) deflate

uint64_t sdz_deflate_fast_bound(uint64_t in_len, int32_t format, uint32_t fname_len) {
    const uint64_t tiles = (in_len + FT_TILE_BYTES - 1) / FT_TILE_BYTES;
    return tiles * (FT_TILE_BYTES + 10) + 18 + fname_len + 1;
}

int sdz_deflate_fast_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                                  uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap,
                                  sdz_deflate_record* rec, uint32_t n, int32_t format,
                                  const uint8_t* fname, uint32_t fname_len, uint32_t mtime, void* stream) {
    if (int rc = ensure_device()) return rc;
    if (n == 0) return SDZ_API_OK;
    if (format < SDZ_DEFLATE_RAW || format > SDZ_DEFLATE_GZIP)
        return fail(SDZ_API_BAD_ARG, "container must be one of `raw`, `deflate`, `gzip`");
    if (!in || !in_off || !in_len || !out || !out_off || !out_cap || !rec)
        return fail(SDZ_API_BAD_ARG, "sdz_deflate_fast_batch_device: null pointer");
    hipStream_t s = (hipStream_t)stream;
    DevLock lk;
    if (lk.rc) return lk.rc;
    // the tiles: which stream, which of its tiles (host plan from the input sizes)
    std::vector<uint64_t> len(n);
    HIPCHK(hipMemcpyAsync(len.data(), in_len, n * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    std::vector<uint32_t> tile0(n), ts, ti;
    for (uint32_t i = 0; i < n; ++i) {
        tile0[i] = (uint32_t)ts.size();
        const uint64_t nt = (len[i] + FT_TILE_BYTES - 1) / FT_TILE_BYTES;
        for (uint64_t k = 0; k < nt; ++k) { ts.push_back(i); ti.push_back((uint32_t)k); }
    }
    const uint32_t ntiles = (uint32_t)ts.size();
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    size_t o = 0;
    const size_t o_tout = o; o = al(o + (size_t)ntiles * FT_TILE_OUT);
    const size_t o_tlen = o; o = al(o + (size_t)ntiles * 4);
    const size_t o_ts = o; o = al(o + (size_t)ntiles * 4);
    const size_t o_ti = o; o = al(o + (size_t)ntiles * 4);
    const size_t o_t0 = o; o = al(o + (size_t)n * 4);
    const size_t o_ck = o; o = al(o + (size_t)n * 4);
    void* base = nullptr;
    PoolUse use(g_deflate_state, s);
    if (int rc = use.get(o + fname_len + 64, &base)) return rc;
    uint8_t* B = (uint8_t*)base;
    uint8_t* d_fname = fname_len ? B + o : nullptr;
    if (ntiles) {
        HIPCHK(hipMemcpyAsync(B + o_ts, ts.data(), ntiles * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(B + o_ti, ti.data(), ntiles * 4, hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipMemcpyAsync(B + o_t0, tile0.data(), n * 4, hipMemcpyHostToDevice, s));
    if (fname_len) HIPCHK(hipMemcpyAsync(d_fname, fname, fname_len, hipMemcpyHostToDevice, s));
    DeflateArgs a{};
    a.in = in; a.in_off = in_off; a.in_len = in_len;
    a.out = out; a.out_off = out_off; a.out_cap = out_cap;
    a.rec = rec; a.n = n; a.level = 6; a.format = format;
    a.fname = d_fname; a.fname_len = fname_len; a.mtime = mtime;
    timing_begin(s);
    launch_checksum(in, in_off, in_len, nullptr, (int32_t*)(B + o_ck), n, format == SDZ_DEFLATE_GZIP ? 1 : 0, s);
    launch_fast_tiles(in, in_off, in_len, (const uint32_t*)(B + o_ts), (const uint32_t*)(B + o_ti), ntiles,
                      B + o_tout, (uint32_t*)(B + o_tlen), s);
    launch_fast_concat(a, (const uint32_t*)(B + o_t0), B + o_tout, (const uint32_t*)(B + o_tlen),
                       (const int32_t*)(B + o_ck), s);
    timing_end(s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));                     // (the host plan vectors are copy sources)
    return SDZ_API_OK;
}

// ----------------------------------------------------------------- one host Inflater

}  // extern "C"

struct sdz_inflater {
    int32_t format = SDZ_FMT_CONTAINER;
    uint8_t* d_state = nullptr;
    uint8_t* d_dict = nullptr;
    uint32_t dict_len = 0;
    uint8_t* d_in = nullptr;
    size_t in_cap = 0;
    uint8_t* d_out = nullptr;
    uint64_t* d_meta = nullptr;                   // in_off, in_len, out_off, out_cap
    sdz_inflate_record* d_rec = nullptr;
    std::vector<uint8_t> out;
    uint64_t in_total = 0;                        // stream bytes passed before this append
    // a first append holding a whole stream went through the one-pass path (block-parallel
    // decode); later appends return its final record again, as the incremental state would
    bool one_pass = false;
    sdz_inflate_record done_rec{};
    uint8_t* d_big = nullptr;
    size_t big_cap = 0;
    ~sdz_inflater() {
        for (void* p : { (void*)d_state, (void*)d_dict, (void*)d_in, (void*)d_out, (void*)d_meta, (void*)d_rec,
                         (void*)d_big })
            if (p) hipFree(p);
    }
};

extern "C" {

sdz_inflater* sdz_inflater_create(int32_t format, const uint8_t* dict, size_t dict_len) {
    if (ensure_device()) return nullptr;
    if (format != SDZ_FMT_RAW && format != SDZ_FMT_CONTAINER) {
        fail(SDZ_API_BAD_ARG, "sdz_inflater_create: format must be RAW or CONTAINER");
        return nullptr;
    }
    sdz_inflater* z = new sdz_inflater;
    z->format = format;
    hipError_t e = hipMalloc(&z->d_state, sdz_inflate_state_bytes(1));
    if (e == hipSuccess) e = hipMalloc(&z->d_out, kInflaterOutCap + 64);
    if (e == hipSuccess) e = hipMalloc(&z->d_meta, 4 * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc(&z->d_rec, sizeof(sdz_inflate_record));
    if (e == hipSuccess && dict) {
        z->dict_len = (uint32_t)dict_len;
        e = hipMalloc(&z->d_dict, dict_len + 64);
        if (e == hipSuccess && dict_len) e = hipMemcpy(z->d_dict, dict, dict_len, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess || sdz_inflate_state_reset_device(z->d_state, 1, nullptr) != SDZ_API_OK) {
        if (e != hipSuccess) hip_fail(e, "sdz_inflater_create");
        delete z;
        return nullptr;
    }
    return z;
}

int sdz_inflater_append(sdz_inflater* z, const uint8_t* data, size_t len, const uint8_t** out,
                        size_t* out_len, sdz_inflate_record* rec) {
    if (!z || !out || !out_len || !rec || (!data && len)) return fail(SDZ_API_BAD_ARG, "sdz_inflater_append: null pointer");
    z->out.clear();
    if (len + 64 > z->in_cap) {
        if (z->d_in) hipFree(z->d_in);
        z->d_in = nullptr;
        z->in_cap = std::max<size_t>(len + 64, 1 << 16);
        HIPCHK(hipMalloc(&z->d_in, z->in_cap));
    }
    if (z->one_pass) {
        *rec = z->done_rec;
        rec->out_len = 0;
        *out = z->out.data();
        *out_len = 0;
        return SDZ_API_OK;
    }
    if (len) HIPCHK(hipMemcpy(z->d_in, data, len, hipMemcpyHostToDevice));
    if (z->in_total == 0 && len >= kInflaterOnePassMin && !getenv("SDZ_INFLATER_STREAM_ONLY")) {
        // The first append, a large one: when the stream ends inside it (one buffer appended
        // whole, the common use) the one-pass path -- block-parallel decode of long streams
        // (k_split.hip) -- gives the same bytes and the same record (its running checksum is
        // counted from the stream start, as an append's from its own output start).  Anything
        // else (the stream continues, an error, output past the slot) leaves no trace: the
        // incremental path below runs as before.
        // Its output slot is only a try: if it cannot be had, the incremental path runs; it is
        // freed on every way out (the bytes are copied to the host on success).
        const uint64_t cap = std::min<uint64_t>((uint64_t)len * 8 + (1u << 20), 1ull << 31);
        uint8_t* big = nullptr;
        if (hipMalloc(&big, cap + 64) != hipSuccess) {
            (void)hipGetLastError();                      // (clear the sticky error: not a failure)
            big = nullptr;
        }
        struct BigFree { uint8_t*& p; ~BigFree() { if (p) hipFree(p); } } bigfree{ big };
        sdz_inflate_record r{};
        r.status = SDZ_INTERNAL;
        if (big) {
            uint64_t meta[4] = { 0, len, 0, cap };
            HIPCHK(hipMemcpy(z->d_meta, meta, sizeof meta, hipMemcpyHostToDevice));
            int rc = sdz_inflate_batch_device(z->d_in, z->d_meta, z->d_meta + 1, big, z->d_meta + 2, z->d_meta + 3,
                                              z->d_rec, 1, z->format, z->d_dict, z->dict_len, nullptr);
            if (rc) return rc;
            HIPCHK(hipMemcpy(&r, z->d_rec, sizeof r, hipMemcpyDeviceToHost));
        }
        if (r.status == SDZ_OK) {
            z->out.resize(r.out_len);
            if (r.out_len) HIPCHK(hipMemcpy(z->out.data(), big, r.out_len, hipMemcpyDeviceToHost));
            z->one_pass = true;
            z->done_rec = r;
            z->in_total += len;
            *rec = r;
            *out = z->out.data();
            *out_len = z->out.size();
            return SDZ_API_OK;
        }
    }
    // more calls while the output slot fills up; each passes the chunk's bytes the device
    // did not take (record in_used: stream offset of the first byte not consumed or held)
    for (uint64_t from = 0;;) {
        uint64_t meta[4] = { from, len - from, 0, kInflaterOutCap };
        HIPCHK(hipMemcpy(z->d_meta, meta, sizeof meta, hipMemcpyHostToDevice));
        const uint64_t hint = len - from;                 // (host-known: no device sum)
        int rc = inflate_append_impl(z->d_state, z->d_in, z->d_meta, z->d_meta + 1, z->d_out, z->d_meta + 2,
                                     z->d_meta + 3, z->d_rec, 1, z->format, z->d_dict, z->dict_len, &hint, nullptr);
        if (rc) return rc;
        HIPCHK(hipMemcpy(rec, z->d_rec, sizeof *rec, hipMemcpyDeviceToHost));
        size_t o = z->out.size();
        z->out.resize(o + rec->out_len);
        if (rec->out_len) HIPCHK(hipMemcpy(z->out.data() + o, z->d_out, rec->out_len, hipMemcpyDeviceToHost));
        const uint64_t sent_end = z->in_total + len;        // stream offset after this chunk
        if (!rec->out_full) break;
        from = len - (sent_end - rec->in_used);
    }
    z->in_total += len;
    *out = z->out.data();
    *out_len = z->out.size();
    return SDZ_API_OK;
}

void sdz_inflater_destroy(sdz_inflater* z) { delete z; }

}  // extern "C"

// A Deflater runs on the record path while it can: every append re-runs the record path
// over all input so far in NO_FLUSH mode (the parse stops where deflate(NO_FLUSH) returns
// NeedMore, only the blocks cut before that are flushed) and returns the bytes past what
// earlier calls returned -- the same bytes the reference's append() returns, since the parse,
// the block cuts and the bit layout do not depend on where earlier calls stopped.  Two cases
// would differ, and switch the Deflater to the serial kernel, replaying every earlier append
// into its state: a block the record path hands back (the pending_buf overlay overtaken,
// SURVEY A7, or a slot overflow), and a call stopping exactly where the window slides one step
// earlier than in one pass (fill_window at strstart = 65274 + 32 Ki e with no more input).
// Dictionaries, inputs past kDeflateRecMax and SDZ_SERIAL_PARSE take the serial kernel from
// the start.
struct sdz_deflater {
    int32_t level = 6, format = SDZ_DEFLATE_ZLIB;
    std::vector<uint8_t> fname;
    uint32_t mtime = 0;
    uint8_t* d_state = nullptr;
    uint8_t* d_dict = nullptr;
    uint32_t dict_len = 0;
    uint8_t* d_in = nullptr;
    size_t in_cap = 0;
    uint8_t* d_out = nullptr;
    size_t out_cap = 0;
    uint64_t* d_meta = nullptr;                   // in_off, in_len, out_off, out_cap
    sdz_deflate_record* d_rec = nullptr;
    std::vector<uint8_t> out;
    // record mode
    bool rec_mode = false;
    int32_t status = 0;                           // 0 nothing appended, 1 appending, 2 finished
    std::vector<uint8_t> hist;                    // every byte appended (the serial replay's source)
    std::vector<size_t> calls;                    // each append's length (the replay's call boundaries)
    uint64_t total = 0, out_done = 0;
    uint64_t redo = 0;                            // input bytes the record-mode calls have processed
    int32_t running = 0;                          // the chunk-wise running checksum
    uint8_t* d_all = nullptr;                     // the input so far, on the device
    size_t all_cap = 0;
    int32_t* d_ck = nullptr;
    std::vector<uint8_t> trailer;                 // a second finish() returns it again
    // the record path's records and links, kept between calls: only the positions the new
    // bytes can change are searched again (records from MIN_LOOKAHEAD before the old end,
    // links from 2 before it)
    uint64_t* d_recs = nullptr;
    uint16_t* d_links = nullptr;
    size_t recs_cap = 0;                          // positions
    ~sdz_deflater() {
        for (void* p : { (void*)d_state, (void*)d_dict, (void*)d_in, (void*)d_out, (void*)d_meta, (void*)d_rec,
                         (void*)d_all, (void*)d_ck, (void*)d_recs, (void*)d_links })
            if (p) hipFree(p);
    }
};

namespace {
// one call of the serial kernel (k_deflate_stream) on the Deflater's device state
int deflater_serial_call(sdz_deflater* z, const uint8_t* data, size_t len, int32_t finish, sdz_deflate_record* rec,
                         bool keep_out) {
    if (len + 64 > z->in_cap) {
        if (z->d_in) hipFree(z->d_in);
        z->d_in = nullptr;
        z->in_cap = std::max<size_t>(len + 64, 1 << 16);
        HIPCHK(hipMalloc(&z->d_in, z->in_cap));
    }
    const uint64_t cap = sdz_deflate_append_bound(len, z->format, (uint32_t)z->fname.size());
    if (cap > z->out_cap) {
        if (z->d_out) hipFree(z->d_out);
        z->d_out = nullptr;
        z->out_cap = cap;
        HIPCHK(hipMalloc(&z->d_out, z->out_cap));
    }
    if (len) HIPCHK(hipMemcpy(z->d_in, data, len, hipMemcpyHostToDevice));
    uint64_t meta[4] = { 0, len, 0, cap };
    HIPCHK(hipMemcpy(z->d_meta, meta, sizeof meta, hipMemcpyHostToDevice));
    int rc = sdz_deflate_append_batch_device(z->d_state, z->d_in, z->d_meta, z->d_meta + 1, z->d_out, z->d_meta + 2,
                                             z->d_meta + 3, z->d_rec, 1, z->level, z->format,
                                             z->fname.empty() ? nullptr : z->fname.data(), (uint32_t)z->fname.size(),
                                             z->mtime, z->d_dict, z->dict_len, finish, nullptr);
    if (rc) return rc;
    HIPCHK(hipMemcpy(rec, z->d_rec, sizeof *rec, hipMemcpyDeviceToHost));
    if (keep_out) {
        z->out.resize(rec->out_len);
        if (rec->out_len) HIPCHK(hipMemcpy(z->out.data(), z->d_out, rec->out_len, hipMemcpyDeviceToHost));
    }
    return SDZ_API_OK;
}

// leave the record path: the serial state after every append so far (their outputs were
// returned already and are not read again)
int deflater_to_serial(sdz_deflater* z, size_t upto_calls) {
    z->rec_mode = false;
    size_t o = 0;
    for (size_t i = 0; i < upto_calls; ++i) {
        sdz_deflate_record r{};
        if (int rc = deflater_serial_call(z, z->hist.data() + o, z->calls[i], 0, &r, false)) return rc;
        o += z->calls[i];
    }
    std::vector<uint8_t>().swap(z->hist);
    std::vector<size_t>().swap(z->calls);
    if (z->d_all) { hipFree(z->d_all); z->d_all = nullptr; z->all_cap = 0; }
    if (z->d_recs) { hipFree(z->d_recs); z->d_recs = nullptr; }
    if (z->d_links) { hipFree(z->d_links); z->d_links = nullptr; }
    z->recs_cap = 0;
    return SDZ_API_OK;
}

// one append / finish on the record path; *how: 0 done, 1 done but later calls run serially
// (the window-slide corner), 2 handed back (nothing changed: the call is to be redone serially)
int deflater_record_call(sdz_deflater* z, const uint8_t* data, size_t len, int32_t finish, sdz_deflate_record* rec,
                         int* how) {
    *how = 0;
    const uint64_t total = z->total + len;
    if (total + 64 > z->all_cap) {
        const size_t cap = std::max<size_t>(std::max<size_t>(total + 64, 2 * z->all_cap), 1 << 16);
        uint8_t* p = nullptr;
        HIPCHK(hipMalloc(&p, cap));
        if (z->total) HIPCHK(hipMemcpy(p, z->d_all, z->total, hipMemcpyDeviceToDevice));
        if (z->d_all) hipFree(z->d_all);
        z->d_all = p;
        z->all_cap = cap;
    }
    if (len) HIPCHK(hipMemcpy(z->d_all + z->total, data, len, hipMemcpyHostToDevice));
    if (!z->d_ck) HIPCHK(hipMalloc(&z->d_ck, 64));
    // the running checksum over this chunk only, seeded with the last (adler32.ts's NMAX
    // quirk applies per chunk, as in sd-deflate.ts:185-190)
    const int kind = z->format == SDZ_DEFLATE_GZIP ? 1 : 0;
    const int32_t seed = z->status == 0 ? (kind ? 0 : 1) : z->running;
    launch_checksum_one(z->d_all + z->total, len, kind, seed, z->d_ck, nullptr);
    HIPCHK(hipGetLastError());
    const uint64_t cap = sdz_deflate_bound(total, z->format, (uint32_t)z->fname.size());
    if (cap > z->out_cap) {
        if (z->d_out) hipFree(z->d_out);
        z->d_out = nullptr;
        z->out_cap = std::max<size_t>(cap, 2 * z->out_cap);
        HIPCHK(hipMalloc(&z->d_out, z->out_cap));
    }
    uint64_t meta[4] = { 0, total, 0, cap };
    HIPCHK(hipMemcpy(z->d_meta, meta, sizeof meta, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(z->d_rec, 0xff, sizeof(sdz_deflate_record)));      // a handed-back stream leaves it so
    const size_t npos = (total + 63) & ~(size_t)63;
    if (npos > z->recs_cap) {                         // grow, keeping what earlier calls found
        const size_t c = std::max<size_t>(npos, 2 * z->recs_cap);
        uint64_t* r = nullptr;
        uint16_t* l = nullptr;
        HIPCHK(hipMalloc(&r, c * 8));
        HIPCHK(hipMalloc(&l, c * 2 + 256));
        if (z->recs_cap) {                            // records at [0, cap), quarter words at [cap, 2 cap) (u32)
            HIPCHK(hipMemcpy(r, z->d_recs, z->recs_cap * 4, hipMemcpyDeviceToDevice));
            HIPCHK(hipMemcpy((uint32_t*)r + c, (const uint32_t*)z->d_recs + z->recs_cap, z->recs_cap * 4,
                             hipMemcpyDeviceToDevice));
            HIPCHK(hipMemcpy(l, z->d_links, z->recs_cap * 2, hipMemcpyDeviceToDevice));
        }
        if (z->d_recs) hipFree(z->d_recs);
        if (z->d_links) hipFree(z->d_links);
        z->d_recs = r; z->d_links = l; z->recs_cap = c;
    }
    const uint64_t old = z->total;
    rt::DeflateExt ext{ z->d_recs, z->d_links, old >= 262 ? old - 262 : 0, old >= 2 ? old - 2 : 0, z->recs_cap };
    int rc = rt::deflate_batch_device(z->d_all, z->d_meta, z->d_meta + 1, z->d_out, z->d_meta + 2, z->d_meta + 3,
                                      z->d_rec, 1, z->level, z->format, z->fname.empty() ? nullptr : z->fname.data(),
                                      (uint32_t)z->fname.size(), z->mtime, nullptr, 0, nullptr, &total,
                                      finish ? 0u : 1u, z->d_ck, &ext);
    if (rc) return rc;
    sdz_deflate_record r{};
    HIPCHK(hipMemcpy(&r, z->d_rec, sizeof r, hipMemcpyDeviceToHost));
    if (r.status != SDZ_OK) { *how = 2; return SDZ_API_OK; }
    if (!finish) {
        // a stop at strstart = 65274 + 32 Ki e: the reference's fill_window slides there
        // (no more input), one pass would a step later -- serial from the next call on
        const uint64_t st = r.reserved;
        if (st >= 65274 && st % 32768 == 32506) *how = 1;
        // tests: leave the record path after this many calls (the replay, exercised)
        if (const char* e = getenv("SDZ_DEFLATER_SWITCH_AT"))
            if (z->calls.size() + 1 >= (size_t)atoi(e)) *how = 1;
    }
    if (r.out_len < z->out_done) return fail(SDZ_API_HIP_ERROR, "deflater: output shrank");
    z->out.resize(r.out_len - z->out_done);
    if (!z->out.empty())
        HIPCHK(hipMemcpy(z->out.data(), z->d_out + z->out_done, z->out.size(), hipMemcpyDeviceToHost));
    z->out_done = r.out_len;
    z->total = total;
    z->running = r.checksum;
    *rec = r;
    rec->out_len = z->out.size();
    rec->reserved = 0;
    return SDZ_API_OK;
}
}  // namespace

extern "C" {

sdz_deflater* sdz_deflater_create(int32_t level, int32_t format, const uint8_t* fname, size_t fname_len,
                                  uint32_t mtime, const uint8_t* dict, size_t dict_len) {
    if (ensure_device()) return nullptr;
    if (level < 1 || level > 9) { fail(SDZ_API_BAD_ARG, "level must be between 1 and 9, inclusive"); return nullptr; }
    if (format < SDZ_DEFLATE_RAW || format > SDZ_DEFLATE_GZIP) {
        fail(SDZ_API_BAD_ARG, "container must be one of `raw`, `deflate`, `gzip`");
        return nullptr;
    }
    if (dict && format != SDZ_DEFLATE_ZLIB) {
        fail(SDZ_API_BAD_ARG, "Can only provide a dictionary for `deflate` containers.");
        return nullptr;
    }
    sdz_deflater* z = new sdz_deflater;
    z->level = level; z->format = format; z->mtime = mtime;
    z->rec_mode = !dict && !getenv("SDZ_SERIAL_PARSE") && !getenv("SDZ_SERIAL_DEFLATER");
    if (fname && fname_len) z->fname.assign(fname, fname + fname_len);
    hipError_t e = hipMalloc(&z->d_state, sdz_deflate_state_bytes(1));
    if (e == hipSuccess) e = hipMalloc(&z->d_meta, 4 * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc(&z->d_rec, sizeof(sdz_deflate_record));
    if (e == hipSuccess && dict) {
        z->dict_len = (uint32_t)dict_len;
        e = hipMalloc(&z->d_dict, dict_len + 64);
        if (e == hipSuccess && dict_len) e = hipMemcpy(z->d_dict, dict, dict_len, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess || sdz_deflate_state_reset_device(z->d_state, 1, nullptr) != SDZ_API_OK) {
        if (e != hipSuccess) hip_fail(e, "sdz_deflater_create");
        delete z;
        return nullptr;
    }
    return z;
}

int sdz_deflater_append(sdz_deflater* z, const uint8_t* data, size_t len, int32_t finish,
                        const uint8_t** out, size_t* out_len, sdz_deflate_record* rec) {
    if (!z || !out || !out_len || !rec || (!data && len)) return fail(SDZ_API_BAD_ARG, "sdz_deflater_append: null pointer");
    z->out.clear();
    *out = z->out.data();
    *out_len = 0;
    if (z->rec_mode && z->total + len > kDeflateRecMax)
        if (int rc = deflater_to_serial(z, z->calls.size())) return rc;
    if (z->rec_mode) {
        // the reference's call protocol (sd-deflate.ts:180-182, 211-214, 232-234), as k_deflate_stream
        sdz_deflate_record r{};
        r.status = SDZ_OK;
        r.checksum = z->running;
        if ((finish && z->status == 0) || (!finish && z->status == 2 && len)) {
            r.status = SDZ_DATA_ERROR;
            *rec = r;
            return SDZ_API_OK;
        }
        if (!finish && len == 0) { *rec = r; return SDZ_API_OK; }
        if (finish && z->status == 2) {                       // deflate(FINISH) again: the trailer again
            z->out = z->trailer;
            *out = z->out.data();
            *out_len = z->out.size();
            *rec = r;
            return SDZ_API_OK;
        }
        // Each record-mode call redoes the parse, the block cuts and the encoding over all the
        // input so far, so many small appends cost O(calls x total).  Once that redone work
        // passes kDeflaterRedo x the input (+ a floor), the Deflater goes serial (linear).
        const uint64_t after = z->total + len;
        uint64_t rfloor = kDeflaterRedoFloor;
        if (const char* e = getenv("SDZ_DEFLATER_REDO_FLOOR")) rfloor = strtoull(e, nullptr, 10);   // tests
        if (!finish && z->redo + after > kDeflaterRedo * after + rfloor) {
            if (int rc = deflater_to_serial(z, z->calls.size())) return rc;
            if (int rc = deflater_serial_call(z, data, len, finish, rec, true)) return rc;
            z->status = 1;
            *out = z->out.data();
            *out_len = z->out.size();
            return SDZ_API_OK;
        }
        int how = 0;
        if (int rc = deflater_record_call(z, data, len, finish, rec, &how)) return rc;
        if (how < 2) z->redo += after;
        if (how < 2) {
            z->hist.insert(z->hist.end(), data, data + len);
            z->calls.push_back(len);
            z->status = finish ? 2 : 1;
            if (finish) {
                const size_t t = z->format == SDZ_DEFLATE_ZLIB ? 4 : z->format == SDZ_DEFLATE_GZIP ? 8 : 0;
                z->trailer.assign(z->out.end() - std::min(t, z->out.size()), z->out.end());
            }
            if (how == 1) {                                   // later calls: serial, from this state
                std::vector<uint8_t> keep;
                keep.swap(z->out);
                if (int rc = deflater_to_serial(z, z->calls.size())) return rc;
                z->out.swap(keep);
            }
            *out = z->out.data();
            *out_len = z->out.size();
            return SDZ_API_OK;
        }
        // handed back: replay the earlier calls into the serial state, then this one
        z->out.clear();
        if (int rc = deflater_to_serial(z, z->calls.size())) return rc;
    }
    if (int rc = deflater_serial_call(z, data, len, finish, rec, true)) return rc;
    *out = z->out.data();
    *out_len = z->out.size();
    return SDZ_API_OK;
}

void sdz_deflater_destroy(sdz_deflater* z) { delete z; }

}  // extern "C"
