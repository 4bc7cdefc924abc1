// runtime.h -- host runtime pieces shared by sdz_runtime.cpp (single-device entry points)
// and sdz_host.cpp (host-buffer batches, multi-GPU, RCCL): error reporting, per-device
// locks and the stream-ordered device pools.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <string>

#include "sdz.h"

namespace sdz {
namespace rt {

int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define HIPCHK(x)                                             \
    do {                                                      \
        hipError_t e_ = (x);                                  \
        if (e_ != hipSuccess) return ::sdz::rt::hip_fail(e_, #x); \
    } while (0)

int ensure_device();
// sdz_inflate_batch_device with the input lengths and output capacities optionally on the host
int inflate_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint8_t* out,
                         const uint64_t* out_off, const uint64_t* out_cap, sdz_inflate_record* rec, uint32_t n,
                         int32_t format, const uint8_t* dict, uint32_t dict_len, void* stream, const uint64_t* host_len,
                         const uint64_t* host_cap, bool host_no_gzip = false);
// a Deflater's own record and link buffers (one stream, positions from 0): records below
// rec_from and links below pv_from are final from earlier calls and not recomputed
struct DeflateExt {
    uint64_t* rec;
    uint16_t* pv;
    uint64_t rec_from, pv_from;
    uint64_t rec_cap;                 // positions the record buffer holds (its quarter words start there)
};
// sdz_deflate_batch_device with the input lengths optionally known on the host
int deflate_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, uint8_t* out,
                         const uint64_t* out_off, const uint64_t* out_cap, sdz_deflate_record* rec, uint32_t n,
                         int32_t level, int32_t format, const uint8_t* fname, uint32_t fname_len, uint32_t mtime,
                         const uint8_t* dict, uint32_t dict_len, void* stream, const uint64_t* host_len,
                         uint32_t noflush = 0, const int32_t* cks_in = nullptr, const DeflateExt* ext = nullptr);

// Calls on one device are serialised (its pools and side stream are shared; recursive: a
// host-batch call holds it around the *_device call it makes); calls on different devices
// run concurrently -- sdz_*_batch_multi drives one host thread per GPU.
constexpr int kMaxDev = 64;
extern std::recursive_mutex g_dev_mu[kMaxDev];
int cur_device(int* d);
struct DevLock {
    std::unique_lock<std::recursive_mutex> lk;
    int rc = SDZ_API_OK;
    DevLock() {
        int d = 0;
        rc = cur_device(&d);
        if (rc == SDZ_API_OK) lk = std::unique_lock<std::recursive_mutex>(g_dev_mu[d]);
    }
};

// Grow-only device scratch, one allocation per (purpose, device).  The *_device entry
// points are asynchronous on the caller's stream, so a pool is stream-ordered: get()
// makes the caller's stream wait for the event recorded after the pool's previous use
// (on whatever stream that was), and done() records that event once this call's work
// is enqueued.  Callers hold their device's lock (DevLock) between get() and done(), and
// take each pool at most once per call.
struct Pool {
    struct Slot {
        void* p = nullptr;
        size_t cap = 0;
        hipEvent_t ev = nullptr;      // recorded after the last enqueued use
        bool pending = false;
    };
    Slot slots[kMaxDev];              // indexed by device id
    int get(size_t bytes, hipStream_t s, void** out, Slot** slot);
    static int done(Slot* S, hipStream_t s);
};
// Deferred done events.  Each hipEventRecord is a marker in the stream, and a marker between two
// launches delayed the second by ~5 us on small calls (rocprofv3 trace, profiles/r05/lat).  While a
// DeferScope is alive on this thread, Pool::done / Pinned::done on its stream queue their event
// instead of recording it; a get() of a slot whose event is queued records it first; the scope's
// flush() (after the call's last launch) and its destructor record the rest.  A later event only
// makes the next user wait longer.
// If the scope's owner synchronises the stream after its last launch (synced()), the queued
// events are dropped instead and their slots marked idle: the work they would mark is done.
struct DeferScope {
    explicit DeferScope(hipStream_t s);
    ~DeferScope();
    static void flush();
    static void synced();
};
// records the pool's event on every exit path once get() succeeded
struct PoolUse {
    Pool& pool;
    hipStream_t s;
    Pool::Slot* slot = nullptr;
    PoolUse(Pool& p, hipStream_t st) : pool(p), s(st) {}
    int get(size_t bytes, void** out) { return pool.get(bytes, s, out, &slot); }
    ~PoolUse() { if (slot) Pool::done(slot, s); }
};
extern Pool g_host;                   // host-buffer batches: staged inputs, outputs, records
// kernel timing (sdz_set_timing): HIP events on the launch stream around a call's kernels
void timing_begin(hipStream_t s);
void timing_end(hipStream_t s);

// pinned host staging, grow-only, one per device (used under the device's lock).  A user that
// leaves copies from it in flight calls done(stream); the next get() waits for them.
struct Pinned {
    void* p[kMaxDev] = {};
    size_t cap[kMaxDev] = {};
    hipEvent_t ev[kMaxDev] = {};
    bool pending[kMaxDev] = {};
    // wait = false: the caller does not write the buffer from the host (only stream-ordered
    // device work does), so the pending copies are not waited for unless it must grow
    // busy: a stream on which this caller's copies from the buffer may still run (a growing get()
    // waits for it before the old buffer is freed)
    int get(size_t bytes, void** out, bool wait = true, hipStream_t busy = nullptr);
    int done(hipStream_t s);
};
// a few pinned host words of this thread for the round drivers' counter read-backs (a copy into
// pageable memory goes through a staging buffer; null if the allocation failed)
uint32_t* pinned_words();
extern Pinned g_pinned;
extern Pinned g_plan_pinned;                      // the deflate plan's staging (beside a host batch's)

}  // namespace rt
}  // namespace sdz
