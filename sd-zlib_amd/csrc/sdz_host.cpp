// sdz_host.cpp -- host-buffer batches, batched span copies, multi-GPU sharding and the RCCL
// communicator of libsdz.so (include/sdz.h).
//
// Host-buffer batches (sdz_inflate_batch / sdz_deflate_batch: what inflate() / deflate() of
// the facade call, sd-inflate.ts:189-228, sd-deflate.ts:263-274) stage through per-device,
// grow-only pools -- a device pool for inputs, outputs and records and a pinned host buffer
// -- so a call makes no hipMalloc / hipFree and no device-wide synchronisation: inputs are
// packed into pinned memory and sent in one copy, the codec runs on the device's stream,
// the records come back in one copy, and the outputs either directly (a few streams) or
// compacted on the device by one k_gather launch and sent back in one copy.
//
// Multi-GPU: streams are independent, so a batch is cut into LPT shards,
// one host thread per GPU runs the host-batch path on its shard, and the fixed-size records
// are all-gathered over RCCL (ncclAllGather; xGMI on MI355X nodes) -- the only collective.
// No codec runs on the CPU here.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <numeric>
#include <queue>
#include <string>
#include <thread>
#include <vector>

#include "runtime.h"
#include "sdz_internal.h"

using namespace sdz;
using namespace sdz::rt;

namespace {

constexpr uint32_t kDirectOut = 32;            // up to this many streams: outputs copied one by one
constexpr uint64_t kPackInMax = 256ull << 20;  // inputs up to this size are packed (pinned, one copy)
constexpr uint64_t kEagerOut = 4ull << 20;     // output slots up to this total come back with the records

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// codec parameters of one host batch (inflate or deflate)
struct Codec {
    bool inflate = true;
    int32_t format = SDZ_FMT_AUTO;
    int32_t level = 6;
    const uint8_t* fname = nullptr;
    uint32_t fname_len = 0;
    uint32_t mtime = 0;
    const uint8_t* dict = nullptr;             // host bytes
    size_t dict_len = 0;
    size_t rec_size() const { return inflate ? sizeof(sdz_inflate_record) : sizeof(sdz_deflate_record); }
};

// What one shard (the streams `ids` of the caller's batch, on the current device) produced.
struct ShardOut {
    std::vector<uint32_t> order;               // caller index of device record k
    void* d_rec = nullptr;                     // device records, rec_cap slots (padding zeroed)
    bool timed = false;                        // kernel_ms wanted (events around the codec's launches)
    float kernel_ms = 0.f;
    uint64_t bytes_in = 0, bytes_out = 0;
};

uint64_t al(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// Run the streams `ids` on the current device: inputs in, codec, outputs back to the caller's
// buffers.  rec_host (nullable) receives each stream's record at its caller index; the device
// records stay in the pool (rec_cap slots) for a gather.  Holds the device's lock.
int host_shard(const uint8_t* const* in, const size_t* in_len, uint8_t* const* out, const size_t* out_cap,
               const std::vector<uint32_t>& ids, uint32_t rec_cap, const Codec& C, void* rec_host, ShardOut& R,
               void* rec_dev = nullptr) {
    DevLock lk;
    if (lk.rc) return lk.rc;
    const uint32_t m = (uint32_t)ids.size();
    const size_t rsz = C.rec_size();
    hipStream_t s = nullptr;
    DeferScope defer(s);                           // the call's done events after its copy back
    R.order = ids;
    if (C.inflate)                                 // longest streams first: a wave decodes similar lengths
        std::stable_sort(R.order.begin(), R.order.end(), [&](uint32_t a, uint32_t b) { return in_len[a] > in_len[b]; });
    // device layout: in | out | compacted out | meta (4 m) | gather meta (3 m) | records | dict
    std::vector<uint64_t> meta(4 * (size_t)m);
    uint64_t ti = 0, to = 0;
    for (uint32_t k = 0; k < m; ++k) {
        const uint32_t i = R.order[k];
        meta[k] = ti; meta[m + k] = in_len[i];
        meta[2 * (size_t)m + k] = to; meta[3 * (size_t)m + k] = out_cap[i];
        ti += al(in_len[i], 16);
        to += al(out_cap[i], 8);
        R.bytes_in += in_len[i];
    }
    const bool compact = m > kDirectOut;
    // in and meta adjacent (one host-to-device copy of both), out and records adjacent (one copy
    // back of both for small outputs): a small call is a few copies and the codec's launches
    size_t o = 0;
    const size_t o_in = o; o = al(o + ti + 128, 256);
    const size_t o_meta = o; o = al(o + 7 * (size_t)m * 8, 256);
    const size_t o_out = o; o = al(o + to + 64, 256);
    const size_t o_rec = o; o = al(o + (size_t)std::max(rec_cap, m) * rsz, 256);
    const size_t o_cmp = o; o = al(o + (compact ? to : 0), 256);
    const size_t o_dict = o; o = al(o + (C.dict ? C.dict_len + 64 : 0), 256);
    void* base = nullptr;
    PoolUse use(g_host, s);
    if (int rc = use.get(o, &base)) return rc;
    uint8_t* B = (uint8_t*)base;
    uint64_t* d_meta = (uint64_t*)(B + o_meta);
    // pinned staging: packed inputs + meta (the outputs reuse it after the records are back)
    const bool pack = ti <= kPackInMax;
    void* pin = nullptr;
    // packed: the staging mirrors the device's [in | meta] (one copy); else the meta alone
    const size_t pin_meta = pack ? o_meta - o_in : 0;
    if (int rc = g_pinned.get(pin_meta + meta.size() * 8 + 64, &pin)) return rc;
    uint8_t* P = (uint8_t*)pin;
    if (pack) {
        for (uint32_t k = 0; k < m; ++k)
            if (in_len[R.order[k]]) std::memcpy(P + meta[k], in[R.order[k]], in_len[R.order[k]]);
    } else {
        for (uint32_t k = 0; k < m; ++k)
            if (in_len[R.order[k]])
                HIPCHK(hipMemcpyAsync(B + o_in + meta[k], in[R.order[k]], in_len[R.order[k]], hipMemcpyHostToDevice, s));
    }
    std::memcpy(P + pin_meta, meta.data(), meta.size() * 8);
    // the staging's done event goes in after the copy back (a marker between the input copy and
    // the first kernel delays that kernel); an error return before it waits for the copies here
    struct SyncOnExit {
        hipStream_t s;
        bool armed = true;
        ~SyncOnExit() { if (armed) (void)hipStreamSynchronize(s); }
    } staged{s};
    if (pack) HIPCHK(hipMemcpyAsync(B + o_in, P, pin_meta + meta.size() * 8, hipMemcpyHostToDevice, s));
    else HIPCHK(hipMemcpyAsync(d_meta, P, meta.size() * 8, hipMemcpyHostToDevice, s));
    uint8_t* d_dict = nullptr;
    if (C.dict) {
        d_dict = B + o_dict;
        if (C.dict_len) HIPCHK(hipMemcpyAsync(d_dict, C.dict, C.dict_len, hipMemcpyHostToDevice, s));
    }
    if (rec_cap > m) HIPCHK(hipMemsetAsync(B + o_rec + (size_t)m * rsz, 0, (size_t)(rec_cap - m) * rsz, s));
    // the shard's kernel-time events (multi-GPU stats only: each is a marker in the stream, and
    // a marker between two launches delayed the second by ~5 us on small calls): made once per
    // thread and device
    static thread_local hipEvent_t evs[kMaxDev][2] = {};
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDev) return fail(SDZ_API_BAD_ARG, "host batch: device index");
    if (R.timed && !evs[dev][0]) { HIPCHK(hipEventCreate(&evs[dev][0])); HIPCHK(hipEventCreate(&evs[dev][1])); }
    hipEvent_t e0 = evs[dev][0], e1 = evs[dev][1];
    if (R.timed) HIPCHK(hipEventRecord(e0, s));
    // no input starts with the gzip magic (or the format is raw): the crc32 finalize is not needed
    bool no_gzip = C.inflate;
    for (uint32_t k = 0; no_gzip && C.format != SDZ_FMT_RAW && k < m; ++k) {
        const uint32_t i = R.order[k];
        no_gzip = in_len[i] < 2 || !(in[i][0] == 0x1f && in[i][1] == 0x8b);
    }
    int rc = C.inflate
        ? rt::inflate_batch_device(B + o_in, d_meta, d_meta + m, B + o_out, d_meta + 2 * (size_t)m,
                                   d_meta + 3 * (size_t)m, (sdz_inflate_record*)(B + o_rec), m, C.format, d_dict,
                                   (uint32_t)C.dict_len, s, meta.data() + m, meta.data() + 3 * (size_t)m, no_gzip)
        : rt::deflate_batch_device(B + o_in, d_meta, d_meta + m, B + o_out, d_meta + 2 * (size_t)m,
                                   d_meta + 3 * (size_t)m, (sdz_deflate_record*)(B + o_rec), m, C.level, C.format,
                                   C.fname, C.fname_len, C.mtime, d_dict, (uint32_t)C.dict_len, s, meta.data() + m);
    if (rc) return rc;
    if (R.timed) HIPCHK(hipEventRecord(e1, s));
    // records back (one copy), then the outputs; small output slots come back with the
    // records, under the same wait (the drop-in's one-buffer calls)
    std::vector<uint8_t> recs((size_t)m * rsz);
    const bool eager = !compact && to <= kEagerOut;
    uint8_t* ebuf = nullptr;
    if (eager) {                                   // outputs and records: one copy
        void* ep = nullptr;
        const size_t nb = o_rec - o_out + recs.size();
        // (written by stream-ordered device work only: no wait for the input copy)
        // (a growing get() first waits for this call's input copy from the staging it replaces)
        if (int rc2 = g_pinned.get(al(nb, 256), &ep, false, s)) return rc2;
        ebuf = (uint8_t*)ep;
        // the bytes written and the records, by a kernel into the mapped staging (a copy engine
        // started ~20 us late on small calls); SDZ_COPY_BACK=0: the whole region by hipMemcpyAsync
        static const bool kb = !getenv("SDZ_COPY_BACK") || atoi(getenv("SDZ_COPY_BACK")) != 0;
        void* dp = nullptr;
        if (kb && hipHostGetDevicePointer(&dp, ep, 0) == hipSuccess && dp) {
            const uint32_t len_off = C.inflate ? (uint32_t)offsetof(sdz_inflate_record, out_len)
                                               : (uint32_t)offsetof(sdz_deflate_record, out_len);
            launch_copy_back((uint8_t*)dp, B + o_out, d_meta + 2 * (size_t)m, d_meta + 3 * (size_t)m, o_rec - o_out,
                             (uint32_t)rsz, len_off, m, s);
            HIPCHK(hipGetLastError());
        } else {
            HIPCHK(hipMemcpyAsync(ebuf, B + o_out, nb, hipMemcpyDeviceToHost, s));
        }
    } else {
        HIPCHK(hipMemcpyAsync(recs.data(), B + o_rec, recs.size(), hipMemcpyDeviceToHost, s));
    }
    // multi-GPU: the records (rec_cap slots, padding zeroed) into the caller's gather slot, which
    // the caller keeps (its own pool use) until the all-gather is done
    if (rec_dev) HIPCHK(hipMemcpyAsync(rec_dev, B + o_rec, (size_t)rec_cap * rsz, hipMemcpyDeviceToDevice, s));
    if (int rc2 = g_pinned.done(s)) return rc2;     // (the next get() waits for the copies above)
    staged.armed = false;
    HIPCHK(hipStreamSynchronize(s));
    if (eager) std::memcpy(recs.data(), ebuf + (o_rec - o_out), recs.size());
    if (R.timed) HIPCHK(hipEventElapsedTime(&R.kernel_ms, e0, e1));
    auto out_len_of = [&](uint32_t k) -> uint64_t {
        const uint8_t* r = recs.data() + (size_t)k * rsz;
        const uint64_t len = C.inflate ? ((const sdz_inflate_record*)r)->out_len : ((const sdz_deflate_record*)r)->out_len;
        return std::min<uint64_t>(len, out_cap[R.order[k]]);
    };
    if (eager) {
        for (uint32_t k = 0; k < m; ++k) {
            const uint64_t len = out_len_of(k);
            R.bytes_out += len;
            if (len && out[R.order[k]]) std::memcpy(out[R.order[k]], ebuf + meta[2 * (size_t)m + k], len);
        }
    } else if (!compact) {
        for (uint32_t k = 0; k < m; ++k) {
            const uint64_t len = out_len_of(k);
            R.bytes_out += len;
            if (len && out[R.order[k]])
                HIPCHK(hipMemcpyAsync(out[R.order[k]], B + o_out + meta[2 * (size_t)m + k], len, hipMemcpyDeviceToHost, s));
        }
        HIPCHK(hipStreamSynchronize(s));
    } else {
        // compact on the device (one k_gather), one copy back, then host copies
        std::vector<uint64_t> gm(3 * (size_t)m);
        uint64_t tot = 0;
        for (uint32_t k = 0; k < m; ++k) {
            const uint64_t len = out_len_of(k);
            gm[k] = tot; gm[m + k] = meta[2 * (size_t)m + k]; gm[2 * (size_t)m + k] = len;
            tot += len;
        }
        R.bytes_out = tot;
        uint64_t* d_gm = d_meta + 4 * (size_t)m;
        if (int rc2 = g_pinned.get(al(tot, 256) + gm.size() * 8, &pin)) return rc2;
        P = (uint8_t*)pin;
        std::memcpy(P + al(tot, 256), gm.data(), gm.size() * 8);
        HIPCHK(hipMemcpyAsync(d_gm, P + al(tot, 256), gm.size() * 8, hipMemcpyHostToDevice, s));
        launch_gather(B + o_cmp, d_gm, B + o_out, d_gm + m, d_gm + 2 * (size_t)m, m, s);
        HIPCHK(hipGetLastError());
        if (tot) HIPCHK(hipMemcpyAsync(P, B + o_cmp, tot, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (uint32_t k = 0; k < m; ++k)
            if (gm[2 * (size_t)m + k] && out[R.order[k]]) std::memcpy(out[R.order[k]], P + gm[k], gm[2 * (size_t)m + k]);
    }
    if (rec_host)
        for (uint32_t k = 0; k < m; ++k)
            std::memcpy((uint8_t*)rec_host + (size_t)R.order[k] * rsz, recs.data() + (size_t)k * rsz, rsz);
    R.d_rec = rec_dev ? rec_dev : B + o_rec;
    DeferScope::synced();                          // (nothing enqueued after the last wait above)
    return SDZ_API_OK;
}

int check_batch(const uint8_t* const* in, const size_t* in_len, uint8_t* const* out, const size_t* out_cap,
                const void* rec, uint32_t n) {
    if (!in || !in_len || !out || !out_cap || !rec) return fail(SDZ_API_BAD_ARG, "host batch: null pointer");
    for (uint32_t i = 0; i < n; ++i)
        if (!in[i] && in_len[i]) return fail(SDZ_API_BAD_ARG, "host batch: null input with a nonzero length");
    return SDZ_API_OK;
}

int host_batch(const uint8_t* const* in, const size_t* in_len, uint8_t* const* out, const size_t* out_cap,
               void* rec, uint32_t n, const Codec& C) {
    if (int rc = ensure_device()) return rc;
    if (n == 0) return SDZ_API_OK;
    if (int rc = check_batch(in, in_len, out, out_cap, rec, n)) return rc;
    std::vector<uint32_t> ids(n);
    std::iota(ids.begin(), ids.end(), 0u);
    ShardOut R;
    return host_shard(in, in_len, out, out_cap, ids, n, C, rec, R);
}

// ------------------------------------------------------------------ multi-GPU

// RCCL communicators of one device list, made once (ncclCommInitAll) and kept
std::mutex g_comm_mu;
std::map<std::vector<int32_t>, std::vector<ncclComm_t>> g_comms;

int comms_for(const std::vector<int32_t>& devs, std::vector<ncclComm_t>** out) {
    std::lock_guard<std::mutex> lk(g_comm_mu);
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
        std::vector<ncclComm_t> c(devs.size());
        ncclResult_t r = ncclCommInitAll(c.data(), (int)devs.size(), devs.data());
        if (r != ncclSuccess) return fail(SDZ_API_HIP_ERROR, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
        it = g_comms.emplace(devs, std::move(c)).first;
    }
    *out = &it->second;
    return SDZ_API_OK;
}

// a one-use barrier for the shard threads (compute | gather, timed apart)
struct Barrier {
    std::mutex mu;
    std::condition_variable cv;
    int left;
    explicit Barrier(int n) : left(n) {}
    void wait() {
        std::unique_lock<std::mutex> lk(mu);
        if (--left == 0) cv.notify_all();
        else cv.wait(lk, [&] { return left == 0; });
    }
};

Pool g_gather;                                   // per device: the all-gathered records
// Multi-GPU calls are serialised: each takes a lock per device for its shard and meets the
// others at a barrier, so two calls on overlapping device lists could each hold a device the
// other waits for.  (Single-device calls only take their device's lock and never wait on a
// barrier, so they interleave with a multi call safely.)
std::mutex g_multi_mu;

// a failed or half-done collective leaves the communicators unusable: abort and forget them
void comms_abort(const std::vector<int32_t>& devs) {
    std::lock_guard<std::mutex> lk(g_comm_mu);
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) return;
    for (ncclComm_t c : it->second) (void)ncclCommAbort(c);
    g_comms.erase(it);
}

int multi_batch(const uint8_t* const* in, const size_t* in_len, uint8_t* const* out, const size_t* out_cap,
                void* rec, uint32_t n, const Codec& C, const int32_t* devices, int32_t ndev,
                sdz_multi_stats* stats) {
    std::lock_guard<std::mutex> serial(g_multi_mu);
    const double t0 = now_ms();
    if (int rc = ensure_device()) return rc;
    if (ndev < 1 || ndev > SDZ_MAX_SHARDS || !devices) return fail(SDZ_API_BAD_ARG, "multi: 1..SDZ_MAX_SHARDS devices");
    const int nd = sdz_device_count();
    for (int32_t k = 0; k < ndev; ++k)
        if (devices[k] < 0 || devices[k] >= nd) return fail(SDZ_API_BAD_ARG, "multi: device index out of range");
    if (stats) { std::memset(stats, 0, sizeof *stats); stats->nshards = ndev; }
    if (n == 0) return SDZ_API_OK;
    if (int rc = check_batch(in, in_len, out, out_cap, rec, n)) return rc;
    std::vector<uint64_t> sizes(in_len, in_len + n);
    std::vector<uint32_t> owner(n);
    sdz_lpt_shard(sizes.data(), n, (uint32_t)ndev, owner.data());
    std::vector<std::vector<uint32_t>> ids(ndev);
    for (uint32_t i = 0; i < n; ++i) ids[owner[i]].push_back(i);
    uint32_t max_m = 0;
    for (auto& v : ids) max_m = std::max<uint32_t>(max_m, (uint32_t)v.size());
    const std::vector<int32_t> devs(devices, devices + ndev);
    std::vector<int32_t> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    const bool loopback = std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end();
    // RCCL whenever the devices are distinct (a single device too: a one-rank all-gather)
    const bool rccl = !loopback;
    std::vector<ncclComm_t>* comms = nullptr;
    if (rccl)
        if (int rc = comms_for(devs, &comms)) return rc;
    const size_t rsz = C.rec_size();
    const size_t slot_bytes = (size_t)max_m * rsz;
    std::vector<ShardOut> R(ndev);
    std::vector<int> rcs(ndev, SDZ_API_OK);
    std::vector<std::string> errs(ndev);
    std::vector<uint8_t> gathered;                 // rank 0's all-gathered records (RCCL)
    Barrier bar(ndev), bar2(ndev);
    std::atomic<bool> coll_fail{false};            // some rank's collective failed: all stop waiting
    double t_compute = 0, t_gather0 = 0;
    std::mutex tmu;
    auto shard = [&](int k) {
        int rc = hipSetDevice(devs[k]) == hipSuccess ? SDZ_API_OK : fail(SDZ_API_HIP_ERROR, "hipSetDevice");
        // RCCL: the shard's gather buffer (ndev slots; its own records copied into slot k, an
        // in-place all-gather) is taken BEFORE the barrier and held by this use until the
        // collective is done -- its lifetime does not depend on any lock.  Loopback shards
        // share devices and hand their records to the host themselves (the "gather").
        PoolUse guse(g_gather, nullptr);
        uint8_t* g = nullptr;
        if (rc == SDZ_API_OK && rccl) {
            DevLock lk;                            // (pool get under the device's lock)
            rc = lk.rc;
            void* gp = nullptr;
            if (rc == SDZ_API_OK) rc = guse.get((size_t)ndev * slot_bytes + 256, &gp);
            g = (uint8_t*)gp;
        }
        uint8_t* mine = g ? g + (size_t)k * slot_bytes : nullptr;
        R[k].timed = true;
        if (rc == SDZ_API_OK && !ids[k].empty())
            rc = host_shard(in, in_len, out, out_cap, ids[k], max_m, C, loopback ? rec : nullptr, R[k], mine);
        else if (rc == SDZ_API_OK && rccl) {
            // an empty shard still joins the all-gather with zeroed records
            hipError_t e = hipMemsetAsync(mine, 0, slot_bytes, nullptr);
            if (e != hipSuccess) rc = hip_fail(e, "empty shard: hipMemsetAsync");
            R[k].d_rec = mine;
        }
        rcs[k] = rc;
        if (rc) errs[k] = sdz_last_error();
        {
            std::lock_guard<std::mutex> lk(tmu);
            t_compute = std::max(t_compute, now_ms() - t0);
        }
        // this rank's communicator, read while the cache entry is certainly alive (only a failed
        // collective erases it, after the second barrier below)
        ncclComm_t comm = rccl ? (*comms)[k] : nullptr;
        bar.wait();                                 // every shard computed (or failed) and holds its slot
        if (k == 0) t_gather0 = now_ms();
        bool any_fail = false;
        for (int q = 0; q < ndev; ++q) any_fail = any_fail || rcs[q] != SDZ_API_OK;
        if (any_fail || !rccl) return;              // no rank enqueues a collective
        // RCCL all-gather of the fixed-size records (max_m slots per shard), in place
        int r2 = SDZ_API_OK;
        // tests: SDZ_TEST_GATHER_FAIL=k makes rank k's collective fail without entering it (its
        // peers are then inside a collective that cannot complete: the abort path)
        const char* inj = getenv("SDZ_TEST_GATHER_FAIL");
        ncclResult_t nr = inj && atoi(inj) == k ? ncclInternalError
                                                : ncclAllGather(mine, g, slot_bytes, ncclUint8, comm, nullptr);
        if (nr != ncclSuccess) r2 = fail(SDZ_API_HIP_ERROR, std::string("ncclAllGather: ") + ncclGetErrorString(nr));
        if (r2 == SDZ_API_OK && k == 0) {
            gathered.resize((size_t)ndev * slot_bytes);
            if (hipMemcpyAsync(gathered.data(), g, gathered.size(), hipMemcpyDeviceToHost, nullptr) != hipSuccess)
                r2 = fail(SDZ_API_HIP_ERROR, "records to host");
        }
        if (r2 != SDZ_API_OK) coll_fail.store(true);
        // wait for the collective, or for another rank's failure (its peers would wait forever on
        // a collective one rank never entered): poll rather than block, and give up after
        // SDZ_GATHER_TIMEOUT_MS (default 120 s: a collective that hangs without any rank failing
        // ends the call with an error instead of spinning every thread forever)
        static const long long limit_ms = getenv("SDZ_GATHER_TIMEOUT_MS") ? atoll(getenv("SDZ_GATHER_TIMEOUT_MS")) : 120000;
        const auto t0 = std::chrono::steady_clock::now();
        while (r2 == SDZ_API_OK) {
            const hipError_t q = hipStreamQuery(nullptr);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) { r2 = hip_fail(q, "gather sync"); coll_fail.store(true); break; }
            if (coll_fail.load()) { r2 = fail(SDZ_API_HIP_ERROR, "gather: another shard's collective failed"); break; }
            if (limit_ms > 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(limit_ms)) {
                r2 = fail(SDZ_API_HIP_ERROR, "gather: the collective did not complete within SDZ_GATHER_TIMEOUT_MS");
                coll_fail.store(true);
                break;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        // every rank has left the collective (done, failed, or given up); one of them aborts the
        // communicators and drops them from the cache, none of the others touches them after this
        bar2.wait();
        if (k == 0 && coll_fail.load()) comms_abort(devs);
        if (r2) { rcs[k] = r2; errs[k] = sdz_last_error(); }
    };
    std::vector<std::thread> th;
    for (int k = 1; k < ndev; ++k) th.emplace_back(shard, k);
    int dev0 = 0;
    (void)hipGetDevice(&dev0);
    shard(0);
    for (auto& t : th) t.join();
    (void)hipSetDevice(dev0);                        // the caller's device stays current
    for (int k = 0; k < ndev; ++k)
        if (rcs[k]) return fail(rcs[k], "shard " + std::to_string(k) + " (device " + std::to_string(devs[k]) + "): " + errs[k]);
    if (rccl)                                        // records in the caller's order
        for (int k = 0; k < ndev; ++k)
            for (size_t j = 0; j < R[k].order.size(); ++j)
                std::memcpy((uint8_t*)rec + (size_t)R[k].order[j] * rsz,
                            gathered.data() + ((size_t)k * max_m + j) * rsz, rsz);
    if (stats) {
        const double t1 = now_ms();
        stats->wall_ms = t1 - t0;
        stats->compute_ms = t_compute;
        stats->gather_ms = rccl ? t1 - t_gather0 : 0.0;
        stats->collective = rccl ? 1 : 0;
        for (int k = 0; k < ndev; ++k) {
            stats->kernel_ms[k] = R[k].kernel_ms;
            stats->bytes_in[k] = R[k].bytes_in;
            stats->bytes_out[k] = R[k].bytes_out;
            stats->streams[k] = (uint32_t)ids[k].size();
        }
    }
    return SDZ_API_OK;
}

}  // namespace

struct sdz_comm {
    ncclComm_t c = nullptr;
    int dev = 0;
    double* d_val = nullptr;
};

extern "C" {

int sdz_gather_device(uint8_t* dst, const uint64_t* dst_off, const uint8_t* src, const uint64_t* src_off,
                      const uint64_t* len, uint32_t n, void* stream) {
    if (int rc = ensure_device()) return rc;
    if (n == 0) return SDZ_API_OK;
    if (!dst || !dst_off || !src || !src_off || !len) return fail(SDZ_API_BAD_ARG, "sdz_gather_device: null pointer");
    timing_begin((hipStream_t)stream);
    launch_gather(dst, dst_off, src, src_off, len, n, (hipStream_t)stream);
    timing_end((hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return SDZ_API_OK;
}

int sdz_inflate_batch(const uint8_t* const* in, const size_t* in_len, uint8_t* const* out,
                      const size_t* out_cap, sdz_inflate_record* rec, uint32_t n, int32_t format,
                      const uint8_t* dict, size_t dict_len) {
    Codec C;
    C.inflate = true; C.format = format; C.dict = dict; C.dict_len = dict_len;
    return host_batch(in, in_len, out, out_cap, rec, n, C);
}

int sdz_deflate_batch(const uint8_t* const* in, const size_t* in_len, uint8_t* const* out,
                      const size_t* out_cap, sdz_deflate_record* rec, uint32_t n, int32_t level,
                      int32_t format, const uint8_t* fname, size_t fname_len, uint32_t mtime,
                      const uint8_t* dict, size_t dict_len) {
    Codec C;
    C.inflate = false; C.level = level; C.format = format; C.fname = fname; C.fname_len = (uint32_t)fname_len;
    C.mtime = mtime; C.dict = dict; C.dict_len = dict_len;
    return host_batch(in, in_len, out, out_cap, rec, n, C);
}

int sdz_lpt_shard(const uint64_t* sizes, uint32_t n, uint32_t nshards, uint32_t* owner) {
    if (nshards < 1 || (n && (!sizes || !owner))) return fail(SDZ_API_BAD_ARG, "sdz_lpt_shard: bad arguments");
    std::vector<uint32_t> ord(n);
    std::iota(ord.begin(), ord.end(), 0u);
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return sizes[a] > sizes[b]; });
    // (load, shard) min-heap: ties go to the lower shard
    typedef std::pair<uint64_t, uint32_t> L;
    std::priority_queue<L, std::vector<L>, std::greater<L>> heap;
    for (uint32_t r = 0; r < nshards; ++r) heap.push(L(0, r));
    for (uint32_t i : ord) {
        L t = heap.top();
        heap.pop();
        owner[i] = t.second;
        heap.push(L(t.first + sizes[i], t.second));
    }
    return SDZ_API_OK;
}

int sdz_inflate_batch_multi(const uint8_t* const* in, const size_t* in_len, uint8_t* const* out,
                            const size_t* out_cap, sdz_inflate_record* rec, uint32_t n, int32_t format,
                            const uint8_t* dict, size_t dict_len, const int32_t* devices, int32_t ndev,
                            sdz_multi_stats* stats) {
    Codec C;
    C.inflate = true; C.format = format; C.dict = dict; C.dict_len = dict_len;
    return multi_batch(in, in_len, out, out_cap, rec, n, C, devices, ndev, stats);
}

int sdz_deflate_batch_multi(const uint8_t* const* in, const size_t* in_len, uint8_t* const* out,
                            const size_t* out_cap, sdz_deflate_record* rec, uint32_t n, int32_t level,
                            int32_t format, const uint8_t* fname, size_t fname_len, uint32_t mtime,
                            const uint8_t* dict, size_t dict_len, const int32_t* devices, int32_t ndev,
                            sdz_multi_stats* stats) {
    if (level < 1 || level > 9) return fail(SDZ_API_BAD_ARG, "level must be between 1 and 9, inclusive");
    if (format < SDZ_DEFLATE_RAW || format > SDZ_DEFLATE_GZIP)
        return fail(SDZ_API_BAD_ARG, "container must be one of `raw`, `deflate`, `gzip`");
    Codec C;
    C.inflate = false; C.level = level; C.format = format; C.fname = fname; C.fname_len = (uint32_t)fname_len;
    C.mtime = mtime; C.dict = dict; C.dict_len = dict_len;
    return multi_batch(in, in_len, out, out_cap, rec, n, C, devices, ndev, stats);
}

// ------------------------------------------------------------------ one process per GPU

int sdz_comm_unique_id(uint8_t* id) {
    if (!id) return fail(SDZ_API_BAD_ARG, "sdz_comm_unique_id: null pointer");
    static_assert(sizeof(ncclUniqueId) == SDZ_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return fail(SDZ_API_HIP_ERROR, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(id, &u, sizeof u);
    return SDZ_API_OK;
}

sdz_comm* sdz_comm_init_rank(const uint8_t* id, int32_t nranks, int32_t rank) {
    if (ensure_device()) return nullptr;
    if (!id || nranks < 1 || rank < 0 || rank >= nranks) { fail(SDZ_API_BAD_ARG, "sdz_comm_init_rank: bad arguments"); return nullptr; }
    sdz_comm* c = new sdz_comm;
    (void)hipGetDevice(&c->dev);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclResult_t r = ncclCommInitRank(&c->c, nranks, u, rank);
    if (r != ncclSuccess) { fail(SDZ_API_HIP_ERROR, std::string("ncclCommInitRank: ") + ncclGetErrorString(r)); delete c; return nullptr; }
    if (hipMalloc(&c->d_val, 64) != hipSuccess) { fail(SDZ_API_OOM, "sdz_comm_init_rank: hipMalloc"); ncclCommDestroy(c->c); delete c; return nullptr; }
    return c;
}

int sdz_comm_allgather_device(sdz_comm* c, const void* send, void* recv, uint64_t bytes) {
    if (!c || (bytes && (!send || !recv))) return fail(SDZ_API_BAD_ARG, "sdz_comm_allgather_device: bad arguments");
    ncclResult_t r = ncclAllGather(send, recv, bytes, ncclUint8, c->c, nullptr);
    if (r != ncclSuccess) return fail(SDZ_API_HIP_ERROR, std::string("ncclAllGather: ") + ncclGetErrorString(r));
    HIPCHK(hipStreamSynchronize(nullptr));
    return SDZ_API_OK;
}

int sdz_comm_allreduce_max(sdz_comm* c, double* v) {
    if (!c || !v) return fail(SDZ_API_BAD_ARG, "sdz_comm_allreduce_max: bad arguments");
    HIPCHK(hipMemcpy(c->d_val, v, sizeof *v, hipMemcpyHostToDevice));
    ncclResult_t r = ncclAllReduce(c->d_val, c->d_val, 1, ncclFloat64, ncclMax, c->c, nullptr);
    if (r != ncclSuccess) return fail(SDZ_API_HIP_ERROR, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    HIPCHK(hipMemcpy(v, c->d_val, sizeof *v, hipMemcpyDeviceToHost));
    return SDZ_API_OK;
}

int sdz_comm_destroy(sdz_comm* c) {
    if (!c) return SDZ_API_OK;
    if (c->d_val) (void)hipFree(c->d_val);
    ncclResult_t r = ncclCommDestroy(c->c);
    delete c;
    if (r != ncclSuccess) return fail(SDZ_API_HIP_ERROR, std::string("ncclCommDestroy: ") + ncclGetErrorString(r));
    return SDZ_API_OK;
}

}  // extern "C"
