// k_gather.hip -- batched span copy on the device: dst[dst_off[i] ..] <- src[src_off[i] ..]
// for n spans of len[i] bytes, in ONE launch (sdz_gather_device).
//
// Used to stage batches: the bench places 65,536 input slices at arbitrary source offsets
// into their stream slots with one launch instead of 65,536 hipMemcpy dispatches (which a
// --pmc pass instruments one by one), and the host-batch entry points scatter the records'
// payloads out of the device pool the same way.  Not on the codec path: no reference
// function behind it; pure HBM traffic (read len + write len per span).
//
// Layout: blockIdx.y cuts each span into GA_SLICES interleaved 4 KiB pieces, so a few huge
// spans still spread over many CUs; a block copies its pieces as aligned destination dwords
// (source dwords assembled from two aligned reads with v_alignbyte), head / tail bytes
// separately.  Aligned source reads never leave the allocation a valid span lies in.
#include "sdz_internal.h"

namespace sdz {

#define GA_THREADS 256
#define GA_SLICES 8
#define GA_PIECE 4096u

__global__ __launch_bounds__(GA_THREADS) void k_gather(uint8_t* dst, const uint64_t* dst_off, const uint8_t* src,
                                                       const uint64_t* src_off, const uint64_t* len, uint32_t n) {
    const uint32_t sid = blockIdx.x;
    if (sid >= n) return;
    const uint64_t L = len[sid];
    if (L == 0) return;
    uint8_t* d = dst + dst_off[sid];
    const uint8_t* s = src + src_off[sid];
    if ((((uintptr_t)d | (uintptr_t)s) & 15) == 0) {     // both 16-aligned: 16-byte vectors
        const uint64_t nv = L >> 4;
        const uint64_t vpp = GA_PIECE / 16;
        for (uint64_t p0 = (uint64_t)blockIdx.y * vpp; p0 < nv; p0 += (uint64_t)GA_SLICES * vpp) {
            const uint64_t pe = p0 + vpp < nv ? p0 + vpp : nv;
            for (uint64_t q = p0 + threadIdx.x; q < pe; q += GA_THREADS) ((uint4*)d)[q] = ((const uint4*)s)[q];
        }
        const uint64_t t0 = nv << 4;
        if (blockIdx.y == GA_SLICES - 1 && threadIdx.x < L - t0) d[t0 + threadIdx.x] = s[t0 + threadIdx.x];
        return;
    }
    // head: bytes until d is 4-aligned (block y = 0 only)
    const uint32_t h0 = (uint32_t)((4u - ((uintptr_t)d & 3u)) & 3u);
    const uint64_t h = L < h0 ? L : h0;
    if (blockIdx.y == 0 && threadIdx.x < h) d[threadIdx.x] = s[threadIdx.x];
    const uint64_t nw = (L - h) >> 2;                    // whole destination dwords
    uint32_t* dw = (uint32_t*)(d + h);
    const uint8_t* sb = s + h;
    const uint32_t k = (uint32_t)((uintptr_t)sb & 3u);
    const uint32_t* sw = (const uint32_t*)(sb - k);
    const uint64_t wpp = GA_PIECE / 4;                   // dwords per piece
    for (uint64_t p0 = (uint64_t)blockIdx.y * wpp; p0 < nw; p0 += (uint64_t)GA_SLICES * wpp) {
        const uint64_t pe = p0 + wpp < nw ? p0 + wpp : nw;
        for (uint64_t q = p0 + threadIdx.x; q < pe; q += GA_THREADS) {
            const uint32_t lo = sw[q];
            // the second dword holds bytes of this span only when k != 0
            const uint32_t hi = k ? sw[q + 1] : 0u;
            dw[q] = __builtin_amdgcn_alignbyte(hi, lo, k);
        }
    }
    // tail bytes
    const uint64_t t0 = h + 4 * nw;
    if (blockIdx.y == GA_SLICES - 1 && threadIdx.x < L - t0) d[t0 + threadIdx.x] = s[t0 + threadIdx.x];
}

void launch_gather(uint8_t* dst, const uint64_t* dst_off, const uint8_t* src, const uint64_t* src_off,
                   const uint64_t* len, uint32_t n, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_gather, dim3(n, GA_SLICES), dim3(GA_THREADS), 0, s, dst, dst_off, src, src_off, len, n);
}

// The host path's copy back of a small call: the [outputs | records] region of the device pool
// into the same layout in pinned host memory, only the bytes each stream wrote (its record's
// out_len, at len_off) and the m records.  Block k < m: stream k's output; block m: the records.
// A copy engine's copy of the whole region started ~20 us after the last kernel on a one-stream
// inflate (rocprofv3 trace, profiles/r05/lat); this kernel follows the codec's last launch.
// dst is device-mapped pinned memory; out_off are 8-byte aligned, rec_off 256-byte aligned.
__global__ __launch_bounds__(GA_THREADS) void k_copy_back(uint8_t* dst, const uint8_t* src, const uint64_t* out_off,
                                                          const uint64_t* out_cap, uint64_t rec_off, uint32_t rsz,
                                                          uint32_t len_off, uint32_t m) {
    const uint32_t k = blockIdx.x;
    uint64_t o, L;
    if (k == m) {
        o = rec_off;
        L = (uint64_t)m * rsz;
    } else {
        o = out_off[k];
        const uint64_t ol = *(const uint64_t*)(src + rec_off + (uint64_t)k * rsz + len_off);
        L = ol < out_cap[k] ? ol : out_cap[k];
    }
    const uint64_t nq = L >> 3;
    const uint64_t* s8 = (const uint64_t*)(src + o);
    uint64_t* d8 = (uint64_t*)(dst + o);
    for (uint64_t q = threadIdx.x; q < nq; q += GA_THREADS) d8[q] = s8[q];
    const uint64_t t = nq << 3;
    if (threadIdx.x < L - t) dst[o + t + threadIdx.x] = src[o + t + threadIdx.x];
}

void launch_copy_back(uint8_t* dst, const uint8_t* src, const uint64_t* out_off, const uint64_t* out_cap,
                      uint64_t rec_off, uint32_t rsz, uint32_t len_off, uint32_t m, hipStream_t s) {
    hipLaunchKernelGGL(k_copy_back, dim3(m + 1), dim3(GA_THREADS), 0, s, dst, src, out_off, out_cap, rec_off, rsz,
                       len_off, m);
}

}  // namespace sdz
