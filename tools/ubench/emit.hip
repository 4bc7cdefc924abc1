// emit_fast latency microbenchmark (development aid): one wave per CU calls the resolve
// kernel's emit_fast on synthetic text-like tokens (literals and copies of 3-12 bytes,
// distances 64-20000, ~30% literals) and reports wall-clock ns per call.
#include "../../sd-zlib_amd/csrc/k_resolve.hip"
#include <stdio.h>

namespace sdz {
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ void mskor(uint32_t* p, uint32_t clear, uint32_t set) {
    const uint32_t a = (uint32_t)(uintptr_t)(lds_u32*)p;
    asm volatile("ds_mskor_b32 %0, %1, %2" :: "v"(a), "v"(clear), "v"(set) : "memory");
}
// copy/literal/period token as K masked-OR dword writes (tokens up to 4K - 3 bytes)
template <int K>
__device__ __forceinline__ void emit_msk(uint8_t* ring, bool act, uint32_t t, uint32_t d, uint32_t s,
                                         uint32_t len, uint32_t dist) {
    uint32_t* ring32 = (uint32_t*)ring;
    const uint32_t dumi = RS_DUMMY / 4;
    const bool lit = (t >> 31) == 0;
    const bool per = !lit && dist < 4u;
    const uint32_t kd = d & 3u, D0 = d >> 2;
    const uint32_t sx = s - kd, xa = sx >> 2, k = sx & 3u;
    uint32_t x[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) x[j] = ring32[act && !lit ? xa + j : dumi];
    const uint32_t m = (k + kd) >> 2, ks = (k + kd) & 3u;
    const uint32_t H = __builtin_amdgcn_alignbyte(m ? x[2] : x[1], m ? x[1] : x[0], ks);
    const uint32_t ph0 = dist == 3u ? (3u - kd % 3u) % 3u : dist == 2u ? kd & 1u : 0u;
    uint32_t ph = ph0;
    const uint32_t e = kd + len;                        // end byte, relative to dword D0
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const uint32_t lo = j == 0 ? kd : 0u;
        const int32_t hi = (int32_t)e - 4 * j;           // bytes of this dword in the token: [lo, min(hi, 4))
        const uint32_t hm = hi >= 4 ? 0xffffffffu : hi <= 0 ? 0u : (1u << (8 * hi)) - 1u;
        const uint32_t mask = act ? hm & (0xffffffffu << (8 * lo)) : 0u;
        uint32_t v = per ? rep4(H, dist, ph) : __builtin_amdgcn_alignbyte(x[j + 1], x[j], k);
        if (lit) v = j == 0 ? t << (8 * kd) : (kd ? t >> (32u - 8 * kd) : 0u);
        ph = dist == 3u ? (ph == 2u ? 0u : ph + 1u) : ph;
        mskor(mask ? ring32 + D0 + j : ring32 + dumi, mask, v & mask);
    }
}
template <int MODE>
__global__ __launch_bounds__(64) void k_emit_bench(uint32_t* out, uint32_t iters) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[RS_R + 256];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < (RS_R + 256) / 4; i += 64) ((uint32_t*)ring)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t x = lane * 7919u + 1u, P = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        x = x * 1664525u + 1013904223u;
        const bool lit = (x >> 28) < 5u;
        const uint32_t len = lit ? 1u + ((x >> 8) & 1u) : 3u + ((x >> 12) % 10u);
        const uint32_t dist = lit ? 0u : 64u + ((x >> 4) % 20000u);
        const uint32_t t = lit ? (((len - 1u) << 24) | (x & 0xffffu)) : (0x80000000u | ((len - 3u) << 16) | (dist - 1u));
        const uint32_t off = lane * 8u;
        const uint32_t d = ridx((int32_t)(P + off));
        const uint32_t s = ridx((int32_t)(P + off) - (int32_t)dist);
        if (MODE == 0) emit_fast(ring, true, t, d, s, len, dist);
        if (MODE == 1) emit_tokens(ring, true, t, d, s, len, dist);
        if (MODE == 5) emit_msk<5>(ring, true, t, d, s, len, dist);
        if (MODE == 6) emit_msk<3>(ring, true, t, d, s, len, dist);
        if (MODE == 2) {                                  // 6 sub-dword stores (two store_part)
            store_part(ring, true, d & ~3u, x, d & 3u, 4u);
            store_part(ring, true, (d + 8u) & ~3u, x, 0u, 1u + (x & 3u));
        }
        if (MODE == 3) {                                  // 13 reads, 8 dword writes
            uint32_t* r32 = (uint32_t*)ring;
            uint32_t acc = 0, xs[13];
#pragma unroll
            for (int j = 0; j < 13; ++j) xs[j] = r32[(s >> 2) + j];
#pragma unroll
            for (int j = 0; j < 8; ++j) r32[(d >> 2) + j] = __builtin_amdgcn_alignbyte(xs[j + 1], xs[j], s & 3u) + xs[12];
            (void)acc;
        }
        if (MODE == 4) {                                  // 13 reads only, summed
            uint32_t* r32 = (uint32_t*)ring;
            uint32_t acc = 0;
#pragma unroll
            for (int j = 0; j < 13; ++j) acc += r32[(s >> 2) + j];
            r32[RS_DUMMY / 4] = acc;
        }
        P = ridx((int32_t)(P + 512u));
    }
    out[lane] = ring[lane * 97u];
}
}  // namespace sdz

template <int MODE> void run(const char* name) {
    uint32_t* d; (void)hipMalloc(&d, 4096);
    const uint32_t iters = 20000;
    hipLaunchKernelGGL(sdz::k_emit_bench<MODE>, dim3(256), dim3(64), 0, 0, d, iters);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(sdz::k_emit_bench<MODE>, dim3(256), dim3(64), 0, 0, d, iters);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-24s %8.1f ns per call\n", name, ms * 1e6 / iters);
    (void)hipFree(d);
}
int main() {
    run<0>("emit_fast");
    run<1>("emit_tokens (general)");
    run<5>("emit_msk<5>");
    run<6>("emit_msk<3>");
    run<2>("6 sub-dword stores");
    run<3>("13 reads + 8 dword writes");
    run<4>("13 reads + 1 write");
    return 0;
}
