// Resolve-emit latency microbenchmark (development aid): one wave per CU calls the resolve
// kernel's token writers on synthetic text-like tokens (literals and copies of 3-12 bytes,
// distances 64-20000, ~30% literals) and reports wall-clock ns per call.
//   emit_msk     masked dword RMWs (the kernel's path)
//   emit_tokens  the general path (head / dword body / tail stores)
#include "../../sd-zlib_amd/csrc/k_resolve.hip"
#include <stdio.h>

namespace sdz {
template <int MODE>
__global__ __launch_bounds__(64) void k_emit_bench(uint32_t* out, uint32_t iters) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[RS_R + 256];
    __shared__ __attribute__((aligned(16))) uint8_t fmap[RS_BM];
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
        const uint32_t mp = (P + off) & (RS_BM / 2 - 1);
        if (MODE == 0) emit_msk(ring, fmap, true, t, d, s, len, dist, mp, 1u);
        if (MODE == 1) emit_tokens(ring, fmap, true, t, d, s, len, dist, mp, 1u);
        P = ridx((int32_t)(P + 512u));
    }
    out[lane] = ring[lane * 97u] + fmap[lane];
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
    run<0>("emit_msk");
    run<1>("emit_tokens (general)");
    return 0;
}
