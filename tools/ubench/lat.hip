// Latency microbenchmark (development aid): one wave per CU, dependent chains of
// LDS reads, VALU ops, ballot->SALU branches and readlane, in wall-clock nanoseconds
// per step (hipEvents; s_memtime is not trusted as a core-clock counter here).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define N 32768
template <int MODE>
__global__ __launch_bounds__(64) void k(uint32_t* out, uint32_t iters) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[N / 4];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < N / 4; i += 64) lds[i] = (i * 97u + 13u) & (N / 4 - 1);
    __syncthreads();
    uint32_t a = t * 37u, acc = t;
    for (uint32_t it = 0; it < iters; ++it) {
        if (MODE == 0) { a = lds[a & (N / 4 - 1)]; }                       // dependent ds_read_b32
        if (MODE == 1) { a = a * 3u + 1u; a ^= a >> 3; a = a * 5u + it; a ^= a >> 7; }   // 8 dependent VALU
        if (MODE == 2) { uint64_t b = __ballot((a & 1u) != 0); if (b & 1) a += 3; else a += 5; a = a * 3u + (uint32_t)b; }
        if (MODE == 3) { a = (uint32_t)__builtin_amdgcn_readlane((int)(a * 3u + 1u), (int)(it & 63u)) + t; }
        if (MODE == 4) { ((uint8_t*)lds)[(a & (N - 1))] = (uint8_t)it; a = lds[(a >> 2) & (N / 4 - 1)] + t; }   // write then dependent read
        if (MODE == 5) { a = lds[a & (N / 4 - 1)]; a = lds[(a + 1) & (N / 4 - 1)]; a = lds[(a + 2) & (N / 4 - 1)]; a = lds[(a + 3) & (N / 4 - 1)]; }
    }
    if (a == 0xdeadbeef) out[1] = acc;
    out[0] = a;
}
template <int MODE> void run(const char* name, double per) {
    uint32_t* d; hipMalloc(&d, 64);
    const uint32_t iters = 20000;
    hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(64), 0, 0, d, iters);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(64), 0, 0, d, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-34s %8.2f ns/iter  %7.2f ns per step\n", name, ms * 1e6 / iters, ms * 1e6 / iters / per);
    hipFree(d);
}
int main() {
    run<0>("dependent ds_read_b32", 1);
    run<5>("4 dependent ds_read_b32", 4);
    run<1>("8 dependent VALU", 8);
    run<2>("ballot -> SALU branch (+3 VALU)", 1);
    run<3>("readlane chain (+2 VALU)", 1);
    run<4>("ds_write_b8 + dependent ds_read", 1);
    return 0;
}
