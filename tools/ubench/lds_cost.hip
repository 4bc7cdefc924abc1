// LDS instruction cost microbenchmark (development aid): cycles per wave-instruction of
// aligned / unaligned dword and byte LDS reads and writes, and of LDS atomics,
// with 8 waves per SIMD (4 x 512-thread workgroups per CU) all issuing.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define N 40000
template <int MODE>
__global__ __launch_bounds__(512) void k(uint32_t* out, uint32_t stride, uint32_t iters) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[N];
    const uint32_t t = threadIdx.x, lane = t & 63;
    for (uint32_t i = t; i < N / 4; i += 512) ((uint32_t*)lds)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t acc = 0;
    uint32_t a = (t * stride) % (N - 64);
    long long c0 = clock64();
    for (uint32_t it = 0; it < iters; ++it) {
        uint32_t ad = (a + it * 4) % (N - 64);
        if (MODE == 0) { uint32_t v; __builtin_memcpy(&v, lds + (ad & ~3u), 4); acc += v; }
        if (MODE == 1) { uint32_t v; __builtin_memcpy(&v, lds + ad + 1, 4); acc += v; }
        if (MODE == 2) { acc += lds[ad + 1]; }
        if (MODE == 3) { uint32_t v = acc + it; __builtin_memcpy(lds + (ad & ~3u), &v, 4); }
        if (MODE == 4) { uint32_t v = acc + it; __builtin_memcpy(lds + ad + 1, &v, 4); }
        if (MODE == 5) { lds[ad + 1] = (uint8_t)(acc + it); }
        if (MODE == 6) { atomicOr((uint32_t*)(lds + (ad & ~3u)), it); }
        if (MODE == 7) { atomicOr((uint32_t*)(lds + ((ad >> 5) & ~3u)), it); }   // ~8 lanes per word
        if (MODE == 8) { uint16_t v = (uint16_t)(acc + it); __builtin_memcpy(lds + ad + 1, &v, 2); }
    }
    long long c1 = clock64();
    if (lane == 0) atomicAdd((unsigned long long*)out, (unsigned long long)(c1 - c0));
    if (acc == 12345) out[4] = acc;
}
template <int MODE> void run(const char* name, uint32_t stride) {
    uint32_t* d; hipMalloc(&d, 64); hipMemset(d, 0, 64);
    const uint32_t iters = 4096, blocks = 256 * 4;
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(512), 0, 0, d, stride, iters);
    hipMemset(d, 0, 64);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(512), 0, 0, d, stride, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long cyc; hipMemcpy(&cyc, d, 8, hipMemcpyDeviceToHost);
    double per_wave = (double)cyc / (blocks * 8) / iters;
    // CU-level: 32 waves share one LDS; wall cycles per wave-instruction per CU
    double wall_cyc_per_inst_cu = ms * 1e-3 * 2.1e9 / (32.0 * iters);
    printf("%-28s stride %3u: %7.2f cyc/iter per wave, %6.2f CU-cycles per wave-instr (%.3f ms)\n",
           name, stride, per_wave, wall_cyc_per_inst_cu, ms);
    hipFree(d);
}
int main() {
    for (uint32_t st : {4u, 5u, 61u}) {
        run<0>("read b32 aligned", st);
        run<1>("read b32 unaligned", st);
        run<2>("read u8", st);
        run<3>("write b32 aligned", st);
        run<4>("write b32 unaligned", st);
        run<5>("write b8", st);
        run<8>("write b16 unaligned", st);
        run<6>("atomic or (distinct)", st);
        run<7>("atomic or (~8 lanes/word)", st);
    }
    return 0;
}
