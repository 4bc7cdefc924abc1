// LDS access-pattern microbenchmark (development aid): CU-cycles per wave-instruction of the
// resolve's store patterns -- masked dword RMWs (ds_mskor_b32), plain dword stores, adds and byte
// stores at the lane spacings a group of short tokens produces -- and of random dword reads, with
// 8 waves per SIMD (4 x 512-thread workgroups per CU) all issuing.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define N 36864
typedef __attribute__((address_space(3))) uint32_t lds_u32;
template <int OP>
__device__ __forceinline__ void op(uint8_t* lds, uint32_t byteaddr, uint32_t v) {
    uint32_t* p = (uint32_t*)(lds + (byteaddr & ~3u));
    const uint32_t a = (uint32_t)(uintptr_t)(lds_u32*)p;
    if (OP == 0) asm volatile("ds_mskor_b32 %0, %1, %2" :: "v"(a), "v"(0xffu << (8 * (byteaddr & 3u))), "v"(v) : "memory");
    if (OP == 1) asm volatile("ds_write_b32 %0, %1" :: "v"(a), "v"(v) : "memory");
    if (OP == 2) asm volatile("ds_add_u32 %0, %1" :: "v"(a), "v"(v) : "memory");
    if (OP == 3) lds[byteaddr] = (uint8_t)v;
    if (OP == 4) asm volatile("ds_or_b32 %0, %1" :: "v"(a), "v"(v) : "memory");
}
// PAT: byte address of lane l: 0 -- 4 l (one dword each); 1 -- 5 l (tokens of 5 bytes: 64 lanes over
// 80 dwords); 2 -- 2 l (two lanes per dword); 3 -- l (four lanes per dword); 4 -- random
template <int OP, int PAT>
__global__ __launch_bounds__(512) void k(uint32_t* out, uint32_t iters) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[N + 64];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (uint32_t i = t; i < N / 4; i += 512) ((uint32_t*)lds)[i] = i * 2654435761u;
    __syncthreads();
    uint32_t x = t * 2654435761u + 12345u;
    uint32_t acc = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        const uint32_t base = ((w * 4099u + it * 389u) * 4u) % (N - 1024);
        x = x * 1664525u + 1013904223u;
        const uint32_t ba = PAT == 0 ? base + 4 * lane : PAT == 1 ? base + 5 * lane : PAT == 2 ? base + 2 * lane
                          : PAT == 3 ? base + lane : (x >> 8) % (N - 8);
        if (OP == 9) { uint32_t v; __builtin_memcpy(&v, lds + (ba & ~3u), 4); acc += v; }
        else op<OP>(lds, ba, it ^ lane);
    }
    if (acc == 12345) out[4] = acc;
}
template <int OP, int PAT> void run(const char* name) {
    uint32_t* d; hipMalloc(&d, 64);
    const uint32_t iters = 8192, blocks = 256 * 4;
    hipLaunchKernelGGL((k<OP, PAT>), dim3(blocks), dim3(512), 0, 0, d, iters);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k<OP, PAT>), dim3(blocks), dim3(512), 0, 0, d, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    // 32 waves per CU share one LDS: wall cycles (at 2.1 GHz) per wave-instruction per CU
    printf("%-14s pat %d: %6.2f CU-cycles per wave-instruction (%.3f ms)\n", name, PAT, ms * 1e-3 * 2.1e9 / (32.0 * iters), ms);
    hipFree(d);
}
#define ALL(OP, NAME) run<OP, 0>(NAME); run<OP, 1>(NAME); run<OP, 2>(NAME); run<OP, 3>(NAME); run<OP, 4>(NAME);
int main() {
    ALL(0, "ds_mskor_b32");
    ALL(1, "ds_write_b32");
    ALL(2, "ds_add_u32");
    ALL(3, "ds_write_b8");
    ALL(4, "ds_or_b32");
    ALL(9, "ds_read_b32");
    return 0;
}
