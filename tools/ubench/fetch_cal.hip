// FETCH_SIZE / WRITE_SIZE calibration for the access widths the deflate and inflate kernels use
// (MI355X_MICROARCH.md, HBM/rocprofv3: only 16-byte-per-lane streaming reads are calibrated, at
// 1/2).  Each kernel touches a known set of bytes of a 2 GiB buffer (well past the 256 MiB
// Infinity Cache), once:
//   k_stream16   16 B per lane, coalesced, the whole buffer               (bytes = 2 GiB)
//   k_scatter1   1 B per lane at a distinct 128-B line (a permutation)    (lines = 16 Mi)
//   k_scatter8   8 B per lane at a distinct 128-B line                    (lines = 16 Mi)
//   k_scatter2   1 B in each 64-B half of a distinct 128-B line           (lines = 16 Mi)
//                (against k_scatter1: does a byte load fetch the line or its 64-B half?)
//   k_lane8      8 B per lane, lane i reading line-sequentially its own 64 KiB span
//                (k_dfl_parse's lane-per-stream record walk)            (bytes = 2 GiB)
//   k_lane16     16 B per lane, the same per-lane spans (k_inflate_decode's input refills)
//                                                                        (bytes = 2 GiB)
//   k_store8     8 B per lane, the same lane-per-span pattern as a store  (bytes = 2 GiB)
// tools/ubench/fetch_cal.sh runs it under separate FETCH_SIZE / WRITE_SIZE passes and prints
// counter KiB x 1024 / known bytes per kernel.  `fetch_cal time` times each read kernel instead
// (best of 5): the read-only rates a kernel's calibrated traffic can be checked against
// (streaming bytes, and 128-B lines x 128 B for the scattered kernels).
//   hipcc --offload-arch=gfx950 -O3 -o fetch_cal tools/ubench/fetch_cal.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

static constexpr uint64_t kBytes = 2ull << 30;
static constexpr uint64_t kLines = kBytes / 128;

__global__ void k_stream16(const uint4* __restrict__ a, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < kBytes / 16; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
// line index of the i-th access: an odd multiplier mod 2^24 is a permutation of the lines
__device__ __forceinline__ uint64_t perm(uint64_t i) { return (i * 2654435761ull) & (kLines - 1); }
__global__ void k_scatter1(const uint8_t* __restrict__ a, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < kLines; i += (uint64_t)gridDim.x * 256)
        acc += a[perm(i) * 128 + (i & 127)];
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_scatter8(const uint64_t* __restrict__ a, uint32_t* out) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < kLines; i += (uint64_t)gridDim.x * 256)
        acc += a[perm(i) * 16 + (i & 15)];
    if (acc == 0x12345678u) out[0] = (uint32_t)acc;
}
__global__ void k_scatter2(const uint8_t* __restrict__ a, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < kLines; i += (uint64_t)gridDim.x * 256)
        acc += a[perm(i) * 128 + (i & 63)] + a[perm(i) * 128 + 64 + (i & 63)];
    if (acc == 0x12345678u) out[0] = acc;
}
// 32 Ki lanes, each walking its own 64 KiB span 8 bytes at a time
__global__ void k_lane8(const uint64_t* __restrict__ a, uint32_t* out) {
    const uint64_t lane = blockIdx.x * 256ull + threadIdx.x;
    const uint64_t* p = a + lane * (65536 / 8);
    uint64_t acc = 0;
    for (uint32_t k = 0; k < 65536 / 8; ++k) acc += p[k];
    if (acc == 0x12345678u) out[0] = (uint32_t)acc;
}
__global__ void k_lane16(const uint4* __restrict__ a, uint32_t* out) {
    const uint64_t lane = blockIdx.x * 256ull + threadIdx.x;
    const uint4* p = a + lane * (65536 / 16);
    uint32_t acc = 0;
    for (uint32_t k = 0; k < 65536 / 16; ++k) { const uint4 v = p[k]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_store8(uint64_t* __restrict__ a) {
    const uint64_t lane = blockIdx.x * 256ull + threadIdx.x;
    uint64_t* p = a + lane * (65536 / 8);
    for (uint32_t k = 0; k < 65536 / 8; ++k) p[k] = lane * 31 + k;
}

int main(int argc, char** argv) {
    uint8_t* a = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&a, kBytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(a, 1, kBytes);
    (void)hipDeviceSynchronize();
    const uint32_t lanes = (uint32_t)(kBytes / 65536);   // 32 Ki spans of 64 KiB
    if (argc > 1) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        const char* names[6] = {"stream16", "scatter1", "scatter8", "lane8", "lane16", "scatter2"};
        for (int k = 0; k < 6; ++k) {
            float best = 1e30f;
            for (int r = 0; r < 5; ++r) {
                (void)hipEventRecord(e0, 0);
                if (k == 0) hipLaunchKernelGGL(k_stream16, dim3(4096), dim3(256), 0, 0, (const uint4*)a, out);
                if (k == 1) hipLaunchKernelGGL(k_scatter1, dim3(4096), dim3(256), 0, 0, a, out);
                if (k == 2) hipLaunchKernelGGL(k_scatter8, dim3(4096), dim3(256), 0, 0, (const uint64_t*)a, out);
                if (k == 3) hipLaunchKernelGGL(k_lane8, dim3(lanes / 256), dim3(256), 0, 0, (const uint64_t*)a, out);
                if (k == 4) hipLaunchKernelGGL(k_lane16, dim3(lanes / 256), dim3(256), 0, 0, (const uint4*)a, out);
                if (k == 5) hipLaunchKernelGGL(k_scatter2, dim3(4096), dim3(256), 0, 0, a, out);
                (void)hipEventRecord(e1, 0);
                if (hipEventSynchronize(e1) != hipSuccess) return 1;
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            printf("READ %s %.4f ms %.1f GB/s\n", names[k], best, (double)kBytes / (best * 1e6));
        }
        return 0;
    }
    hipLaunchKernelGGL(k_stream16, dim3(4096), dim3(256), 0, 0, (const uint4*)a, out);
    hipLaunchKernelGGL(k_scatter1, dim3(4096), dim3(256), 0, 0, a, out);
    hipLaunchKernelGGL(k_scatter8, dim3(4096), dim3(256), 0, 0, (const uint64_t*)a, out);
    hipLaunchKernelGGL(k_scatter2, dim3(4096), dim3(256), 0, 0, a, out);
    hipLaunchKernelGGL(k_lane8, dim3(lanes / 256), dim3(256), 0, 0, (const uint64_t*)a, out);
    hipLaunchKernelGGL(k_lane16, dim3(lanes / 256), dim3(256), 0, 0, (const uint4*)a, out);
    hipLaunchKernelGGL(k_store8, dim3(lanes / 256), dim3(256), 0, 0, (uint64_t*)a);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("known bytes: stream16 %llu, scatter1 lines %llu (x128 B %llu), scatter8 lines %llu, lane8 %llu, store8 %llu\n",
           (unsigned long long)kBytes, (unsigned long long)kLines, (unsigned long long)(kLines * 128),
           (unsigned long long)kLines, (unsigned long long)kBytes, (unsigned long long)kBytes);
    return 0;
}
