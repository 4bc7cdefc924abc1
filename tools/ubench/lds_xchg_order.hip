// Does ds_wrxchg_rtn serialize same-address lanes of one wave instruction in lane order?
// (lane l must get lane l-1's value among lanes sharing an address).  Development aid.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(uint32_t* bad, uint32_t iters, uint32_t seed) {
    __shared__ uint32_t tab[64];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    __shared__ uint32_t slots[4][64];
    uint32_t x = seed * 2654435761u + blockIdx.x * 97u + threadIdx.x;
    uint32_t nbad = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        x = x * 1664525u + 1013904223u;
        const uint32_t key = (x >> 28) & (it & 1 ? 3u : 15u);     // few distinct addresses
        uint32_t* t = &slots[w][0];
        if (lane < 16) t[lane] = 0xffffffffu;
        __builtin_amdgcn_wave_barrier();
        const uint32_t old = atomicExch(&t[key], lane);
        // expected: the largest lane < lane with the same key, else 0xffffffff
        uint32_t exp = 0xffffffffu;
        for (uint32_t l = 0; l < 64; ++l) {                         // uniform loop: all lanes shuffle
            const uint32_t kl = (uint32_t)__shfl((int)key, (int)l);
            if (l < lane && kl == key) exp = l;
        }
        nbad += old != exp;
        __builtin_amdgcn_wave_barrier();
    }
    (void)tab;
    atomicAdd(bad, nbad);
}
int main() {
    uint32_t* d; hipMalloc(&d, 4); hipMemset(d, 0, 4);
    hipLaunchKernelGGL(k, dim3(1024), dim3(256), 0, 0, d, 2000u, 7u);
    uint32_t h = 0; hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("mismatches: %u of %u\n", h, 1024u * 256u * 2000u);
    return 0;
}
