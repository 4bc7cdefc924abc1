// k_checksum.hip -- batched adler32 / crc32 (src/adler32.ts:17-105, src/crc32.ts:17-216).
//
// One wave per buffer.  adler32 is evaluated block-wise on the reference's NMAX
// (5552-byte) grid so the adler32.ts:67 quirk (sum2 += BASE, reduced only when a
// remainder exists) is reproduced exactly: per block the wave reduces the byte
// sum T and the weighted sum W = sum (5552 - i) * b_i, and lane 0 chains
//   sum2 += 5552 * s1 + W + BASE;  s1 = (s1 + T) mod BASE.
// crc32 (crc32_dev.h): 64 lane chunks, slicing-by-8 over 8-byte loads, merged with GF(2)
// polynomial shifts (x^(8 len) mod P) in a log2(64)-step tree.
#include "sdz_internal.h"
#include "crc32_dev.h"

namespace sdz {

#define CK_THREADS 64

// block sid = blockIdx.x of a batch (in_off / in_len / seed / result indexed by it)
__device__ __forceinline__ void k_checksum_body(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                                                const int32_t* seed, int32_t* result, int kind) {
    __shared__ CrcTables ct;
    uint32_t lane = threadIdx.x;
    if (kind != 0) crc_tables_init(ct);
    __syncthreads();
    uint32_t sid = blockIdx.x;
    const uint8_t* p = in + in_off[sid];
    uint64_t len = in_len[sid];
    uint32_t sd = (uint32_t)(seed ? seed[sid] : (kind == 0 ? 1 : 0));

    if (kind == 0) {                                     // adler32
        uint64_t s1 = sd & 0xffffu, s2 = (sd >> 16) & 0xffffu;
        uint64_t nblk = len / 5552, rem = len % 5552;
        for (uint64_t b = 0; b <= nblk; ++b) {
            uint32_t blen = b < nblk ? 5552u : (uint32_t)rem;
            if (blen == 0) break;
            const uint8_t* q = p + b * 5552;
            uint64_t T = 0, W = 0;
            for (uint32_t i = lane; i < blen; i += CK_THREADS) {
                uint32_t v = q[i];
                T += v;
                W += (uint64_t)(blen - i) * v;
            }
            for (int o = 32; o > 0; o >>= 1) {
                T += __shfl_xor(T, o);
                W += __shfl_xor(W, o);
            }
            s2 += (uint64_t)blen * s1 + W;
            s1 += T;
            if (b < nblk) { s1 %= 65521u; s2 += 65521u; }
            else { s1 %= 65521u; s2 %= 65521u; }
        }
        if (lane == 0) result[sid] = (int32_t)((uint32_t)s1 | ((uint32_t)s2 << 16));
    } else {                                             // crc32
        const uint32_t crc = crc32_wave(p, len, ct);
        if (lane == 0) result[sid] = (int32_t)(gf2_mulmod(gf2_xbytes(len, ct.x2n), sd) ^ crc);
    }
}

__global__ __launch_bounds__(CK_THREADS) void k_checksum(const uint8_t* in, const uint64_t* in_off,
                                                         const uint64_t* in_len, const int32_t* seed,
                                                         int32_t* result, uint32_t n, int kind) {
    if (blockIdx.x >= n) return;                         // (block-uniform: before any barrier)
    k_checksum_body(in, in_off, in_len, seed, result, kind);
}

// one buffer, arguments by value: the DICTID of a preset dictionary, computed on the call's
// stream so that no entry point waits for it on the host
__global__ __launch_bounds__(CK_THREADS) void k_checksum_one(const uint8_t* in, uint64_t len, int32_t seed,
                                                             int32_t* result, int kind) {
    __shared__ uint64_t off_len[2];
    __shared__ int32_t sd;
    if (threadIdx.x == 0) { off_len[0] = 0; off_len[1] = len; sd = seed; }
    __syncthreads();
    // (the batched kernel's body, one buffer: it reads in_off / in_len / seed through pointers)
    k_checksum_body(in, off_len, off_len + 1, &sd, result, kind);
}

void launch_checksum_one(const uint8_t* in, uint64_t len, int kind, int32_t seed, int32_t* result, hipStream_t s) {
    hipLaunchKernelGGL(k_checksum_one, dim3(1), dim3(CK_THREADS), 0, s, in, len, seed, result, kind);
}

void launch_checksum(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                     const int32_t* seed, int32_t* result, uint32_t n, int kind, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_checksum, dim3(n), dim3(CK_THREADS), 0, s, in, in_off, in_len, seed, result, n, kind);
}

}  // namespace sdz
