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

#define CK_THREADS 256
#define CK_BLK 256                        // adler32 NMAX blocks per pass (LDS partials)

// block sid = blockIdx.x of a batch (in_off / in_len / seed / result indexed by it).
// adler32: the stream's 5552-byte blocks go to the workgroup's waves (16-byte loads, byte sums
// and index-weighted sums by v_dot4), their partials T = sum b_i and W = sum (blen - i) b_i into
// LDS, and one thread chains them exactly as adler32.ts does (a one-wave serial walk over the
// blocks with byte loads took 0.88 ms for a 481 KB buffer; one-buffer deflate() waits for it).
// crc32: wave 0 (crc32_wave).
__device__ __forceinline__ void k_checksum_body(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                                                const int32_t* seed, int32_t* result, int kind) {
    __shared__ CrcTables ct;
    __shared__ uint32_t ck_T[CK_BLK];
    __shared__ uint64_t ck_W[CK_BLK];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    if (kind != 0) crc_tables_init(ct);
    __syncthreads();
    uint32_t sid = blockIdx.x;
    const uint8_t* p = in + in_off[sid];
    uint64_t len = in_len[sid];
    uint32_t sd = (uint32_t)(seed ? seed[sid] : (kind == 0 ? 1 : 0));

    if (kind == 0) {                                     // adler32
        uint64_t s1 = sd & 0xffffu, s2 = (sd >> 16) & 0xffffu;
        const uint64_t nblk = len / 5552, rem = len % 5552, nall = nblk + (rem ? 1u : 0u);
        for (uint64_t c0 = 0; c0 < nall; c0 += CK_BLK) {
            const uint32_t nc = (uint32_t)(nall - c0 < CK_BLK ? nall - c0 : CK_BLK);
            for (uint32_t k = wv; k < nc; k += CK_THREADS / 64) {
                const uint64_t b = c0 + k;
                const uint32_t blen = b < nblk ? 5552u : (uint32_t)rem;
                const uint8_t* q = p + b * 5552;
                // 16-byte aligned pieces covering [q, q + blen): each holds a byte of the block,
                // so no load leaves the pages the buffer lies in; bytes outside are masked off
                const uintptr_t a0 = (uintptr_t)q & ~(uintptr_t)15;
                const uint32_t lead = (uint32_t)((uintptr_t)q - a0), npc = (lead + blen + 15u) >> 4;
                uint32_t T = 0;
                int64_t I = 0;                                // sum i b_i (block index i)
                for (uint32_t c = lane; c < npc; c += 64) {
                    const uint4 v4 = *(const uint4*)(a0 + 16u * (uintptr_t)c);
                    const uint32_t wd[4] = { v4.x, v4.y, v4.z, v4.w };
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int32_t ib = (int32_t)(16u * c + 4u * (uint32_t)j) - (int32_t)lead;   // index of byte 0
                        const int32_t lo = ib < 0 ? -ib : 0, hi = (int32_t)blen - ib;               // valid bytes [lo, hi)
                        const uint32_t mlo = lo >= 4 ? 0u : ~0u << (8 * lo);
                        const uint32_t mhi = hi >= 4 ? ~0u : hi <= 0 ? 0u : (1u << (8 * hi)) - 1u;
                        const uint32_t x = wd[j] & mlo & mhi;
                        const uint32_t sb = __builtin_amdgcn_udot4(x, 0x01010101u, 0u, false);
                        T += sb;
                        I += (int64_t)ib * sb + __builtin_amdgcn_udot4(x, 0x03020100u, 0u, false);
                    }
                }
                for (int o = 32; o > 0; o >>= 1) {
                    T += __shfl_xor(T, o);
                    I += __shfl_xor(I, o);
                }
                if (lane == 0) { ck_T[k] = T; ck_W[k] = (uint64_t)blen * T - (uint64_t)I; }
            }
            __syncthreads();
            if (tid == 0)
                for (uint32_t k = 0; k < nc; ++k) {               // adler32.ts:45-67, block by block
                    const uint64_t b = c0 + k;
                    const uint32_t blen = b < nblk ? 5552u : (uint32_t)rem;
                    s2 += (uint64_t)blen * s1 + ck_W[k];
                    s1 += ck_T[k];
                    if (b < nblk) { s1 %= 65521u; s2 += 65521u; }
                    else { s1 %= 65521u; s2 %= 65521u; }
                }
            __syncthreads();
        }
        if (tid == 0) result[sid] = (int32_t)((uint32_t)s1 | ((uint32_t)s2 << 16));
    } else if (wv == 0) {                                // crc32
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
