// k_checksum.hip -- batched adler32 / crc32 (src/adler32.ts:17-105, src/crc32.ts:17-216).
//
// One wave per buffer.  adler32 is evaluated block-wise on the reference's NMAX
// (5552-byte) grid so the adler32.ts:67 quirk (sum2 += BASE, reduced only when a
// remainder exists) is reproduced exactly: per block the wave reduces the byte
// sum T and the weighted sum W = sum (5552 - i) * b_i, and lane 0 chains
//   sum2 += 5552 * s1 + W + BASE;  s1 = (s1 + T) mod BASE.
// crc32 splits the buffer into 64 lane chunks (byte-wise LDS table) and merges
// them with GF(2) polynomial shifts (x^(8 len) mod P), a log2(64)-step tree.
#include "sdz_internal.h"

namespace sdz {

#define CK_THREADS 64

__device__ uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = b & 1 ? (b >> 1) ^ 0xedb88320u : b >> 1;
    }
    return p;
}

// x^(n * 2^3) mod P, i.e. the shift for n bytes
__device__ uint32_t xbytes(uint64_t n, const uint32_t* x2n) {
    uint32_t p = 1u << 31;
    unsigned k = 3;
    while (n) {
        if (n & 1) p = multmodp(x2n[k & 31], p);
        n >>= 1;
        k++;
    }
    return p;
}

__global__ __launch_bounds__(CK_THREADS) void k_checksum(const uint8_t* in, const uint64_t* in_off,
                                                         const uint64_t* in_len, const int32_t* seed,
                                                         int32_t* result, uint32_t n, int kind) {
    __shared__ uint32_t tab[256];
    __shared__ uint32_t x2n[32];
    uint32_t lane = threadIdx.x;
    for (uint32_t v = lane; v < 256; v += CK_THREADS) {
        uint32_t c = v;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
        tab[v] = c;
    }
    if (lane == 0) {
        uint32_t p = 1u << 30;
        x2n[0] = p;
        for (int k = 1; k < 32; ++k) x2n[k] = p = multmodp(p, p);
    }
    __syncthreads();
    uint32_t sid = blockIdx.x;
    if (sid >= n) return;
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
        uint64_t chunk = (len + CK_THREADS - 1) / CK_THREADS;
        uint64_t b0 = (uint64_t)lane * chunk;
        uint64_t b1 = b0 + chunk < len ? b0 + chunk : len;
        uint64_t clen = b1 > b0 ? b1 - b0 : 0;
        uint32_t c = 0xffffffffu;
        for (uint64_t i = b0; i < b1; ++i) c = tab[(c ^ p[i]) & 255] ^ (c >> 8);
        uint32_t crc = ~c;
        uint64_t l = clen;
        for (int o = 1; o < CK_THREADS; o <<= 1) {
            uint32_t rc = __shfl_down(crc, o);
            uint64_t rl = __shfl_down(l, o);
            if ((lane & (2 * o - 1)) == 0 && lane + o < CK_THREADS) {
                crc = multmodp(xbytes(rl, x2n), crc) ^ rc;
                l += rl;
            }
        }
        if (lane == 0) result[sid] = (int32_t)(multmodp(xbytes(len, x2n), sd) ^ crc);
    }
}

void launch_checksum(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                     const int32_t* seed, int32_t* result, uint32_t n, int kind, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_checksum, dim3(n), dim3(CK_THREADS), 0, s, in, in_off, in_len, seed, result, n, kind);
}

}  // namespace sdz
