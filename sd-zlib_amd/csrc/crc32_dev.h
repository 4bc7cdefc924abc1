// crc32_dev.h -- reflected CRC-32 (poly 0xEDB88320; src/crc32.ts:48-106, 179-216) of one
// buffer per wave, shared by k_checksum (sdz_crc32*, Deflater gzip trailers) and
// k_inflate_finalize (gzip verdicts).
//
// The buffer is cut into 64 lane chunks (multiples of 8 bytes).  Each lane runs
// slicing-by-8 over aligned 8-byte loads (8 LDS table lookups per 8 bytes), and the lane
// CRCs are merged with GF(2) shifts x^(8 n) mod P in a log2(64)-step tree.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace sdz {

struct CrcTables {
    uint32_t t[8][256];               // t[k][b]: CRC of byte b followed by k zero bytes
    uint32_t x2n[32];                 // x^(2^k) mod P
};

__device__ inline uint32_t gf2_mulmod(uint32_t a, uint32_t b) {   // a * b mod P (reflected)
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
__device__ inline uint32_t gf2_xbytes(uint64_t n, const uint32_t* x2n) {   // x^(8 n) mod P
    uint32_t p = 1u << 31;
    unsigned k = 3;
    while (n) {
        if (n & 1) p = gf2_mulmod(x2n[k & 31], p);
        n >>= 1;
        k++;
    }
    return p;
}

// the byte-wise CRC of v (the reference's table, crc32.ts:179-216)
__device__ inline uint32_t crc_byte(uint32_t v) {
    for (int k = 0; k < 8; ++k) v = (v & 1) ? 0xedb88320u ^ (v >> 1) : v >> 1;
    return v;
}
// fill the tables with the whole block; the caller synchronises before use
__device__ inline void crc_tables_init(CrcTables& T) {
    for (uint32_t v = threadIdx.x; v < 256; v += blockDim.x) {
        uint32_t c = crc_byte(v);
        T.t[0][v] = c;
        for (int k = 1; k < 8; ++k) {                    // t[k][v] = (t[k-1][v] >> 8) ^ t[0][t[k-1][v] & 255]
            c = (c >> 8) ^ crc_byte(c & 255u);
            T.t[k][v] = c;
        }
    }
    if (threadIdx.x == 0) {
        uint32_t p = 1u << 30;
        T.x2n[0] = p;
        for (int k = 1; k < 32; ++k) T.x2n[k] = p = gf2_mulmod(p, p);
    }
}

// CRC-32 (init ~0, final ~) of p[0, len), called by one whole wave; the result is valid in
// lane 0
__device__ inline uint32_t crc32_wave(const uint8_t* p, uint64_t len, const CrcTables& T) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t chunk = (((len + 63) >> 6) + 7) & ~7ull;
    const uint64_t b0 = (uint64_t)lane * chunk < len ? (uint64_t)lane * chunk : len;
    const uint64_t b1 = b0 + chunk < len ? b0 + chunk : len;
    const uint8_t* q = p + b0;
    uint64_t n = b1 - b0;
    uint32_t c = 0xffffffffu;
    // head bytes up to 8-byte alignment (the same count for every lane: chunks are 8 x k)
    while (n && ((uintptr_t)q & 7u)) {
        c = T.t[0][(c ^ *q++) & 255u] ^ (c >> 8);
        --n;
    }
    for (; n >= 8; n -= 8, q += 8) {
        const uint2 w = *(const uint2*)q;
        const uint32_t lo = w.x ^ c, hi = w.y;
        c = T.t[7][lo & 255u] ^ T.t[6][(lo >> 8) & 255u] ^ T.t[5][(lo >> 16) & 255u] ^ T.t[4][lo >> 24] ^
            T.t[3][hi & 255u] ^ T.t[2][(hi >> 8) & 255u] ^ T.t[1][(hi >> 16) & 255u] ^ T.t[0][hi >> 24];
    }
    while (n--) c = T.t[0][(c ^ *q++) & 255u] ^ (c >> 8);
    uint32_t crc = ~c;
    uint64_t l = b1 - b0;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t rc = __shfl_down(crc, o);
        const uint64_t rl = __shfl_down(l, o);
        if ((lane & (2 * o - 1)) == 0 && lane + o < 64) {
            crc = gf2_mulmod(gf2_xbytes(rl, T.x2n), crc) ^ rc;
            l += rl;
        }
    }
    return crc;
}

}  // namespace sdz
