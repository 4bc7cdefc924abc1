// k_deflate_fast.hip -- the opt-in fast compressor: valid DEFLATE /
// zlib / gzip streams at GPU throughput, NOT bit-exact with the reference (which the
// bit-exact path, k_deflate.hip, is).  The container, header and trailer follow
// sd-deflate.ts:98-165 (zlib 78 01, gzip with MTIME/FNAME/OS 0xff, adler32 / crc32 of the
// input), so every inflater reads it; the block structure and the matches are this
// kernel's own.
//
// A stream is cut into 8 KiB TILES, each compressed by one workgroup on its own (matches
// reach back to the tile start only) into one dynamic-Huffman block -- or a stored block
// when that is smaller -- that ends on a byte boundary (a non-final tile is followed by an
// empty stored block, as zlib's Z_SYNC_FLUSH does), so the tiles of a stream concatenate as
// bytes (k_fast_concat).  Per tile, in LDS:
//  1. candidates: position p's most recent earlier position with the same 4-byte hash, from
//     a 2048-bucket table filled 256 positions at a time (positions of the same 256-block
//     do not see each other);
//  2. a greedy parse (a match of >= 4 bytes is taken, else a literal), 32 positions per
//     thread from the segment start, then one thread walks the segment boundaries in order
//     and re-parses from where the previous segment's last token really ended until the
//     parse meets the speculative one (greedy parses converge within a few tokens);
//  3. symbol frequencies; literal/length and distance code lengths in parallel: ceil(log2(F/f))
//     per symbol (Kraft sum <= 1), then the gap filled exactly by promoting symbols between
//     length classes (the shortest classes first); canonical codes by wave ballots; the
//     code-length code by two-queue Huffman limited to 7 bits (zlib's gen_bitlen fix);
//  4. every thread packs its tokens at a prefix-summed bit offset (LDS atomics on words).
// LDS ~45 KB per workgroup: three tiles per CU, so one tile's serial steps (the boundary
// walk, the run-length coding) overlap the others' parallel ones.
#include "sdz_internal.h"

namespace sdz {

#define FT_TILE 8192
static_assert(FT_TILE == FT_TILE_BYTES, "tile size shared with the runtime");
#define FT_THREADS 256
#define FT_SEG (FT_TILE / FT_THREADS)          // 32 positions per thread
#define FT_HBITS 11
#define FT_NONE 0xffffu
#define FT_OUT_WORDS ((FT_TILE + 512) / 4)    // output bit buffer (dynamic blocks only when smaller than stored)

__constant__ uint8_t c_ft_border[19] = { 16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15 };

// length 3..258 -> code 257..285 and extra bits; distance 1..32768 -> code 0..29 and extra
__device__ __forceinline__ uint32_t ft_lcode(uint32_t len, uint32_t& eb, uint32_t& ev) {
    const uint32_t x = len - 3u;
    if (len == 258u) { eb = 0; ev = 0; return 285u; }
    if (x < 8u) { eb = 0; ev = 0; return 257u + x; }
    const uint32_t e = 31u - __builtin_clz(x) - 2u;       // x in [4 << e, 8 << e)
    eb = e; ev = x & ((1u << e) - 1u);
    return 257u + 4u * (e + 1u) + ((x >> e) & 3u);
}
__device__ __forceinline__ uint32_t ft_dcode(uint32_t dist, uint32_t& eb, uint32_t& ev) {
    const uint32_t x = dist - 1u;
    if (x < 4u) { eb = 0; ev = 0; return x; }
    const uint32_t e = 31u - __builtin_clz(x) - 1u;       // x in [2 << e, 4 << e)
    eb = e; ev = x & ((1u << e) - 1u);
    return 2u * (e + 1u) + ((x >> e) & 1u);
}

struct FtShared {
    uint32_t src32[FT_TILE / 4 + 4];                      // the tile (+ zero pad for word reads)
    union {
        uint32_t ht[1 << FT_HBITS];                       // step 1: hash -> last position (+1; 0 none)
        uint32_t out[FT_OUT_WORDS];                       // step 4: the block's bits
    };
    uint16_t cand[FT_TILE];                               // earlier position with p's hash, or FT_NONE
    uint8_t mlen[FT_TILE];                                // at token starts: 0 literal, len - 3 for a match
    uint32_t tbits[FT_TILE / 32];                         // token starts
    uint32_t freq[286 + 30 + 19];
    uint16_t code[286 + 30 + 19];                         // bit-reversed canonical codes
    uint8_t clen[286 + 30 + 19];
    uint32_t sortd[32];                                   // the code-length code: (freq << 9 | sym) ascending
    uint32_t rstart[10];                                  // run starts of the code-length sequence
    uint32_t hq[320];                                     // two-queue Huffman: internal node weights
    uint16_t hpar[2 * 286];                               // parent links (leaf i, node 286 + j)
    uint8_t hdep[286], hndep[286];
    uint16_t rle[320];                                    // code-length code symbols (sym | extra << 5)
    uint32_t segbits[FT_THREADS / 64];                    // the waves' bit totals
    uint32_t segend[FT_THREADS];                          // end of the segment's speculative parse
    uint16_t newend[FT_THREADS];                          // end of the chain its word holds now
    uint16_t ent[FT_THREADS];                             // the entry that chain was parsed from
    uint32_t mism[FT_THREADS / 32];                       // segments whose chain may not be the true one
    uint32_t bl[16], blf[16];                             // code lengths: first / final counts per length
    uint32_t misc[12];                                    // 0 nrle, 1 header bits, 2 hlit, 3 hdist, 4 hclen, 5 stored?,
                                                          // 6 end bits, 7 bytes, 8 lit/len count, 9 matches, 10 data bits
};

__device__ __forceinline__ uint32_t ft_byte(const FtShared& S, uint32_t p) { return (S.src32[p >> 2] >> (8 * (p & 3u))) & 255u; }
__device__ __forceinline__ uint32_t ft_word(const FtShared& S, uint32_t p) {   // bytes p .. p+3
    return __builtin_amdgcn_alignbyte(S.src32[(p >> 2) + 1], S.src32[p >> 2], p & 3u);
}
__device__ __forceinline__ bool ft_bit(const FtShared& S, uint32_t p) { return (S.tbits[p >> 5] >> (p & 31u)) & 1u; }

// match length at p against its candidate (0 when none, or shorter than 4)
__device__ __forceinline__ uint32_t ft_match(const FtShared& S, uint32_t p, uint32_t n) {
    const uint32_t c = S.cand[p];
    if (c == FT_NONE) return 0;
    const uint32_t lim = n - p < 258u ? n - p : 258u;
    uint32_t l = 0;
    while (l < lim) {
        const uint32_t x = ft_word(S, p + l) ^ ft_word(S, c + l);
        if (x) { l += __builtin_ctz(x) >> 3; break; }
        l += 4;
    }
    if (l > lim) l = lim;
    return l >= 4 ? l : 0;
}

// One thread: Huffman code lengths, at most maxbits, for the m used symbols key[0 .. m)
// (ascending frequency) into S.clen + f0 (zeroed for the ns symbols first): two-queue
// Huffman (leaves and merged nodes are both consumed in ascending weight), depths from the
// root down, then zlib's overflow fix (deftree.ts:102-131) on the per-length counts with the
// lengths handed out longest-first to the least frequent symbols.
__device__ void ft_lengths(FtShared& S, const uint32_t* key, uint32_t m, uint32_t f0, uint32_t ns, uint32_t maxbits) {
    for (uint32_t s = 0; s < ns; ++s) S.clen[f0 + s] = 0;
    if (m == 0) return;
    if (m == 1) { S.clen[f0 + (key[0] & 511u)] = 1; return; }   // (the caller completes it)
    uint32_t li = 0, ni = 0, nn = 0;
    while (nn < m - 1) {
        uint32_t w[2], id[2];
        for (int q = 0; q < 2; ++q) {
            if (li < m && (ni >= nn || (key[li] >> 9) <= S.hq[ni])) { w[q] = key[li] >> 9; id[q] = li++; }
            else { w[q] = S.hq[ni]; id[q] = 286u + ni++; }
        }
        S.hq[nn] = w[0] + w[1];
        S.hpar[id[0]] = (uint16_t)nn;
        S.hpar[id[1]] = (uint16_t)nn;
        ++nn;
    }
    uint32_t bl[16];
    for (int b = 0; b < 16; ++b) bl[b] = 0;
    S.hndep[nn - 1] = 0;                                 // the root; nodes come after their children
    for (int j = (int)nn - 2; j >= 0; --j) S.hndep[j] = (uint8_t)(S.hndep[S.hpar[286 + j]] + 1);
    uint32_t over = 0;
    for (uint32_t i = 0; i < m; ++i) {
        uint32_t d = S.hndep[S.hpar[i]] + 1u;
        if (d > maxbits) { d = maxbits; ++over; }
        S.hdep[i] = (uint8_t)d;
        bl[d]++;
    }
    if (over) {
        do {
            uint32_t bits = maxbits - 1;
            while (bl[bits] == 0) --bits;
            bl[bits]--;
            bl[bits + 1] += 2;
            bl[maxbits]--;
            over = over >= 2 ? over - 2 : 0;
        } while (over);
        uint32_t i = 0;
        for (uint32_t bits = maxbits; bits >= 1; --bits)
            for (uint32_t k = 0; k < bl[bits]; ++k) S.hdep[i++] = (uint8_t)bits;
    }
    for (uint32_t i = 0; i < m; ++i) S.clen[f0 + (key[i] & 511u)] = S.hdep[i];
}

// All threads: literal/length or distance code lengths for the used symbols of
// freq[f0 .. f0 + ns) (F = their total), no sort: l = ceil(log2(F / f)) keeps the Kraft sum
// <= 1 (2^-l <= f / F) and is <= 15 for F <= 2^15; the gap to exactly 1 -- a multiple of the
// longest class's 2^-l -- is closed by moving symbols one class shorter, the shortest classes
// first (largest steps), in closed form per class and pass.  Final lengths go out in order of
// (first length, symbol): the first bl[1] symbols get 1 bit, and so on -- monotone in the
// frequency up to ties within a class.  Within a few percent of Huffman.
__device__ void ft_lengths_par(FtShared& S, uint32_t f0, uint32_t ns, uint32_t F) {
    const uint32_t tid = threadIdx.x;
    if (tid < 16) S.bl[tid] = 0;                         // bl[0]: used symbols
    __syncthreads();
    for (uint32_t s = tid; s < ns; s += FT_THREADS) {
        const uint32_t f = S.freq[f0 + s];
        uint32_t l = 0;
        if (f) {
            const uint32_t q = (F + f - 1) / f;
            l = q <= 1 ? 1u : 32u - __builtin_clz(q - 1);
            l = l < 15u ? l : 15u;
            atomicAdd(&S.bl[l], 1u);
            atomicAdd(&S.bl[0], 1u);
        }
        S.clen[f0 + s] = (uint8_t)l;                     // the first length
    }
    __syncthreads();
    const uint32_t m = S.bl[0];
    if (m <= 1) {                                        // one code (or none): two codes of length 1
        if (tid == 0) {
            uint32_t s1 = 0;
            for (uint32_t s = 0; s < ns; ++s) if (S.clen[f0 + s]) s1 = s;
            for (uint32_t s = 0; s < ns; ++s) S.clen[f0 + s] = 0;
            S.clen[f0 + s1] = 1;
            S.clen[f0 + (s1 ? 0 : 1)] = 1;
        }
        __syncthreads();
        return;
    }
    if (tid == 0) {
        uint32_t b[16], K = 0;
#pragma unroll
        for (int l = 1; l < 16; ++l) { b[l] = S.bl[l]; K += b[l] << (15 - l); }
        uint32_t G = K < 32768u ? 32768u - K : 0u;
        while (G) {
#pragma unroll
            for (int l = 2; l < 16; ++l) {
                const uint32_t step = 1u << (15 - l), k = b[l] < G / step ? b[l] : G / step;
                b[l] -= k; b[l - 1] += k; G -= k * step;
            }
        }
#pragma unroll
        for (int l = 1; l < 16; ++l) S.blf[l] = b[l];    // final counts
    }
    __syncthreads();
    if (tid < 64) {                                      // ranks by (first length, symbol); wave 0
        const uint32_t lane = tid;
        const uint64_t lt = (1ull << lane) - 1ull;
        uint32_t off[16], cum[16];
        uint32_t acc = 0, accf = 0;
#pragma unroll
        for (int l = 1; l < 16; ++l) { off[l] = acc; acc += S.bl[l]; accf += S.blf[l]; cum[l] = accf; }
        uint32_t fin[5];
#pragma unroll
        for (uint32_t ci = 0; ci < 5; ++ci) {
            const uint32_t c = 64 * ci;
            const uint32_t l0 = c + lane < ns ? S.clen[f0 + c + lane] : 0u;
            uint32_t r = 0;
#pragma unroll
            for (int L = 1; L < 16; ++L) {
                const uint64_t mk = __ballot(l0 == (uint32_t)L);
                if (l0 == (uint32_t)L) r = off[L] + (uint32_t)__popcll(mk & lt);
                off[L] += (uint32_t)__popcll(mk);
            }
            uint32_t lf = 0;
            if (l0) {
                lf = 15;
#pragma unroll
                for (int L = 15; L >= 1; --L) if (r < cum[L]) lf = (uint32_t)L;
            }
            fin[ci] = lf;
        }
#pragma unroll
        for (uint32_t ci = 0; ci < 5; ++ci)               // (all first lengths were read before)
            if (64 * ci + lane < ns) S.clen[f0 + 64 * ci + lane] = (uint8_t)fin[ci];
    }
    __syncthreads();
}

// Wave 0: canonical codes (deftree.ts:155-182), bit-reversed for LSB-first output: counts per
// length and each symbol's rank among its length by ballots over 64-symbol chunks
__device__ void ft_codes_wave(FtShared& S, uint32_t f0, uint32_t ns) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t next[16];
#pragma unroll
    for (int L = 0; L < 16; ++L) next[L] = 0;
    for (uint32_t c = 0; c < ns; c += 64) {
        const uint32_t l = c + lane < ns ? S.clen[f0 + c + lane] : 0u;
#pragma unroll
        for (int L = 1; L < 16; ++L) next[L] += (uint32_t)__popcll(__ballot(l == (uint32_t)L));
    }
    uint32_t code = 0, prev = 0;
#pragma unroll
    for (int L = 1; L < 16; ++L) {                        // counts -> first code of each length
        const uint32_t cntL = next[L];
        code = (code + prev) << 1;
        next[L] = code;
        prev = cntL;
    }
    for (uint32_t c = 0; c < ns; c += 64) {
        const uint32_t l = c + lane < ns ? S.clen[f0 + c + lane] : 0u;
        uint32_t mine = 0;
#pragma unroll
        for (int L = 1; L < 16; ++L) {
            const uint64_t mk = __ballot(l == (uint32_t)L);
            if (l == (uint32_t)L) mine = next[L] + (uint32_t)__popcll(mk & lt);
            next[L] += (uint32_t)__popcll(mk);
        }
        if (c + lane < ns) S.code[f0 + c + lane] = l ? (uint16_t)(__builtin_bitreverse32(mine) >> (32 - l)) : (uint16_t)0;
    }
}

// the parse's step at p: the match there, unless the match at p + 1 is longer (one step of
// lazy evaluation, as deflate_slow does; only for matches shorter than FT_LAZY) -- then a
// literal.  A function of p alone, so parses from different entries still meet.  Off by
// default: FT_LAZY 32 gave ratio 0.520 against 0.523 for 12 % less throughput (C3 layout).
#ifndef FT_LAZY
#define FT_LAZY 0u
#endif
__device__ __forceinline__ uint32_t ft_token(const FtShared& S, uint32_t p, uint32_t n) {
    const uint32_t l = ft_match(S, p, n);
    if (l && l < FT_LAZY && p + 1 < n && ft_match(S, p + 1, n) > l) return 0;
    return l;
}

// All threads: exclusive prefix sum of v over the block; *total = the sum
__device__ __forceinline__ uint32_t ft_scan(FtShared& S, uint32_t v, uint32_t* total) {
    const uint32_t tid = threadIdx.x;
    uint32_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t x = __shfl_up(incl, d);
        if ((tid & 63u) >= (uint32_t)d) incl += x;
    }
    __syncthreads();                                     // (segbits reuse)
    if ((tid & 63u) == 63u) S.segbits[tid >> 6] = incl;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < FT_THREADS / 64; ++w) {
        const uint32_t x = S.segbits[w];
        base += w < (tid >> 6) ? x : 0u;
        tot += x;
    }
    *total = tot;
    return base + incl - v;
}

// a run of r equal code lengths v as send_tree codes them (deflate.ts:378-429): the symbol
// count, and (with out) the symbols (sym | extra << 5)
__device__ __forceinline__ uint32_t ft_run(uint32_t v, uint32_t r, uint16_t* out) {
    uint32_t c = 0, left = r;
    if (v == 0) {
        while (left >= 11) { const uint32_t k = left < 138 ? left : 138; if (out) out[c] = (uint16_t)(18 | ((k - 11) << 5)); ++c; left -= k; }
        if (left >= 3) { if (out) out[c] = (uint16_t)(17 | ((left - 3) << 5)); ++c; left = 0; }
    } else {
        if (out) out[c] = (uint16_t)v;
        ++c;
        --left;
        while (left >= 3) { const uint32_t k = left < 6 ? left : 6; if (out) out[c] = (uint16_t)(16 | ((k - 3) << 5)); ++c; left -= k; }
    }
    while (left) { if (out) out[c] = (uint16_t)v; ++c; --left; }
    return c;
}

// clear the token-start bits of positions [a, b)
__device__ __forceinline__ void ft_clear(FtShared& S, uint32_t a, uint32_t b) {
    while (a < b) {
        const uint32_t w = a >> 5, lo = a & 31u, hi = (b - (a & ~31u)) < 32u ? b - (a & ~31u) : 32u;
        const uint32_t mk = (hi == 32u ? ~0u : (1u << hi) - 1u) & (~0u << lo);
        S.tbits[w] &= ~mk;
        a = (a & ~31u) + 32u;
    }
}

// bits v (n <= 32) at bit offset o of the LDS output
__device__ __forceinline__ void ft_put(FtShared& S, uint32_t o, uint32_t v, uint32_t n) {
    if (!n) return;
    const uint32_t w = o >> 5, sh = o & 31u;
    const uint64_t x = (uint64_t)(n == 32 ? v : (v & ((1u << n) - 1u))) << sh;
    atomicOr(&S.out[w], (uint32_t)x);
    if (sh + n > 32) atomicOr(&S.out[w + 1], (uint32_t)(x >> 32));
}

// one tile: A.in stream tile_stream[t], its tile tile_idx[t]; output bytes to
// tile_out + t * FT_TILE_OUT, length to tile_len[t]
#ifdef FT_TIMING                                         // development aid: phase clocks of tile 0
#define FT_STAMP(k) do { if (t == 0) { __syncthreads(); if (tid == 0) { const unsigned long long c_ = clock64(); \
    ftc[k] = c_ - ftl; ftl = c_; } } } while (0)
#else
#define FT_STAMP(k) do {} while (0)
#endif
__global__ __launch_bounds__(FT_THREADS) void k_fast_tiles(const uint8_t* in, const uint64_t* in_off,
                                                           const uint64_t* in_len, const uint32_t* tile_stream,
                                                           const uint32_t* tile_idx, uint32_t ntiles,
                                                           uint8_t* tile_out, uint32_t* tile_len) {
    __shared__ FtShared S;
    const uint32_t t = blockIdx.x, tid = threadIdx.x;
    if (t >= ntiles) return;
#ifdef FT_TIMING
    unsigned long long ftc[12] = {0}, ftl = clock64();
#endif
    const uint32_t sid = tile_stream[t];
    const uint64_t len = in_len[sid];
    const uint64_t t0 = (uint64_t)tile_idx[t] * FT_TILE;
    const uint32_t n = (uint32_t)(len - t0 < FT_TILE ? len - t0 : FT_TILE);
    const bool last = t0 + n == len;
    const uint8_t* src = in + in_off[sid] + t0;
    // 0. load; clear tables
    for (uint32_t k = tid; k < FT_TILE / 4 + 4; k += FT_THREADS) {
        const uint32_t b = 4 * k;
        uint32_t v = 0;
        if (b + 4 <= n) v = (uint32_t)src[b] | ((uint32_t)src[b + 1] << 8) | ((uint32_t)src[b + 2] << 16) | ((uint32_t)src[b + 3] << 24);
        else for (uint32_t j = 0; j < 4; ++j) if (b + j < n) v |= (uint32_t)src[b + j] << (8 * j);
        S.src32[k] = v;
    }
    for (uint32_t k = tid; k < (1u << FT_HBITS); k += FT_THREADS) S.ht[k] = 0;
    for (uint32_t k = tid; k < FT_TILE / 32; k += FT_THREADS) S.tbits[k] = 0;
    for (uint32_t k = tid; k < 286 + 30 + 19; k += FT_THREADS) S.freq[k] = 0;
    __syncthreads();
    FT_STAMP(0);
    // 1. candidates, 256 positions at a time
    for (uint32_t c = 0; c < n; c += FT_THREADS) {
        const uint32_t p = c + tid;
        const bool ok = p + 4 <= n;
        const uint32_t h = ok ? (ft_word(S, p) * 2654435761u) >> (32 - FT_HBITS) : 0u;
        if (p < n) S.cand[p] = ok && S.ht[h] ? (uint16_t)(S.ht[h] - 1) : (uint16_t)FT_NONE;
        __syncthreads();
        if (ok) atomicMax(&S.ht[h], p + 1);
        __syncthreads();
    }
    FT_STAMP(1);
    // 2. speculative greedy parse of each segment from its start
    {
        const uint32_t s0 = tid * FT_SEG;
        uint32_t p = s0;
        while (p < s0 + FT_SEG && p < n) {
            const uint32_t l = ft_token(S, p, n);
            atomicOr(&S.tbits[p >> 5], 1u << (p & 31u));
            S.mlen[p] = l ? (uint8_t)(l - 3) : 0;
            p += l ? l : 1;
        }
        S.segend[tid] = p;
    }
    __syncthreads();
    FT_STAMP(2);
    // the true parse across segment boundaries.  A segment is one token-start word (32
    // positions).  In parallel, each segment re-parses from where its predecessor's
    // speculative parse ended (the true entry whenever the predecessor's own parse met its
    // speculative one, the usual case) until it meets its speculative parse; it commits the
    // word only when that happens inside the segment.  Then one thread redoes, in order, only
    // the segments whose chain was parsed from a wrong entry.
    if (tid < FT_THREADS / 32) S.mism[tid] = 0;
    __syncthreads();
    {
        const uint32_t k = tid, s0 = k * FT_SEG, s1 = s0 + FT_SEG;
        uint32_t ne = S.segend[k], en = s0;
        if (k > 0 && s0 < n && S.segend[k - 1] > s0) {
            const uint32_t ein = S.segend[k - 1];
            uint32_t w = S.tbits[k];
            bool commit = true;
            if (ein >= s1) { w = 0; ne = ein; }
            else {
                w &= ~((1u << (ein - s0)) - 1u);
                uint32_t q = ein;
                bool conv = false;
                while (q < s1 && q < n) {
                    if ((w >> (q - s0)) & 1u) { conv = true; break; }
                    const uint32_t l = ft_token(S, q, n);
                    w |= 1u << (q - s0);
                    S.mlen[q] = l ? (uint8_t)(l - 3) : 0;
                    const uint32_t q1 = q + (l ? l : 1);
                    const uint32_t hi = q1 < s1 ? q1 - s0 : 32u;          // clear (q, q1) within the word
                    const uint32_t lo = q - s0 + 1;
                    if (lo < 32u) w &= ~((hi == 32u ? ~0u : (1u << hi) - 1u) & (~0u << lo));
                    q = q1;
                }
                if (conv) ne = S.segend[k];
                else if (q <= s1 || q >= n) ne = q;                      // ends at the boundary / the tile's end
                else commit = false;                                      // runs into the next word
            }
            if (commit) { S.tbits[k] = w; en = ein; }
            else ne = S.segend[k];
        }
        S.newend[k] = (uint16_t)ne;
        S.ent[k] = (uint16_t)en;
    }
    __syncthreads();
    {   // consistent: the predecessor's chain ends where ours was parsed from
        const uint32_t k = tid, s0 = k * FT_SEG;
        if (k > 0 && s0 < n) {
            const uint32_t pe = S.newend[k - 1];
            const bool ok = pe == S.ent[k] || (pe <= s0 && S.ent[k] == s0);
            if (!ok) atomicOr(&S.mism[k >> 5], 1u << (k & 31u));
        }
    }
    __syncthreads();
    if (tid == 0) {
        auto next_mism = [&](uint32_t k) -> uint32_t {
            for (; k < FT_THREADS; k = (k | 31u) + 1u) {
                const uint32_t w = S.mism[k >> 5] & (~0u << (k & 31u));
                if (w) return (k & ~31u) + __builtin_ctz(w);
            }
            return FT_THREADS;
        };
        for (uint32_t k = next_mism(1); k < FT_THREADS && k * FT_SEG < n;) {
            uint32_t e = S.newend[k - 1];                // true: everything before k is consistent
            for (;;) {                                   // redo segment k from its true entry e
                const uint32_t s0 = k * FT_SEG, s1 = s0 + FT_SEG;
                uint32_t et;
                if (e >= s1) { ft_clear(S, s0, s1 < n ? s1 : n); et = e; }
                else {
                    ft_clear(S, s0, e);
                    uint32_t q = e;
                    bool conv = false;
                    while (q < s1 && q < n) {
                        if (ft_bit(S, q)) { conv = true; break; }
                        const uint32_t l = ft_token(S, q, n);
                        S.tbits[q >> 5] |= 1u << (q & 31u);
                        S.mlen[q] = l ? (uint8_t)(l - 3) : 0;
                        const uint32_t q1 = q + (l ? l : 1);
                        ft_clear(S, q + 1, q1 < n ? q1 : n);
                        q = q1;
                    }
                    et = conv ? S.newend[k] : q;
                }
                S.newend[k] = (uint16_t)et;              // (the true end now)
                const uint32_t k1 = k + 1;
                if (k1 >= FT_THREADS || k1 * FT_SEG >= n) { k = FT_THREADS; break; }
                const uint32_t s2 = k1 * FT_SEG;
                const bool ok = et == S.ent[k1] || (et <= s2 && S.ent[k1] == s2);
                if (ok && !((S.mism[k1 >> 5] >> (k1 & 31u)) & 1u)) { k = next_mism(k1); break; }
                if (ok) { k = k1; break; }               // (k1 is on the list: the outer loop takes it)
                k = k1;
                e = et;
            }
        }
    }
    for (uint32_t k = tid; k < FT_OUT_WORDS; k += FT_THREADS) S.out[k] = 0;   // (the hash table is done)
    if (tid < 12) S.misc[tid] = 0;
    __syncthreads();
    FT_STAMP(3);
    // 3. frequencies
    {
        const uint32_t s0 = tid * FT_SEG;
        uint32_t nt = 0, nm = 0;
        for (uint32_t tw = s0 < n ? S.tbits[tid] : 0u; tw; tw &= tw - 1) {   // the segment's token starts
            const uint32_t p = s0 + __builtin_ctz(tw);
            ++nt;
            const uint32_t ml = S.mlen[p];
            if (ml == 0) atomicAdd(&S.freq[ft_byte(S, p)], 1u);
            else {
                uint32_t eb, ev;
                ++nm;
                atomicAdd(&S.freq[ft_lcode(ml + 3u, eb, ev)], 1u);
                atomicAdd(&S.freq[286 + ft_dcode(p - S.cand[p], eb, ev)], 1u);
            }
        }
        if (nt) atomicAdd(&S.misc[8], nt);
        if (nm) atomicAdd(&S.misc[9], nm);
    }
    if (tid == 0) S.freq[256] = 1;                       // end of block
    __syncthreads();
    FT_STAMP(4);
    ft_lengths_par(S, 0, 286, S.misc[8] + 1);
    ft_lengths_par(S, 286, 30, S.misc[9] ? S.misc[9] : 1);
    FT_STAMP(5);
    // the data bits (the symbols with their extra bits), in parallel
    for (uint32_t sy = tid; sy < 316; sy += FT_THREADS) {
        const uint32_t f = S.freq[sy];
        if (!f) continue;
        uint32_t eb = 0;
        if (sy < 286) eb = sy > 264 && sy < 285 ? (sy - 261) / 4 : 0;
        else eb = sy - 286 < 4 ? 0 : (sy - 286) / 2 - 1;
        atomicAdd(&S.misc[10], f * (S.clen[sy] + eb));
    }
    // HLIT / HDIST: the last used code of each set
    if (tid < 2) S.misc[2 + tid] = 0;
    __syncthreads();
    for (uint32_t sy = tid; sy < 316; sy += FT_THREADS)
        if (S.clen[sy]) atomicMax(&S.misc[sy < 286 ? 2 : 3], sy < 286 ? sy + 1 : sy - 285);
    for (uint32_t k = tid; k < 19; k += FT_THREADS) S.freq[316 + k] = 0;
    if (tid < 10) S.rstart[tid] = 0;
    __syncthreads();
    const uint32_t hlit = S.misc[2] > 257 ? S.misc[2] : 257, hdist = S.misc[3] > 1 ? S.misc[3] : 1;
    const uint32_t tot = hlit + hdist;
    auto cl = [&](uint32_t i) -> uint32_t { return i < hlit ? S.clen[i] : S.clen[286 + i - hlit]; };
    // the code-length sequence, run-length coded: runs start where a length changes; each
    // run's symbols go to a prefix-summed place (two positions per thread)
    uint32_t rv[2] = {0, 0}, rr[2] = {0, 0}, rc[2] = {0, 0};
    bool st[2] = {false, false};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t i = 2 * tid + j;
        st[j] = i < tot && (i == 0 || cl(i) != cl(i - 1));
        if (st[j]) atomicOr(&S.rstart[i >> 5], 1u << (i & 31u));
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (!st[j]) continue;
        const uint32_t i = 2 * tid + j;
        uint32_t nx = tot;                               // the next run's start
        for (uint32_t w = (i + 1) >> 5; w < 10 && (w << 5) < tot; ++w) {
            const uint32_t mk = S.rstart[w] & (w == ((i + 1) >> 5) ? ~0u << ((i + 1) & 31u) : ~0u);
            if (mk) { nx = (w << 5) + __builtin_ctz(mk); break; }
        }
        const uint32_t v = cl(i), r = (nx < tot ? nx : tot) - i;
        rv[j] = v; rr[j] = r; rc[j] = ft_run(v, r, nullptr);
    }
    uint32_t nr;
    const uint32_t rbase = ft_scan(S, rc[0] + rc[1], &nr);
    if (rc[0]) ft_run(rv[0], rr[0], S.rle + rbase);
    if (rc[1]) ft_run(rv[1], rr[1], S.rle + rbase + rc[0]);
    __syncthreads();
    for (uint32_t k = tid; k < nr; k += FT_THREADS) atomicAdd(&S.freq[316 + (S.rle[k] & 31u)], 1u);
    __syncthreads();
    if (tid < 19) {                                      // the code-length code's used symbols, ranked
        const uint32_t f = S.freq[316 + tid];
        if (f) {
            const uint32_t v = (f << 9) | tid;
            uint32_t rk = 0;
            for (uint32_t k = 0; k < 19; ++k) {
                const uint32_t g = S.freq[316 + k];
                rk += g && ((g << 9) | k) < v;
            }
            S.sortd[rk] = v;
        }
    }
    __syncthreads();
    if (tid == 0) {                                      // the code-length code (19 symbols, <= 7 bits)
        uint32_t mb = 0;
        for (uint32_t k = 0; k < 19; ++k) mb += S.freq[316 + k] != 0;
        ft_lengths(S, S.sortd, mb, 316, 19, 7);
        uint32_t nb = 0, b0 = 0;
        for (uint32_t sy = 0; sy < 19; ++sy) if (S.clen[316 + sy]) { ++nb; b0 = sy; }
        if (nb == 1) S.clen[316 + (b0 ? 0 : 1)] = 1;     // (complete: two codes of length 1)
        uint32_t hclen = 19;
        while (hclen > 4 && !S.clen[316 + c_ft_border[hclen - 1]]) --hclen;
        S.misc[0] = nr; S.misc[4] = hclen;
    }
    __syncthreads();
    FT_STAMP(6);
    if (tid < 64) {
        ft_codes_wave(S, 0, 286);
        ft_codes_wave(S, 286, 30);
        ft_codes_wave(S, 316, 19);
    }
    __syncthreads();
    // the block header: 17 fixed bits, HCLEN + 4 3-bit lengths, then the run-length symbols at
    // prefix-summed offsets (two per thread)
    const uint32_t hclen = S.misc[4];
    const uint32_t h0 = 17 + 3 * hclen;
    uint32_t hb[2] = {0, 0};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t k = 2 * tid + j;
        if (k < nr) {
            const uint32_t sy = S.rle[k] & 31u;
            hb[j] = S.clen[316 + sy] + (sy == 16 ? 2 : sy == 17 ? 3 : sy == 18 ? 7 : 0);
        }
    }
    uint32_t hbits;
    const uint32_t hbase = ft_scan(S, hb[0] + hb[1], &hbits);
    const uint64_t bits = (uint64_t)h0 + hbits + S.misc[10];
    const bool stored_blk = bits + 7 >= 8ull * (n + 5);
    if (!stored_blk) {
        if (tid == 0) {
            uint32_t o = 0;
            ft_put(S, o, last ? 5u : 4u, 3); o += 3;      // BFINAL, BTYPE = 2
            ft_put(S, o, hlit - 257, 5); o += 5;
            ft_put(S, o, hdist - 1, 5); o += 5;
            ft_put(S, o, hclen - 4, 4); o += 4;
            for (uint32_t k = 0; k < hclen; ++k) { ft_put(S, o, S.clen[316 + c_ft_border[k]], 3); o += 3; }
        }
        uint32_t o = h0 + hbase;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t k = 2 * tid + j;
            if (k < nr) {
                const uint32_t sy = S.rle[k] & 31u, ex = S.rle[k] >> 5;
                ft_put(S, o, S.code[316 + sy], S.clen[316 + sy]);
                const uint32_t eb = sy == 16 ? 2 : sy == 17 ? 3 : sy == 18 ? 7 : 0;
                ft_put(S, o + S.clen[316 + sy], ex, eb);
                o += hb[j];
            }
        }
    }
    if (tid == 0) { S.misc[5] = stored_blk; S.misc[1] = h0 + hbits; }
    __syncthreads();
    FT_STAMP(7);
    const bool stored = S.misc[5] != 0;
    uint32_t total_bytes;
    if (!stored) {
        // 4. each thread's bits, a block scan, then the tokens at their offsets
        const uint32_t s0 = tid * FT_SEG;
        uint32_t mine = 0;
        for (uint32_t tw = s0 < n ? S.tbits[tid] : 0u; tw; tw &= tw - 1) {   // the segment's token starts
            const uint32_t p = s0 + __builtin_ctz(tw);
            const uint32_t ml = S.mlen[p];
            if (ml == 0) { mine += S.clen[ft_byte(S, p)]; continue; }
            uint32_t eb, ev, db, dv;
            const uint32_t lc = ft_lcode(ml + 3u, eb, ev), dc = ft_dcode(p - S.cand[p], db, dv);
            mine += S.clen[lc] + eb + S.clen[286 + dc] + db;
        }
        // exclusive block scan of the threads' bits: wave scans, then the wave totals
        uint32_t incl = mine;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t v = __shfl_up(incl, d);
            if ((tid & 63u) >= (uint32_t)d) incl += v;
        }
        if ((tid & 63u) == 63u) S.segbits[tid >> 6] = incl;
        __syncthreads();
        uint32_t base = S.misc[1];
        for (uint32_t w = 0; w < (tid >> 6); ++w) base += S.segbits[w];
        if (tid == FT_THREADS - 1) S.misc[6] = base + incl;   // end of the data bits
        __syncthreads();
        // this thread's bits [o, o + mine): gathered in a register, whole words stored; the
        // first and last words are shared with the neighbours (atomic OR)
        const uint32_t o0 = base + incl - mine;
        uint32_t w = o0 >> 5, na = o0 & 31u;
        uint64_t acc = 0;
        bool first = true;
        auto put = [&](uint32_t v, uint32_t nb) {
            acc |= (uint64_t)v << na;
            na += nb;
            if (na >= 32) {
                if (first) { atomicOr(&S.out[w], (uint32_t)acc); first = false; }
                else S.out[w] = (uint32_t)acc;
                ++w;
                acc >>= 32;
                na -= 32;
            }
        };
        for (uint32_t tw = s0 < n ? S.tbits[tid] : 0u; tw; tw &= tw - 1) {   // the segment's token starts
            const uint32_t p = s0 + __builtin_ctz(tw);
            const uint32_t ml = S.mlen[p];
            if (ml == 0) {
                const uint32_t b = ft_byte(S, p);
                put(S.code[b], S.clen[b]);
                continue;
            }
            uint32_t eb, ev, db, dv;
            const uint32_t lc = ft_lcode(ml + 3u, eb, ev), dc = ft_dcode(p - S.cand[p], db, dv);
            put(S.code[lc] | (ev << S.clen[lc]), S.clen[lc] + eb);                  // <= 20 bits
            put(S.code[286 + dc] | (dv << S.clen[286 + dc]), S.clen[286 + dc] + db);  // <= 28 bits
        }
        if (na) atomicOr(&S.out[w], (uint32_t)acc);
        __syncthreads();
        if (tid == 0) {
            uint32_t e = S.misc[6];
            ft_put(S, e, S.code[256], S.clen[256]); e += S.clen[256];     // end of block
            if (!last) {                                 // Z_SYNC_FLUSH: empty stored block, byte aligned
                e += 3;                                  // BFINAL 0, BTYPE 00
                e = (e + 7) & ~7u;
                ft_put(S, e, 0xffff0000u, 32); e += 32;
            } else {
                e = (e + 7) & ~7u;
            }
            S.misc[7] = e >> 3;
        }
        __syncthreads();
        total_bytes = S.misc[7];
    } else {
        // a stored block (infblocks.ts:243-333): BFINAL/BTYPE 00 in a byte, LEN, NLEN, data
        total_bytes = 5 + n;
        uint8_t* o8 = (uint8_t*)S.out;
        if (tid == 0) {
            o8[0] = last ? 1 : 0;
            o8[1] = (uint8_t)n; o8[2] = (uint8_t)(n >> 8);
            o8[3] = (uint8_t)~n; o8[4] = (uint8_t)(~n >> 8);
        }
        for (uint32_t k = tid; k < n; k += FT_THREADS) o8[5 + k] = (uint8_t)ft_byte(S, k);
        __syncthreads();
    }
    FT_STAMP(8);
    uint8_t* dst = tile_out + (uint64_t)t * FT_TILE_OUT;
    const uint8_t* o8 = (const uint8_t*)S.out;
    for (uint32_t k = tid; k < total_bytes; k += FT_THREADS) dst[k] = o8[k];
    if (tid == 0) tile_len[t] = total_bytes;
#ifdef FT_TIMING
    FT_STAMP(9);
    if (t == 0 && tid == 0)
        printf("ft phases: load %llu cand %llu parse %llu fix %llu freq %llu lens %llu rle %llu codes+hdr %llu enc %llu out %llu\n",
               ftc[0], ftc[1], ftc[2], ftc[3], ftc[4], ftc[5], ftc[6], ftc[7], ftc[8], ftc[9]);
#endif
}

// per stream: header (sd-deflate.ts:98-152), the tiles' bytes in order, trailer (154-165)
__global__ __launch_bounds__(256) void k_fast_concat(DeflateArgs A, const uint32_t* tile0, const uint8_t* tile_out,
                                                     const uint32_t* tile_len, const int32_t* cks) {
    __shared__ uint64_t pos[1];
    const uint32_t sid = blockIdx.x;
    if (sid >= A.n) return;
    const uint64_t len = A.in_len[sid];
    uint8_t* out = A.out + A.out_off[sid];
    const uint64_t cap = A.out_cap[sid];
    sdz_deflate_record R;
    R.status = SDZ_OK; R.checksum = cks[sid]; R.out_len = 0; R.reserved = 0;
    if (len == 0) {                                      // sd-deflate.ts:180-182 + 232-234
        if (threadIdx.x == 0) { R.status = SDZ_DATA_ERROR; R.checksum = 0; A.rec[sid] = R; }
        return;
    }
    const bool gzip = A.format == SDZ_DEFLATE_GZIP;
    const uint64_t hdr = A.format == SDZ_DEFLATE_ZLIB ? 2 : gzip ? 10 + (A.fname_len ? A.fname_len + 1 : 0) : 0;
    const uint64_t tl = A.format == SDZ_DEFLATE_ZLIB ? 4 : gzip ? 8 : 0;
    const uint32_t nt = (uint32_t)((len + FT_TILE - 1) / FT_TILE);
    uint64_t total = hdr + tl;
    for (uint32_t k = 0; k < nt; ++k) total += tile_len[tile0[sid] + k];
    if (total > cap) {
        if (threadIdx.x == 0) { R.status = SDZ_OUT_OVERFLOW; A.rec[sid] = R; }
        return;
    }
    if (threadIdx.x == 0) {
        if (A.format == SDZ_DEFLATE_ZLIB) { out[0] = 0x78; out[1] = 0x01; }
        else if (gzip) {
            out[0] = 0x1f; out[1] = 0x8b; out[2] = 8; out[3] = A.fname_len ? 8 : 0;
            out[4] = (uint8_t)A.mtime; out[5] = (uint8_t)(A.mtime >> 8);
            out[6] = (uint8_t)(A.mtime >> 16); out[7] = (uint8_t)(A.mtime >> 24);
            out[8] = 0; out[9] = 0xff;
            for (uint32_t i = 0; i < A.fname_len; i++) out[10 + i] = A.fname[i];
            if (A.fname_len) out[10 + A.fname_len] = 0;
        }
        pos[0] = hdr;
    }
    __syncthreads();
    uint64_t o = pos[0];
    for (uint32_t k = 0; k < nt; ++k) {
        const uint32_t tk = tile0[sid] + k, tb = tile_len[tk];
        const uint8_t* s = tile_out + (uint64_t)tk * FT_TILE_OUT;
        for (uint32_t j = threadIdx.x; j < tb; j += 256) out[o + j] = s[j];
        o += tb;
    }
    if (threadIdx.x == 0) {
        const uint32_t c = (uint32_t)cks[sid], z = (uint32_t)len;
        if (A.format == SDZ_DEFLATE_ZLIB) {
            out[o] = (uint8_t)(c >> 24); out[o + 1] = (uint8_t)(c >> 16); out[o + 2] = (uint8_t)(c >> 8); out[o + 3] = (uint8_t)c;
        } else if (gzip) {
            for (int k = 0; k < 4; k++) out[o + k] = (uint8_t)(c >> (8 * k));
            for (int k = 0; k < 4; k++) out[o + 4 + k] = (uint8_t)(z >> (8 * k));
        }
        R.out_len = total;
        A.rec[sid] = R;
    }
}

void launch_fast_tiles(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, const uint32_t* tile_stream,
                       const uint32_t* tile_idx, uint32_t ntiles, uint8_t* tile_out, uint32_t* tile_len, hipStream_t s) {
    if (ntiles) hipLaunchKernelGGL(k_fast_tiles, dim3(ntiles), dim3(FT_THREADS), 0, s, in, in_off, in_len, tile_stream,
                                   tile_idx, ntiles, tile_out, tile_len);
}
void launch_fast_concat(const DeflateArgs& a, const uint32_t* tile0, const uint8_t* tile_out, const uint32_t* tile_len,
                        const int32_t* cks, hipStream_t s) {
    if (a.n) hipLaunchKernelGGL(k_fast_concat, dim3(a.n), dim3(256), 0, s, a, tile0, tile_out, tile_len, cks);
}

}  // namespace sdz
