// k_inflate.hip -- batched DEFLATE decoder for gfx950 (MI355X).
//
// Replaces the serial hot path of @stardazed/zlib's inflate:
//   Inflate.inflate container FSM   src/inflate.ts:132-473
//   InfBlocks.proc block FSM        src/infblocks.ts:123-628
//   InfCodes inflate_fast / proc    src/infcodes.ts:62-676
//   huft_build + tree builders      src/inftree.ts:95-392
//   Inflater.append/finish verdicts src/sd-inflate.ts:87-179
//
// Design: one LANE per stream.  A batch of independent streams is
// the only parallelism DEFLATE offers without changing the format, and a wave
// that decodes 64 streams in lock-step spends one wave-instruction per 64 symbols,
// where a wave-per-stream decoder spends tens of wave-instructions per symbol.
//  * Huffman decode is table-free in registers: canonical left-justified limits
//    (15 per tree) are compared against the 15 bit-reversed peek bits; only the
//    symbol-by-rank array lives in LDS (612 B per stream -> 256 streams per CU).
//  * Output goes straight to its final HBM slot through an 8-byte aligned
//    accumulator; the slot IS the LZ77 window, matches copy aligned 64-bit words
//    (funnel shift) so stores are whole words.
//  * adler32 / crc32 are fused into the word store (dot4 weighted sums /
//    slicing-by-4 LDS tables): the output is never re-read for checksums.
//  * Block headers are processed in "phases": lanes that hit end-of-block wait
//    until 1/8 of the wave is waiting, then all waiting lanes build their tables
//    together, so the wave does not serialise on one lane's header at a time.
// Reference quirks mirrored: root-bits "need" at end of
// input (infcodes.ts:368-387), huft_build's MANY=1400 table budget, incomplete
// single-code trees, distances before the output start reading zeros/dictionary
// (A12), the gzip FEXTRA mode that never advances (inflate.ts:343-345), the
// Inflater's chunk-wise adler32 with the NMAX quirk (adler32.ts:67).
#include "sdz_internal.h"

namespace sdz {

#define IL_THREADS 256
#define IL_REGION 612                 // bytes of LDS per stream (153 dwords: odd stride)
#define IL_DSYM 576                   // distance symbols follow 288 u16 lit/len symbols
#define IL_CRC_OFF (IL_THREADS * IL_REGION)
#define IL_LDS (IL_CRC_OFF + 4096)

__constant__ uint8_t c_border[19] = { 16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15 };

enum : int { LM_TYPE = 0, LM_CODES = 1, LM_TRAILER = 2, LM_DONE = 3 };
enum : int { CK_NONE = 0, CK_ADLER = 1, CK_CRC = 2 };

struct Dec {                          // canonical decoder for one tree
    uint32_t lim[16];                 // left-justified (15-bit) limit per length
    int32_t off[16];                  // rank offset per length
    uint32_t c[5];                    // code counts per length, 3 x 10 bits per word (+dummies)
    int l, g;                         // huft_build root bits and max length
};

struct Lane {
    // bit reader
    const uint4* vp;
    uint4 cur, nxt;
    int ncur;
    uint64_t buf;
    int cnt;
    uint64_t loaded, total;
    // output
    uint64_t* ob;
    uint64_t pos, cap, acc;
    // checksums
    int ck;
    uint32_t s1, s2, crc, snap1, snap2;
    // state
    int mode, last, container, status, zmsg, fixed, nl, nd;
    int32_t stored_ck, stored_size, mtime;
    uint32_t name_off, name_len;
    uint8_t* lens;                    // global scratch for code lengths
    const uint8_t* dict;
    uint32_t dict_len;
};

// ------------------------------------------------------------------ bit reader

__device__ __forceinline__ void br_refill(Lane& L) {
    if (L.cnt <= 32) {
        L.buf |= (uint64_t)L.cur.x << L.cnt;
        L.cnt += 32;
        L.loaded += 32;
        L.cur.x = L.cur.y; L.cur.y = L.cur.z; L.cur.z = L.cur.w;
        if (--L.ncur == 0) { L.cur = L.nxt; L.nxt = *L.vp++; L.ncur = 4; }
    }
}
__device__ __forceinline__ int64_t br_avail(const Lane& L) {
    return (int64_t)L.total - (int64_t)(L.loaded - (uint64_t)L.cnt);
}
__device__ __forceinline__ uint64_t br_consumed(const Lane& L) { return L.loaded - (uint64_t)L.cnt; }
__device__ __forceinline__ uint32_t br_peek(const Lane& L, int n) {
    return (uint32_t)L.buf & ((1u << n) - 1u);
}
__device__ __forceinline__ void br_drop(Lane& L, int n) { L.buf >>= n; L.cnt -= n; }
// read n <= 24 bits; returns false (stall) if the input does not hold them
__device__ __forceinline__ bool br_get(Lane& L, int n, uint32_t& v) {
    br_refill(L);
    if (br_avail(L) < n) return false;
    v = br_peek(L, n);
    br_drop(L, n);
    return true;
}

// ------------------------------------------------------------------ checksums

__device__ __forceinline__ void ck_word(Lane& L, uint64_t w, const uint32_t* crct) {
    uint32_t lo = (uint32_t)w, hi = (uint32_t)(w >> 32);
    if (L.ck == CK_ADLER) {
        uint32_t sum = __builtin_amdgcn_udot4(lo, 0x01010101u, __builtin_amdgcn_udot4(hi, 0x01010101u, 0u, false), false);
        uint32_t wsum = __builtin_amdgcn_udot4(lo, 0x05060708u, __builtin_amdgcn_udot4(hi, 0x01020304u, 0u, false), false);
        uint32_t s2 = L.s2 + 8u * L.s1 + wsum;
        uint32_t s1 = L.s1 + sum;
        L.s1 = s1 >= 65521u ? s1 - 65521u : s1;
        L.s2 = s2 % 65521u;
    } else if (L.ck == CK_CRC) {
        uint32_t c = L.crc ^ lo;
        c = crct[768 + (c & 255)] ^ crct[512 + ((c >> 8) & 255)] ^ crct[256 + ((c >> 16) & 255)] ^ crct[c >> 24];
        c ^= hi;
        c = crct[768 + (c & 255)] ^ crct[512 + ((c >> 8) & 255)] ^ crct[256 + ((c >> 16) & 255)] ^ crct[c >> 24];
        L.crc = c;
    }
}

__device__ __forceinline__ void ck_byte(Lane& L, uint32_t b, const uint32_t* crct) {
    if (L.ck == CK_ADLER) {
        L.s1 += b; if (L.s1 >= 65521u) L.s1 -= 65521u;
        L.s2 += L.s1; if (L.s2 >= 65521u) L.s2 -= 65521u;
    } else if (L.ck == CK_CRC) {
        L.crc = crct[(L.crc ^ b) & 255] ^ (L.crc >> 8);
    }
}

// ------------------------------------------------------------------ output

__device__ __forceinline__ void word_done(Lane& L, uint64_t widx, uint64_t w, const uint32_t* crct) {
    L.ob[widx] = w;
    ck_word(L, w, crct);
    if (((widx + 1) & 2047u) == 0) { L.snap1 = L.s1; L.snap2 = L.s2; }   // 16 KiB chunk boundary
}

__device__ __forceinline__ void put_byte(Lane& L, uint32_t b, const uint32_t* crct) {
    L.acc |= (uint64_t)b << ((L.pos & 7) * 8);
    L.pos++;
    if ((L.pos & 7) == 0) { word_done(L, (L.pos >> 3) - 1, L.acc, crct); L.acc = 0; }
}

// byte at output offset s (s < pos); s < 0 reads the preset dictionary / zeros (A12)
__device__ __forceinline__ uint32_t get_byte(const Lane& L, int64_t s) {
    if (s < 0) {
        int64_t d = (int64_t)L.dict_len + s;
        return d >= 0 ? (uint32_t)L.dict[d] : 0u;
    }
    if ((uint64_t)s >= (L.pos & ~7ull)) return (uint32_t)(L.acc >> ((s & 7) * 8)) & 255u;
    return ((const uint8_t*)L.ob)[s];
}

__device__ __forceinline__ void copy_slow(Lane& L, uint32_t len, uint32_t dist, const uint32_t* crct) {
    for (uint32_t k = 0; k < len; ++k) {
        uint32_t b = get_byte(L, (int64_t)L.pos - (int64_t)dist);
        put_byte(L, b, crct);
    }
}

// LZ77 copy; the output slot is the window (src = already-written output)
__device__ __forceinline__ void copy_match(Lane& L, uint32_t len, uint32_t dist, const uint32_t* crct) {
    if (dist < 8 || (uint64_t)dist > L.pos) { copy_slow(L, len, dist, crct); return; }
    uint64_t end = L.pos + len;
    uint64_t W = L.pos & ~7ull;
    uint64_t acc = L.acc;
    while (W < end) {
        int64_t sw = (int64_t)W - (int64_t)dist;          // source of output byte W (>= -7)
        int64_t a = sw >> 3;
        uint32_t sh = (uint32_t)(sw & 7) * 8;
        uint64_t lo = a >= 0 ? L.ob[a] : 0ull;
        uint64_t val = lo;
        if (sh) { uint64_t hi = L.ob[a + 1]; val = (lo >> sh) | (hi << (64 - sh)); }
        uint32_t o0 = W < L.pos ? (uint32_t)(L.pos - W) : 0u;
        uint64_t rem = end - W;
        uint64_t m = rem >= 8 ? ~0ull : ((1ull << (rem * 8)) - 1ull);
        m &= ~((1ull << (o0 * 8)) - 1ull);
        acc |= val & m;
        if (rem >= 8) { word_done(L, W >> 3, acc, crct); acc = 0; }
        W += 8;
    }
    L.acc = acc;
    L.pos = end;
}

// ------------------------------------------------------------------ canonical decoders

__device__ __forceinline__ uint32_t cnt_get(const uint32_t (&c)[5], int len) {
    int i = (len - 1) / 3;
    uint32_t w = i == 0 ? c[0] : i == 1 ? c[1] : i == 2 ? c[2] : i == 3 ? c[3] : c[4];
    return (w >> (((len - 1) - 3 * i) * 10)) & 1023u;
}
__device__ __forceinline__ void cnt_add(uint32_t (&c)[5], int len, uint32_t v) {
    int i = (len - 1) / 3;
    uint32_t d = v << (((len - 1) - 3 * i) * 10);
    c[0] += i == 0 ? d : 0u; c[1] += i == 1 ? d : 0u; c[2] += i == 2 ? d : 0u;
    c[3] += i == 3 ? d : 0u; c[4] += i == 4 ? d : 0u;
}

// rank of the code whose bit-reversed 15-bit prefix is rc; sets len (16 = invalid)
__device__ __forceinline__ int32_t hdecode(uint32_t rc, const Dec& D, int& len) {
    int l = 1;
    int32_t off = D.off[1];
#pragma unroll
    for (int k = 1; k < 15; ++k) {
        bool ge = rc >= D.lim[k];
        l = ge ? k + 1 : l;
        off = ge ? D.off[k + 1] : off;
    }
    len = l;
    return off + (int32_t)(rc >> (15 - l));
}

// inftree.ts:212-296 table allocation replayed over counts only (c[g] already holds
// the dummy codes): returns the entries allocated; need = bits the reference's
// slow path must have available to resolve the code of canonical rank `target`.
__device__ __noinline__ int huft_replay(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t c4,
                                        int kmin, int g, int l, int target, int* need) {
    uint32_t c[5] = { c0, c1, c2, c3, c4 };
    int i = 0, p = 0, h = -1, w = -l, entries = 0;
    int x1 = 0, x2 = 0, x3 = 0, t0 = 0, t1 = 0, t2 = 0, t3 = 0;
    for (int k = kmin; k <= g; ++k) {
        int a = (int)cnt_get(c, k);
        while (a-- != 0) {
            while (k > w + l) {
                h++;
                w += l;
                int z = g - w;
                z = z > l ? l : z;
                int j = k - w;
                int f = 1 << j;
                if (f > a + 1) {
                    f -= a + 1;
                    int xp = k;
                    if (j < z) {
                        while (++j < z) {
                            f <<= 1;
                            int cx = (int)cnt_get(c, ++xp);
                            if (f <= cx) break;
                            f -= cx;
                        }
                    }
                }
                entries += 1 << j;
                if (h == 0) t0 = j; else if (h == 1) { t1 = j; x1 = i; }
                else if (h == 2) { t2 = j; x2 = i; } else { t3 = j; x3 = i; }
            }
            if (p == target) *need = w + (h == 0 ? t0 : h == 1 ? t1 : h == 2 ? t2 : t3);
            p++;
            int j = 1 << (k - 1);
            while (i & j) { i ^= j; j >>= 1; }
            i ^= j;
            int mask = (1 << w) - 1;
            while (h > 0 && (i & mask) != (h == 1 ? x1 : h == 2 ? x2 : x3)) {
                h--;
                w -= l;
                mask = (1 << w) - 1;
            }
        }
    }
    return entries;
}

// code-length statistics of lens[0..n) -> D (counts, Kraft), returns kraft remainder at 15
struct BuildInfo { int kmin, g, left, nlong; bool allzero; };

__device__ __forceinline__ void finish_dec(Dec& D, const BuildInfo& bi) {
    uint32_t code = 0;
    int32_t idx = 0;
#pragma unroll
    for (int L = 1; L <= 15; ++L) {
        uint32_t cl = cnt_get(D.c, L);
        D.lim[L] = (code + cl) << (15 - L);
        D.off[L] = idx - (int32_t)code;
        idx += (int32_t)cl;
        code = (code + cl) << 1;
    }
    D.lim[0] = 0; D.off[0] = 0;
}

// counts + Kraft for n lengths read from global memory
__device__ __forceinline__ BuildInfo count_lens(Dec& D, const uint8_t* lens, int n, int root) {
    D.c[0] = D.c[1] = D.c[2] = D.c[3] = D.c[4] = 0;
    for (int s = 0; s < n; ++s) {
        int len = lens[s];
        if (len) cnt_add(D.c, len, 1u);
    }
    BuildInfo bi;
    int left = 1, kmin = 16, g = 0;
#pragma unroll
    for (int L = 1; L <= 15; ++L) {
        int cl = (int)cnt_get(D.c, L);
        left = 2 * left - cl;
        if (cl) { kmin = kmin > L ? L : kmin; g = L; }
    }
    bi.allzero = g == 0;
    bi.kmin = kmin;
    bi.g = g;
    bi.left = left;
    int l = root;
    if (!bi.allzero) { if (l < kmin) l = kmin; if (l > g) l = g; }
    D.l = l;
    D.g = g;
    int nlong = 0;
#pragma unroll
    for (int L = 1; L <= 15; ++L) nlong += L > l ? (int)cnt_get(D.c, L) : 0;
    bi.nlong = nlong;
    return bi;
}

// place symbols 0..n-1 into the LDS rank array (canonical order)
template <typename T>
__device__ __forceinline__ void place_syms(const Dec& D, const uint8_t* lens, int n, T* out) {
    uint32_t nx[5] = { 0, 0, 0, 0, 0 };
    uint32_t idx = 0;
#pragma unroll
    for (int L = 1; L <= 15; ++L) { cnt_add(nx, L, idx); idx += cnt_get(D.c, L); }
    for (int s = 0; s < n; ++s) {
        int len = lens[s];
        if (len) {
            uint32_t k = cnt_get(nx, len);
            out[k] = (T)s;
            cnt_add(nx, len, 1u);
        }
    }
}

// add huft_build's dummy codes (c[g] += y) so the replay sees its counts
__device__ __forceinline__ void add_dummies(Dec& D, const BuildInfo& bi) {
    if (!bi.allzero && bi.left > 0) cnt_add(D.c, bi.g, (uint32_t)(bi.left >> (15 - bi.g)));
}
__device__ __forceinline__ void remove_dummies(Dec& D, const BuildInfo& bi) {
    if (!bi.allzero && bi.left > 0) cnt_add(D.c, bi.g, (uint32_t)(-(int)(bi.left >> (15 - bi.g))));
}

// bits the reference's slow path needs before it can resolve this code (infcodes.ts:367-387)
__device__ __noinline__ int dec_need(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t c4,
                                     int l, int kmin, int g, int left, int len, int rank) {
    if (len <= l) return l;
    uint32_t c[5] = { c0, c1, c2, c3, c4 };
    if (left > 0) cnt_add(c, g, (uint32_t)(left >> (15 - g)));
    int need = l;
    huft_replay(c[0], c[1], c[2], c[3], c[4], kmin, g, l, rank, &need);
    return need;
}
#define DEC_NEED(D, B, len, rank) \
    dec_need((D).c[0], (D).c[1], (D).c[2], (D).c[3], (D).c[4], (D).l, (B).kmin, (B).g, (B).left, (len), (rank))

// upper bound on the entries huft_build allocates for these counts (dummies included)
__device__ __forceinline__ int table_bound(const uint32_t (&c)[5], int l, int g) {
    if (g <= l) return 1 << l;
    uint32_t M = 0;
    int nlong2 = 0;
#pragma unroll
    for (int L = 1; L <= 15; ++L) {
        uint32_t cl = cnt_get(c, L);
        M += L > l ? cl << (15 - L) : 0u;
        nlong2 += L > 2 * l ? (int)cl : 0;
    }
    int npref = (int)((M + (1u << (15 - l)) - 1u) >> (15 - l));
    int s1 = g - l < l ? g - l : l;
    int b = (1 << l) + npref * (1 << s1);
    if (g > 2 * l) { int s2 = g - 2 * l < l ? g - 2 * l : l; b += nlong2 * (1 << s2); }
    return b;
}

// ------------------------------------------------------------------ block setup

__device__ __forceinline__ void setup_fixed(Lane& L, Dec& LL, Dec& DD, BuildInfo& bll, BuildInfo& bdd, uint8_t* region) {
    uint16_t* ll = (uint16_t*)region;
    uint8_t* dd = region + IL_DSYM;
    int k = 0;
    for (int s = 256; s < 280; ++s) ll[k++] = (uint16_t)s;
    for (int s = 0; s < 144; ++s) ll[k++] = (uint16_t)s;
    for (int s = 280; s < 288; ++s) ll[k++] = (uint16_t)s;
    for (int s = 144; s < 256; ++s) ll[k++] = (uint16_t)s;
    for (int s = 0; s < 30; ++s) dd[s] = (uint8_t)s;
    LL.c[0] = 0; LL.c[1] = 0; LL.c[2] = 0; LL.c[3] = 0; LL.c[4] = 0;
    cnt_add(LL.c, 7, 24); cnt_add(LL.c, 8, 152); cnt_add(LL.c, 9, 112);
    LL.l = 9; LL.g = 9;
    DD.c[0] = 0; DD.c[1] = 0; DD.c[2] = 0; DD.c[3] = 0; DD.c[4] = 0;
    cnt_add(DD.c, 5, 30);
    DD.l = 5; DD.g = 5;
    bll.kmin = 7; bll.g = 9; bll.left = 0; bll.allzero = false; bll.nlong = 0;
    bdd.kmin = 5; bdd.g = 5; bdd.left = 2 << 10; bdd.allzero = false; bdd.nlong = 0;
    finish_dec(LL, bll);
    finish_dec(DD, bdd);
    L.fixed = 1;
}

// infblocks.ts:334-551 + inftree.ts:313-379.  Returns false when the lane stopped
// (error or stall); L.status/zmsg say which.
__device__ __forceinline__ bool setup_dynamic(Lane& L, Dec& LL, Dec& DD, BuildInfo& bll, BuildInfo& bdd, uint8_t* region) {
    uint32_t t;
    if (!br_get(L, 14, t)) { L.status = SDZ_TRUNCATED; return false; }
    if ((t & 0x1f) > 29 || ((t >> 5) & 0x1f) > 29) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_TOO_MANY_SYMS; return false; }
    int nl = 257 + (int)(t & 0x1f), nd = 1 + (int)((t >> 5) & 0x1f);
    int ncl = 4 + (int)(t >> 10);
    // code-length code lengths in border order (infblocks.ts:17-19)
    uint64_t cl = 0;
    for (int i = 0; i < ncl; ++i) {
        uint32_t v;
        if (!br_get(L, 3, v)) { L.status = SDZ_TRUNCATED; return false; }
        cl |= (uint64_t)v << (3 * c_border[i]);
    }
    // bit-length tree (inflate_trees_bits): counts, Kraft, rank array in the dist area
    uint32_t c7[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c7[k] = 0;
    for (int s = 0; s < 19; ++s) {
        int len = (int)((cl >> (3 * s)) & 7);
#pragma unroll
        for (int k = 1; k < 8; ++k) c7[k] += len == k ? 1u : 0u;
    }
    int left = 1, g7 = 0;
#pragma unroll
    for (int k = 1; k < 8; ++k) { left = 2 * left - (int)c7[k]; if (c7[k]) g7 = k; }
    if (left < 0) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_BL_OVERSUB; return false; }
    if (g7 == 0 || (left > 0 && g7 != 1)) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_BL_INCOMPLETE; return false; }
    uint8_t* cls = region + IL_DSYM;
    uint32_t lim7[8];
    int32_t off7[8];
    {
        uint32_t code = 0; int32_t idx = 0; uint32_t nx[8];
#pragma unroll
        for (int k = 1; k < 8; ++k) {
            lim7[k] = (code + c7[k]) << (7 - k);
            off7[k] = idx - (int32_t)code;
            nx[k] = (uint32_t)idx;
            idx += (int32_t)c7[k];
            code = (code + c7[k]) << 1;
        }
        for (int s = 0; s < 19; ++s) {
            int len = (int)((cl >> (3 * s)) & 7);
            if (len) {
                uint32_t k = 0;
#pragma unroll
                for (int q = 1; q < 8; ++q) k = len == q ? nx[q] : k;
                cls[k] = (uint8_t)s;
#pragma unroll
                for (int q = 1; q < 8; ++q) nx[q] += len == q ? 1u : 0u;
            }
        }
    }
    // decode nl + nd code lengths (infblocks.ts:434-523) into global scratch
    int total = nl + nd, idx = 0, prev = 0;
    while (idx < total) {
        br_refill(L);
        if (br_avail(L) < g7) { L.status = SDZ_TRUNCATED; return false; }
        uint32_t rc = __builtin_bitreverse32((uint32_t)L.buf) >> 25;
        int len = 1;
        int32_t off = off7[1];
#pragma unroll
        for (int k = 1; k < 7; ++k) { bool ge = rc >= lim7[k]; len = ge ? k + 1 : len; off = ge ? off7[k + 1] : off; }
        // g7 == 1 with one code: both patterns read the last entry written (inftree.ts:265-267)
        uint32_t c = cls[(g7 == 1 && left > 0) ? 0 : (off + (int32_t)(rc >> (7 - len)))];
        if (g7 == 1 && left > 0) len = 1;
        br_drop(L, len);
        if (c < 16) {
            L.lens[idx++] = (uint8_t)c;
            prev = (int)c;
        } else {
            int eb = c == 18 ? 7 : (int)c - 14;
            int rep = c == 18 ? 11 : 3;
            uint32_t v;
            if (!br_get(L, eb, v)) { L.status = SDZ_TRUNCATED; return false; }
            rep += (int)v;
            if (idx + rep > total || (c == 16 && idx < 1)) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_BL_REPEAT; return false; }
            int val = c == 16 ? prev : 0;
            for (int r = 0; r < rep; ++r) L.lens[idx++] = (uint8_t)val;
            prev = val;
        }
    }
    // literal/length tree (inftree.ts:344-357); the MANY=1400 budget of huft_build
    // (inftree.ts:242) is checked exactly only when a cheap bound cannot rule it out
    bll = count_lens(LL, L.lens, nl, 9);
    if (bll.left < 0) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_LL_OVERSUB; return false; }
    bdd = count_lens(DD, L.lens + nl, nd, 6);
    int ent_ll = 0, ent_d = 0;
    Dec tl = LL, td = DD;
    add_dummies(tl, bll);
    add_dummies(td, bdd);
    bool exact = false;
    if (!bll.allzero) ent_ll = table_bound(tl.c, LL.l, bll.g);
    if (!bdd.allzero && bdd.left >= 0) ent_d = table_bound(td.c, DD.l, bdd.g);
    if (ent_ll + ent_d > 1400) {
        exact = true;
        int dummy;
        if (!bll.allzero)
            ent_ll = huft_replay(tl.c[0], tl.c[1], tl.c[2], tl.c[3], tl.c[4], bll.kmin, bll.g, LL.l, -1, &dummy);
    }
    if (!bll.allzero && ent_ll > 1400) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_LL_OVERSUB; return false; }
    if (bll.allzero || (bll.left > 0 && bll.g != 1)) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_LL_INCOMPLETE; return false; }
    // distance tree (inftree.ts:359-376)
    if (bdd.left < 0) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_D_OVERSUB; return false; }
    if (exact && !bdd.allzero) {
        int dummy;
        ent_d = huft_replay(td.c[0], td.c[1], td.c[2], td.c[3], td.c[4], bdd.kmin, bdd.g, DD.l, -1, &dummy);
    }
    if (!bdd.allzero && ent_ll + ent_d > 1400) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_D_OVERSUB; return false; }
    if (!bdd.allzero && bdd.left > 0 && bdd.g != 1) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_D_INCOMPLETE; return false; }
    if (bdd.allzero && nl > 257) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_D_EMPTY; return false; }
    finish_dec(LL, bll);
    finish_dec(DD, bdd);
    place_syms<uint16_t>(LL, L.lens, nl, (uint16_t*)region);
    place_syms<uint8_t>(DD, L.lens + nl, nd, region + IL_DSYM);
    L.nl = nl; L.nd = nd;
    L.fixed = 0;
    return true;
}

// ------------------------------------------------------------------ kernel

__device__ __forceinline__ void lane_fail(Lane& L, int status, int zmsg) {
    L.status = status;
    L.zmsg = zmsg;
    L.mode = LM_DONE;
}

// one block-level step for a lane that is not decoding symbols
__device__ __forceinline__ void block_step(Lane& L, Dec& LL, Dec& DD, BuildInfo& bll, BuildInfo& bdd, uint8_t* region,
                           const uint32_t* crct) {
    if (L.mode == LM_TYPE) {
        uint32_t t;
        if (!br_get(L, 3, t)) { lane_fail(L, SDZ_TRUNCATED, 0); return; }
        L.last = (int)(t & 1);
        uint32_t bt = t >> 1;
        if (bt == 0) {                                   // stored (infblocks.ts:184-196, 243-333)
            uint64_t cons = br_consumed(L);
            br_drop(L, (int)((8 - (cons & 7)) & 7));
            uint32_t lo, hi;
            if (!br_get(L, 16, lo) || !br_get(L, 16, hi)) { lane_fail(L, SDZ_TRUNCATED, 0); return; }
            if ((~hi & 0xffffu) != lo) { lane_fail(L, SDZ_DATA_ERROR, ZM_STORED_LENS); return; }
            for (uint32_t k = 0; k < lo; ++k) {
                uint32_t b;
                if (!br_get(L, 8, b)) { lane_fail(L, SDZ_TRUNCATED, 0); return; }
                if (L.pos >= L.cap) { lane_fail(L, SDZ_OUT_OVERFLOW, 0); return; }
                put_byte(L, b, crct);
            }
            L.mode = L.last ? LM_TRAILER : LM_TYPE;
        } else if (bt == 1) {
            setup_fixed(L, LL, DD, bll, bdd, region);
            L.mode = LM_CODES;
        } else if (bt == 2) {
            if (!setup_dynamic(L, LL, DD, bll, bdd, region)) { L.mode = LM_DONE; return; }
            L.mode = LM_CODES;
        } else {
            lane_fail(L, SDZ_DATA_ERROR, ZM_BLOCK_TYPE);
        }
        return;
    }
    if (L.mode == LM_TRAILER) {                          // inflate.ts:403-463
        uint64_t cons = br_consumed(L);
        br_drop(L, (int)((8 - (cons & 7)) & 7));          // WASH + blocks.reset()
        if (L.container == SDZ_CONTAINER_ZLIB) {
            uint32_t v = 0;
            for (int k = 0; k < 4; ++k) {
                uint32_t b;
                if (!br_get(L, 8, b)) { lane_fail(L, SDZ_TRUNCATED, 0); return; }
                v = (v << 8) | b;
            }
            L.stored_ck = (int32_t)v;
        } else if (L.container == SDZ_CONTAINER_GZIP) {
            uint32_t v = 0, z = 0;
            for (int k = 0; k < 4; ++k) {
                uint32_t b;
                if (!br_get(L, 8, b)) { lane_fail(L, SDZ_TRUNCATED, 0); return; }
                v = (v >> 8) | (b << 24);
            }
            L.stored_ck = (int32_t)v;
            for (int k = 0; k < 4; ++k) {
                uint32_t b;
                if (!br_get(L, 8, b)) { lane_fail(L, SDZ_TRUNCATED, 0); return; }
                z = (z >> 8) | (b << 24);
            }
            L.stored_size = (int32_t)z;
        }
        L.mode = LM_DONE;
        L.status = br_avail(L) > 0 ? SDZ_TRAILING : SDZ_OK;
        return;
    }
}

// decode one literal/length symbol (+ its match) -- the hot loop body
__device__ __forceinline__ void decode_step(Lane& L, const Dec& LL, const Dec& DD, const BuildInfo& bll,
                                            const BuildInfo& bdd, const uint8_t* region,
                                            const uint32_t* crct) {
    br_refill(L);
    bool careful = br_avail(L) < 64;
    uint32_t rc = __builtin_bitreverse32((uint32_t)L.buf) >> 17;
    int len;
    int32_t idx = hdecode(rc, LL, len);
    if (careful && br_avail(L) < DEC_NEED(LL, bll, len, idx)) { lane_fail(L, SDZ_TRUNCATED, 0); return; }
    if (rc >= LL.lim[15]) { lane_fail(L, SDZ_DATA_ERROR, ZM_INVALID_LITLEN); return; }
    uint32_t sym = ((const uint16_t*)region)[idx];
    br_drop(L, len);
    if (sym < 256) {
        if (L.pos >= L.cap) { lane_fail(L, SDZ_OUT_OVERFLOW, 0); return; }
        put_byte(L, sym, crct);
        return;
    }
    if (sym == 256) { L.mode = L.last ? LM_TRAILER : LM_TYPE; return; }
    if (sym > 285) { lane_fail(L, SDZ_DATA_ERROR, ZM_INVALID_LITLEN); return; }
    uint32_t li = sym - 257;
    int e;
    uint32_t base;
    if (li < 8) { e = 0; base = li + 3; }
    else if (li == 28) { e = 0; base = 258; }
    else { e = (int)((li - 4) >> 2); base = ((4u + (li & 3u)) << e) + 3u; }
    if (careful && br_avail(L) < e) { lane_fail(L, SDZ_TRUNCATED, 0); return; }
    uint32_t mlen = base + br_peek(L, e);
    br_drop(L, e);
    br_refill(L);
    rc = __builtin_bitreverse32((uint32_t)L.buf) >> 17;
    idx = hdecode(rc, DD, len);
    if (careful && br_avail(L) < DEC_NEED(DD, bdd, len, idx)) { lane_fail(L, SDZ_TRUNCATED, 0); return; }
    if (rc >= DD.lim[15]) { lane_fail(L, SDZ_DATA_ERROR, ZM_INVALID_DIST); return; }
    uint32_t ds = region[IL_DSYM + idx];
    br_drop(L, len);
    uint32_t dbase;
    if (ds < 4) { e = 0; dbase = ds + 1; }
    else { e = (int)((ds - 2) >> 1); dbase = ((2u + (ds & 1u)) << e) + 1u; }
    if (careful && br_avail(L) < e) { lane_fail(L, SDZ_TRUNCATED, 0); return; }
    uint32_t dist = dbase + br_peek(L, e);
    br_drop(L, e);
    if (L.pos + mlen > L.cap) { lane_fail(L, SDZ_OUT_OVERFLOW, 0); return; }
    copy_match(L, mlen, dist, crct);
}

// adler32.ts:34-105 over the final chunk of r bytes, seeded with the chunk-start
// state; reproduces the unreduced sum2 when r is a multiple of NMAX
__device__ int32_t adler_quirk_tail(const uint8_t* p, uint32_t r, uint32_t s1, uint32_t s2in) {
    uint64_t a = s1, s2 = s2in;
    uint32_t off = 0, len = r;
    while (len >= 5552) {
        len -= 5552;
        for (int i = 0; i < 5552; ++i) { a += p[off++]; s2 += a; }
        a %= 65521u;
        s2 += 65521u;
    }
    if (len) {
        while (len--) { a += p[off++]; s2 += a; }
        a %= 65521u;
        s2 %= 65521u;
    }
    return (int32_t)((uint32_t)a | ((uint32_t)s2 << 16));
}

__global__ __launch_bounds__(IL_THREADS, 1) void k_inflate(InflateArgs A) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[IL_LDS];
    uint32_t* crct = (uint32_t*)(lds + IL_CRC_OFF);
    // slicing-by-4 CRC tables (crc32.ts:179-214)
    for (int n = threadIdx.x; n < 256; n += IL_THREADS) {
        uint32_t c = (uint32_t)n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
        crct[n] = c;
    }
    __syncthreads();
    for (int n = threadIdx.x; n < 256; n += IL_THREADS) {
        uint32_t c = crct[n];
        for (int k = 1; k < 4; ++k) { c = crct[c & 255] ^ (c >> 8); crct[256 * k + n] = c; }
    }
    __syncthreads();

    uint8_t* region = lds + threadIdx.x * IL_REGION;
    uint32_t gid = blockIdx.x * IL_THREADS + threadIdx.x;
    bool valid = gid < A.n;
    uint32_t sid = valid ? (A.order ? A.order[gid] : gid) : 0u;

    Lane L;
    Dec LL, DD;
    BuildInfo bll, bdd;
    L.mode = LM_DONE; L.status = SDZ_OK; L.zmsg = 0; L.container = SDZ_CONTAINER_RAW;
    L.pos = 0; L.acc = 0; L.last = 0; L.fixed = 0; L.nl = L.nd = 0;
    L.stored_ck = 0; L.stored_size = 0; L.mtime = 0; L.name_off = 0; L.name_len = 0;
    L.s1 = 1; L.s2 = 0; L.crc = 0xffffffffu; L.snap1 = 1; L.snap2 = 0; L.ck = CK_NONE;
    L.cnt = 0; L.buf = 0; L.loaded = 0; L.total = 0; L.ncur = 1;
    L.dict = A.dict; L.dict_len = A.dict ? A.dict_len : 0;
    LL.l = DD.l = 0; LL.g = DD.g = 0;
    bll.kmin = bdd.kmin = 1; bll.g = bdd.g = 0; bll.left = bdd.left = 0; bll.allzero = bdd.allzero = true;
    bll.nlong = bdd.nlong = 0;
    bool dict_used = false;

    if (valid) {
        uint64_t ioff = A.in_off[sid], ilen = A.in_len[sid];
        uint64_t ooff = A.out_off[sid];
        L.cap = A.out_cap[sid];
        L.ob = (uint64_t*)(A.out + ooff);
        L.lens = A.scratch + (uint64_t)gid * kInflateScratchPerStream;
        uintptr_t addr = (uintptr_t)(A.in + ioff);
        int skip = (int)(addr & 15);
        L.vp = (const uint4*)(addr & ~(uintptr_t)15);
        L.cur = *L.vp++;
        L.nxt = *L.vp++;
        L.ncur = 4;
        for (int k = 0; k < (skip >> 2); ++k) { L.cur.x = L.cur.y; L.cur.y = L.cur.z; L.cur.z = L.cur.w; L.ncur--; }
        br_refill(L);
        L.buf >>= 8 * (skip & 3);
        L.cnt -= 8 * (skip & 3);
        L.loaded = (uint64_t)L.cnt;
        L.total = ilen * 8;
        L.mode = LM_TYPE;
        if (ooff & 7) lane_fail(L, SDZ_BAD_RECORD, 0);

        // ---- container (inflate.ts:142-401; sd-inflate.ts:194-207 for AUTO)
        bool raw = A.format == SDZ_FMT_RAW;
        if (L.mode != LM_DONE && A.format == SDZ_FMT_AUTO) {
            if (ilen < 2) lane_fail(L, SDZ_TOO_SMALL, 0);
            else {
                br_refill(L);
                uint32_t b0 = br_peek(L, 8), b1 = (uint32_t)(L.buf >> 8) & 255u;
                bool ident = (b0 == 0x78 && ((b0 << 8) + b1) % 31 == 0) || (b0 == 0x1f && b1 == 0x8b);
                raw = !ident;
            }
        }
        if (L.mode != LM_DONE && !raw) {
            uint32_t b = 0, method = 0, flg = 0;
            bool ok = br_get(L, 8, b);
            bool gz = false;
            if (ok && b == 0x1f) {
                ok = br_get(L, 8, b);
                if (ok && b != 0x8b) { lane_fail(L, SDZ_DATA_ERROR, ZM_INVALID_GZIP_ID); }
                gz = true;
                if (ok && L.mode != LM_DONE) ok = br_get(L, 8, method);
            } else {
                method = b;
            }
            if (L.mode != LM_DONE) {
                if (!ok) lane_fail(L, SDZ_TRUNCATED, 0);
                else if ((method & 0xf) != 8) lane_fail(L, SDZ_DATA_ERROR, ZM_UNKNOWN_METHOD);
                else if ((method >> 4) + 8 > 15) lane_fail(L, SDZ_DATA_ERROR, ZM_INVALID_WINDOW);
                else if (!br_get(L, 8, flg)) lane_fail(L, SDZ_TRUNCATED, 0);
            }
            if (L.mode != LM_DONE && gz) {
                L.container = SDZ_CONTAINER_GZIP;
                uint32_t mt = 0, v;
                for (int k = 0; k < 4 && L.mode != LM_DONE; ++k) {
                    if (!br_get(L, 8, v)) lane_fail(L, SDZ_TRUNCATED, 0);
                    else mt = (mt >> 8) | (v << 24);
                }
                L.mtime = (int32_t)mt;
                for (int k = 0; k < 2 && L.mode != LM_DONE; ++k)
                    if (!br_get(L, 8, v)) lane_fail(L, SDZ_TRUNCATED, 0);
                if (L.mode != LM_DONE && (flg & 4)) {
                    // inflate.ts:333-346: EXTRA0 never advances; all input is swallowed
                    lane_fail(L, SDZ_TRUNCATED, 0);
                }
                if (L.mode != LM_DONE && (flg & 8)) {
                    L.name_off = (uint32_t)(br_consumed(L) >> 3);
                    while (L.mode != LM_DONE) {
                        if (!br_get(L, 8, v)) { lane_fail(L, SDZ_TRUNCATED, 0); break; }
                        if (v == 0) break;
                        L.name_len++;
                    }
                }
                if (L.mode != LM_DONE && (flg & 16)) {
                    while (L.mode != LM_DONE) {
                        if (!br_get(L, 8, v)) { lane_fail(L, SDZ_TRUNCATED, 0); break; }
                        if (v == 0) break;
                    }
                }
                if (L.mode != LM_DONE && (flg & 2)) {
                    for (int k = 0; k < 2 && L.mode != LM_DONE; ++k)
                        if (!br_get(L, 8, v)) lane_fail(L, SDZ_TRUNCATED, 0);
                }
            } else if (L.mode != LM_DONE) {
                L.container = SDZ_CONTAINER_ZLIB;
                if (((method << 8) + flg) % 31 != 0) lane_fail(L, SDZ_DATA_ERROR, ZM_HEADER_CHECK);
                else if (flg & 0x20) {
                    uint32_t id = 0, v;
                    for (int k = 0; k < 4 && L.mode != LM_DONE; ++k) {
                        if (!br_get(L, 8, v)) lane_fail(L, SDZ_TRUNCATED, 0);
                        else id = (id << 8) | v;
                    }
                    if (L.mode != LM_DONE) {
                        if (!A.dict) lane_fail(L, SDZ_NEED_DICT, ZM_NEED_DICT);
                        else if ((int32_t)id != A.dict_adler) lane_fail(L, SDZ_DICT_MISMATCH, 0);
                        else dict_used = true;
                    }
                }
            }
        }
        if (!dict_used) L.dict_len = 0;
        if (L.dict_len > 32767) { L.dict += L.dict_len - 32767; L.dict_len = 32767; }   // inflate.ts:488-491
        L.ck = L.container == SDZ_CONTAINER_GZIP ? CK_CRC : CK_ADLER;
    }

    // ---- phase loop: lanes at a block boundary advance together, then decode together
    for (;;) {
        while (L.mode != LM_CODES && L.mode != LM_DONE) block_step(L, LL, DD, bll, bdd, region, crct);
        int ncodes = __popcll(__ballot(L.mode == LM_CODES));
        if (ncodes == 0) break;
        int k = ncodes >> 3;
        int stop = ncodes - (k > 0 ? k : 1);
        do {
            if (L.mode == LM_CODES) decode_step(L, LL, DD, bll, bdd, region, crct);
        } while (__popcll(__ballot(L.mode == LM_CODES)) > stop);
    }

    if (!valid) return;
    // ---- final partial word + checksums + verdicts (sd-inflate.ts:134-179)
    uint32_t rem = (uint32_t)(L.pos & 7);
    if (rem && L.status != SDZ_BAD_RECORD) {
        L.ob[L.pos >> 3] = L.acc;
        for (uint32_t k = 0; k < rem; ++k) ck_byte(L, (uint32_t)(L.acc >> (8 * k)) & 255u, crct);
    }
    sdz_inflate_record R;
    R.status = L.status;
    R.zmsg = L.zmsg;
    R.out_len = L.pos;
    uint64_t cons = br_consumed(L);
    R.in_used = (cons + 7) >> 3;
    if (R.in_used > (L.total >> 3)) R.in_used = L.total >> 3;
    R.stored_checksum = L.stored_ck;
    int32_t running;
    bool have = L.pos > 0;                               // Inflater.checksum stays undefined otherwise
    if (L.ck == CK_CRC) {
        running = (int32_t)~L.crc;
    } else {
        uint32_t r = (uint32_t)(L.pos & 16383u);
        if (r == 5552u || r == 11104u) {
            running = adler_quirk_tail((const uint8_t*)L.ob + (L.pos - r), r, L.snap1, L.snap2);
        } else {
            running = (int32_t)(L.s1 | (L.s2 << 16));
        }
    }
    R.running_checksum = have ? running : 0;
    R.stored_size = L.stored_size;
    R.mtime = L.mtime;
    R.name_off = L.name_off;
    R.name_len = L.name_len;
    R.container = (uint8_t)L.container;
    bool complete = L.mode == LM_DONE && (L.status == SDZ_OK || L.status == SDZ_TRAILING);
    R.complete = complete ? 1 : 0;
    uint8_t cv = L.stored_ck == 0 ? SDZ_UNCHECKED : ((have && L.stored_ck == running) ? SDZ_MATCH : SDZ_MISMATCH);
    uint8_t sv = L.stored_size == 0 ? SDZ_UNCHECKED
               : ((int64_t)L.stored_size == (int64_t)L.pos ? SDZ_MATCH : SDZ_MISMATCH);
    R.checksum_verdict = cv;
    R.size_verdict = sv;
    R.success = (complete && cv != SDZ_MISMATCH && sv != SDZ_MISMATCH) ? 1 : 0;
    for (int k = 0; k < 11; ++k) R.reserved[k] = 0;
    A.rec[sid] = R;
}

void launch_inflate(const InflateArgs& a, hipStream_t s) {
    if (a.n == 0) return;
    dim3 grid((a.n + IL_THREADS - 1) / IL_THREADS);
    hipLaunchKernelGGL(k_inflate, grid, dim3(IL_THREADS), 0, s, a);
}

}  // namespace sdz
