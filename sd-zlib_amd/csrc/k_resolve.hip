// k_resolve.hip -- batched DEFLATE decoder, phase 2: tokens -> bytes, adler32, and the
// Inflater verdicts (src/sd-inflate.ts:134-179); k_inflate_finalize adds crc32 for gzip.
//
// One WORKGROUP (4 waves) per stream, four streams per CU.  The stream's LZ77 window
// lives in LDS: a 36 KiB ring holds the last 32 KiB of output plus the batch being
// built, so back-references never leave the CU (a global-memory window re-reads the
// source lines of every match from beyond L2: median distance is ~7 KiB on text).
// Per batch of up to 256 tokens (<= 4 KiB of output):
//   1. block-wide prefix sum of token lengths (DPP within waves, LDS across them);
//   2. literals, and matches whose source lies before the batch, are written in
//      parallel (4-byte unaligned LDS copies; distances 1-3 as repeating words);
//   3. matches reading bytes of this batch resolve in barrier-separated rounds:
//      a match goes once every token it reads from is final (256-bit LDS mask);
//      the earliest pending match is always ready, so rounds terminate;
//   4. the batch is written to HBM as coalesced dwords and folded into adler32
//      (S = sum b, W = sum (B - t) b, wave then block reduction), with the 16 KiB
//      snapshot the Inflater's chunk-wise checksum needs (adler32.ts:67 quirk).
// Positions before the output start read the preset dictionary or zeros.
#include "inflate_state.h"

namespace sdz {

#define RS_THREADS 256
#define RS_WAVES (RS_THREADS / 64)
#define RS_R 35840                    // ring bytes: 32 KiB window + one batch
#define RS_STAGE 3072                 // batch output budget
#define RS_WIN 32768

__device__ __forceinline__ uint32_t ridx(int32_t x) {            // x in (-R, 2R)
    x += x < 0 ? RS_R : 0;
    x -= x >= RS_R ? RS_R : 0;
    return (uint32_t)x;
}

// inclusive wave scan / reduction with DPP row shifts and row broadcasts (gfx9)
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_add(uint32_t x) {
    return x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x = dpp_add<0x111, 0xf>(x);                           // row_shr:1
    x = dpp_add<0x112, 0xf>(x);                           // row_shr:2
    x = dpp_add<0x114, 0xf>(x);                           // row_shr:4
    x = dpp_add<0x118, 0xf>(x);                           // row_shr:8
    x = dpp_add<0x142, 0xa>(x);                           // row_bcast:15 -> rows 1, 3
    x = dpp_add<0x143, 0xc>(x);                           // row_bcast:31 -> rows 2, 3
    return x;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(x), 63);
}

__device__ __forceinline__ uint32_t ld32(const uint8_t* ring, uint32_t i) {   // unaligned ds_read_b32
    uint32_t v;
    __builtin_memcpy(&v, ring + i, 4);
    return v;
}
__device__ __forceinline__ void st32(uint8_t* ring, uint32_t i, uint32_t v) { __builtin_memcpy(ring + i, &v, 4); }
__device__ __forceinline__ void st16(uint8_t* ring, uint32_t i, uint32_t v) {
    uint16_t h = (uint16_t)v;
    __builtin_memcpy(ring + i, &h, 2);
}

// write the low n <= 4 bytes of v at ring index d (no wrap: d + n <= R)
__device__ __forceinline__ void put_tail(uint8_t* ring, uint32_t d, uint32_t v, uint32_t n) {
    if (n == 4) { st32(ring, d, v); return; }
    if (n & 2) { st16(ring, d, v); d += 2; v >>= 16; }
    if (n & 1) ring[d] = (uint8_t)v;
}
// the same across the ring's end
__device__ __forceinline__ void put_wrap(uint8_t* ring, uint32_t d, uint32_t v, uint32_t n) {
    for (uint32_t b = 0; b < n; ++b) ring[ridx((int32_t)(d + b))] = (uint8_t)(v >> (8 * b));
}

// LZ77 copy of len bytes from ring index s to ring index d (s = d - dist mod R)
__device__ __forceinline__ void copy_match(uint8_t* ring, uint32_t d, uint32_t s, uint32_t len, uint32_t dist) {
    const bool nowrap = d + len <= RS_R && s + len + 3 <= RS_R;
    if (dist >= 4) {
        // 4-byte units in order: a unit reads bytes at least 4 behind its own
        if (nowrap) {
            uint32_t k = 0;
            for (; k + 4 <= len; k += 4) st32(ring, d + k, ld32(ring, s + k));
            if (k < len) put_tail(ring, d + k, ld32(ring, s + k), len - k);
            return;
        }
        for (uint32_t k = 0; k < len; k += 4) {
            uint32_t v = 0;
            for (uint32_t b = 0; b < 4; ++b) v |= (uint32_t)ring[ridx((int32_t)(s + k + b))] << (8 * b);
            put_wrap(ring, d + k, v, len - k < 4 ? len - k : 4);
        }
        return;
    }
    // period 1..3: the source bytes repeat; emit them as 4-byte words
    uint32_t p0 = ring[s], p1 = ring[ridx((int32_t)s + 1)], p2 = ring[ridx((int32_t)s + 2)];
    uint32_t w0, w1, w2;
    if (dist == 1) { w0 = w1 = w2 = p0 * 0x01010101u; }
    else if (dist == 2) { w0 = w1 = w2 = (p0 | (p1 << 8)) * 0x00010001u; }
    else {
        w0 = p0 | (p1 << 8) | (p2 << 16) | (p0 << 24);
        w1 = p1 | (p2 << 8) | (p0 << 16) | (p1 << 24);
        w2 = p2 | (p0 << 8) | (p1 << 16) | (p2 << 24);
    }
    if (d + len <= RS_R) {
        uint32_t k = 0;
        for (; k + 4 <= len; k += 4) {
            st32(ring, d + k, w0);
            uint32_t t = w0; w0 = w1; w1 = w2; w2 = t;       // the next unit starts 4 bytes on
        }
        if (k < len) put_tail(ring, d + k, w0, len - k);
        return;
    }
    for (uint32_t k = 0; k < len; k += 4) {
        put_wrap(ring, d + k, w0, len - k < 4 ? len - k : 4);
        uint32_t t = w0; w0 = w1; w1 = w2; w2 = t;
    }
}

// are tokens j0..j1 all final?  (mask of 256 bits; empty range -> true)
__device__ __forceinline__ bool range_final(const uint64_t* fin, int j0, int j1) {
    for (int q = j0 >> 6; q <= (j1 >> 6); ++q) {
        int lo = j0 > 64 * q ? j0 : 64 * q, hi = j1 < 64 * q + 63 ? j1 : 64 * q + 63;
        uint64_t m = (~0ull >> (63 - (hi - lo))) << (lo - 64 * q);
        if ((fin[q] & m) != m) return false;
    }
    return true;
}

// index of the token whose output covers batch byte x (ei = inclusive ends, ascending)
__device__ __forceinline__ int tok_of(const uint32_t* ei, int ntk, uint32_t x) {
    int lo = 0, hi = ntk - 1;                             // first j with ei[j] > x
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (ei[mid] > x) hi = mid; else lo = mid + 1;
    }
    return lo;
}

// adler32.ts:34-105 over r bytes seeded with the chunk-start state (NMAX quirk)
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

// Emit tokens' bytes into the ring -- called by a whole wave; lanes with act set
// write their token.  Loops run to the wave's longest job; writes past a token's
// end go to the lane's dummy slot, so output is exact without divergent branches.
// UNROLL: four 4-byte units per step, all reads before the writes (only for copies
// whose source cannot overlap what the step writes: no in-batch self-overlap).
// Tokens whose destination or source crosses the ring's end go byte-serial.
// redirected writes go to a per-thread slot past the ring (distinct banks: a shared
// dummy address would serialize every inactive lane's store)
#define RS_DUMMY (RS_R + 4u * threadIdx.x)
template <bool UNROLL>
__device__ __forceinline__ void emit_tokens(uint8_t* ring, bool act, uint32_t t, uint32_t d, uint32_t s,
                                            uint32_t len, uint32_t dist) {
    const bool lit = (t >> 31) == 0;
    const bool slow = act && (d + len > RS_R || (!lit && s + len + 3 > RS_R));
    const bool fast = act && !slow;
    const bool per = fast && !lit && dist < 4;
    const bool cp = fast && !lit && dist >= 4;
    const uint32_t nfull = fast && !lit ? len >> 2 : 0u;
    const uint32_t ncp = cp ? nfull : 0u;
    if (UNROLL) {
        for (uint32_t u = 0; __ballot(u < ncp); u += 4) {
            uint32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = ld32(ring, u + k < ncp ? s + 4 * (u + k) : 0u);
#pragma unroll
            for (int k = 0; k < 4; ++k) st32(ring, u + k < ncp ? d + 4 * (u + k) : RS_DUMMY, v[k]);
        }
    } else {
        for (uint32_t u = 0; __ballot(u < ncp); ++u)
            st32(ring, u < ncp ? d + 4 * u : RS_DUMMY, ld32(ring, u < ncp ? s + 4 * u : 0u));
    }
    uint32_t w0 = 0, w1 = 0, w2 = 0;
    if (__ballot(per)) {                                  // period 1..3: repeating words
        const uint32_t p0 = ring[s], p1 = ring[ridx((int32_t)s + 1)], p2 = ring[ridx((int32_t)s + 2)];
        const uint32_t a1 = p0 * 0x01010101u, a2 = (p0 | (p1 << 8)) * 0x00010001u;
        w0 = dist == 1 ? a1 : dist == 2 ? a2 : p0 | (p1 << 8) | (p2 << 16) | (p0 << 24);
        w1 = dist == 1 ? a1 : dist == 2 ? a2 : p1 | (p2 << 8) | (p0 << 16) | (p1 << 24);
        w2 = dist == 1 ? a1 : dist == 2 ? a2 : p2 | (p0 << 8) | (p1 << 16) | (p2 << 24);
        const uint32_t np = per ? nfull : 0u;
        for (uint32_t u = 0; __ballot(u < np); ++u) {     // unit u repeats word u mod 3
            const uint32_t r = u % 3u;
            st32(ring, u < np ? d + 4 * u : RS_DUMMY, r == 0 ? w0 : r == 1 ? w1 : w2);
        }
    }
    const uint32_t tail = fast ? (lit ? len : len & 3u) : 0u;
    if (__ballot(tail != 0)) {
        const uint32_t k = 4 * nfull;
        const uint32_t r = nfull % 3u;
        uint32_t v = ld32(ring, tail && cp ? s + k : 0u);
        v = lit ? t : per ? (r == 0 ? w0 : r == 1 ? w1 : w2) : v;
        st16(ring, tail >= 2 ? d + k : RS_DUMMY, v);
        ring[tail == 1 ? d + k : tail == 3 ? d + k + 2 : RS_DUMMY] = (uint8_t)(tail == 3 ? v >> 16 : v);
    }
    if (__ballot(slow)) {                                 // across the ring's end: byte-serial
        for (uint32_t k = 0; __ballot(slow && k < len); ++k) {
            const bool a = slow && k < len;
            const uint32_t b = lit ? (t >> (8 * (k & 3u))) & 255u : ring[a && !lit ? ridx((int32_t)(s + k)) : 0u];
            ring[a ? ridx((int32_t)(d + k)) : RS_DUMMY] = (uint8_t)b;
        }
    }
}

// does the unresolved-byte bitmap have any bit in [lo, hi)?  (wave-uniform loop)
__device__ __forceinline__ bool any_unres(const uint32_t* unres, bool act, uint32_t lo, uint32_t hi) {
    bool hit = false;
    const uint32_t w0 = lo >> 5, w1 = act && hi > lo ? (hi - 1) >> 5 : 0u;
    const uint32_t nw = act && hi > lo ? w1 - w0 + 1 : 0u;
    for (uint32_t i = 0; __ballot(i < nw); ++i) {
        const uint32_t wd = w0 + i;
        const uint32_t m = i < nw ? (~0u << (wd == w0 ? lo & 31u : 0u)) &
                                    (wd == w1 && (hi & 31u) ? (1u << (hi & 31u)) - 1u : ~0u) : 0u;
        hit = hit || (unres[i < nw ? wd : 0u] & m) != 0;
    }
    return hit;
}
// set the bits [lo, hi) (wave-uniform loop)
__device__ __forceinline__ void mark_unres(uint32_t* unres, uint32_t* dummy, bool act, uint32_t lo, uint32_t hi) {
    const uint32_t w0 = lo >> 5, w1 = act && hi > lo ? (hi - 1) >> 5 : 0u;
    const uint32_t nw = act && hi > lo ? w1 - w0 + 1 : 0u;
    for (uint32_t i = 0; __ballot(i < nw); ++i) {
        const uint32_t wd = w0 + i;
        const uint32_t m = i < nw ? (~0u << (wd == w0 ? lo & 31u : 0u)) &
                                    (wd == w1 && (hi & 31u) ? (1u << (hi & 31u)) - 1u : ~0u) : 0u;
        atomicOr(i < nw ? &unres[wd] : dummy, m);
    }
}

__device__ __forceinline__ uint32_t mod65521(uint64_t x) { return (uint32_t)(x % 65521u); }

__global__ __launch_bounds__(RS_THREADS) void k_inflate_resolve(InflateArgs A, uint32_t round) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[RS_R + 4 * RS_THREADS];   // + per-thread dummies
    __shared__ uint16_t ei[RS_THREADS];                  // inclusive output ends of the batch's tokens
    __shared__ uint32_t unres[RS_STAGE / 32];            // bytes of matches that read this batch
    __shared__ uint64_t remm[RS_WAVES];                  // matches left for the ordered pass
    __shared__ uint32_t jds[RS_THREADS], jl[RS_THREADS]; // their jobs: d | s << 16, len | dist << 16
    __shared__ uint32_t wtot[RS_WAVES];
    __shared__ uint64_t red[RS_WAVES][2];
    __shared__ uint32_t ntk_s;

    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    const uint32_t sid = blockIdx.x;
    if (sid >= A.n) return;
    const uint32_t flag = A.flags[sid];
    if (flag == 2) return;
    RSave* R = (RSave*)A.rsave + sid;
    const DSave* S = (const DSave*)A.dsave + sid;
    const bool gz = S->container == SDZ_CONTAINER_GZIP;
    const uint64_t pos0 = round == 0 ? 0 : R->pos;
    uint64_t pos = pos0;
    uint8_t* out = A.out + A.out_off[sid];
    const uint32_t* tk = A.tokens + (uint64_t)sid * A.round_tokens;
    const uint32_t ntok = A.ntok[sid];
    const int64_t dl = S->dict_used && A.dict ? (A.dict_len > 32767 ? 32767 : A.dict_len) : 0;
    const uint8_t* dict = dl ? A.dict + (A.dict_len - dl) : nullptr;
    uint32_t* dummy = (uint32_t*)(ring + RS_DUMMY);

    // the window: output bytes [pos - 32 KiB, pos), the dictionary / zeros before 0
    uint32_t rp = (uint32_t)(pos % RS_R);
    for (uint32_t k = tid; k < RS_WIN; k += RS_THREADS) {
        int64_t p = (int64_t)pos - RS_WIN + k;
        uint32_t b = 0;
        if (p >= 0) b = round ? out[p] : 0u;
        else if (p >= -dl) b = dict[dl + p];
        ring[ridx((int32_t)((int64_t)rp - RS_WIN + k))] = (uint8_t)b;
    }

    // adler32 as sums over the whole output: s1 = 1 + S, s2 = n + n S - T (mod 65521),
    // S = sum b_i, T = sum i b_i -- per-lane partials, combined once per round
    uint64_t accS = 0, accT = 0;
    uint32_t tnext = tid < ntok ? tk[tid] : 0u;
    const bool timed = A.dbg && tid == 0 && sid < 8;
    unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tlast = timed ? clock64() : 0;
#define RS_TICK(k) do { if (timed) { unsigned long long tn = clock64(); tacc[k] += tn - tlast; tlast = tn; } } while (0)
    for (uint32_t base = 0; base < ntok;) {
        // 1. lengths, block prefix sum
        const bool inr = base + tid < ntok;
        const uint32_t t = tnext;
        const bool ism = (t >> 31) != 0;
        const uint32_t len = !inr ? 0u : ism ? ((t >> 16) & 255u) + 3u : ((t >> 24) & 3u) + 1u;
        const uint32_t dist = (t & 0x7fffu) + 1u;
        uint32_t incl = wave_incl_scan(len);
        if (lane == 63) wtot[w] = incl;
        if (tid == 0) ntk_s = RS_THREADS;
        if (tid < RS_STAGE / 32) unres[tid] = 0;
        __syncthreads();
        RS_TICK(1);
        for (uint32_t q = 0; q < w; ++q) incl += wtot[q];
        const uint32_t off = incl - len;
        const bool take = inr && incl <= RS_STAGE;       // a prefix: token 0 always fits (len <= 258)
        ei[tid] = (uint16_t)(incl < RS_STAGE + 258 ? incl : RS_STAGE + 258);
        const uint64_t nt = ~__ballot(take);
        if (nt && lane == (uint32_t)__builtin_ctzll(nt)) atomicMin(&ntk_s, 64u * w + lane);

        // 2. literals and matches with their source before the batch; matches reading
        //    this batch mark their bytes unresolved
        const bool gen0 = take && (!ism || dist >= off + len);
        const bool pend = take && ism && !gen0;
        const uint32_t d = ridx((int32_t)(rp + off));
        const uint32_t s = ridx((int32_t)rp + (int32_t)off - (int32_t)dist);
        emit_tokens<true>(ring, gen0, t, d, s, len, dist);
        mark_unres(unres, dummy, pend, off, off + len);
        RS_TICK(2);
        __syncthreads();
        RS_TICK(3);
        const uint32_t ntk = ntk_s;
        const uint32_t B = ei[ntk - 1];
        tnext = base + ntk + tid < ntok ? tk[base + ntk + tid] : 0u;

        // 3. matches reading only final bytes go in parallel; the rest, in token order
        const int32_t sb = (int32_t)off - (int32_t)dist;
        const uint32_t lo = sb > 0 ? (uint32_t)sb : 0u;
        const uint32_t hi = (uint32_t)(sb + (int32_t)len < (int32_t)off ? sb + (int32_t)len : (int32_t)off);
        bool ready = false;
        uint64_t pm = __ballot(pend);
        if (pm) {
            ready = pend && !any_unres(unres, pend, lo, hi);
            emit_tokens<false>(ring, ready, t, d, s, len, dist);
        }
        const uint64_t rm = __ballot(pend && !ready);
        if (lane == 0) remm[w] = rm;
        if (pend && !ready) { jds[tid] = d | (s << 16); jl[tid] = len | (dist << 16); }
        __syncthreads();
        RS_TICK(4);
        const uint64_t r0 = remm[0], r1 = remm[1], r2 = remm[2], r3 = remm[3];
        if (r0 | r1 | r2 | r3) {
            if (w == 0) {                                 // ordered pass: one match at a time,
                for (int q = 0; q < RS_WAVES; ++q) {      // 64 bytes per step across the wave
                    uint64_t m = q == 0 ? r0 : q == 1 ? r1 : q == 2 ? r2 : r3;
                    while (m) {
                        const uint32_t i = 64u * q + (uint32_t)__builtin_ctzll(m);
                        m &= m - 1;
                        const uint32_t jdd = jds[i] & 0xffffu, jss = jds[i] >> 16, jll = jl[i];
                        const uint32_t L = jll & 0xffffu, D = jll >> 16;
                        for (uint32_t k = lane; k < L; k += 64) {
                            uint32_t km = k;
                            if (D < L && k >= D) {        // overlapping: byte k repeats byte k mod D
                                int32_t r = (int32_t)k - (int32_t)((float)k * __builtin_amdgcn_rcpf((float)D)) * (int32_t)D;
                                r += r < 0 ? (int32_t)D : 0;
                                r -= r >= (int32_t)D ? (int32_t)D : 0;
                                km = (uint32_t)r;
                            }
                            ring[ridx((int32_t)(jdd + k))] = ring[ridx((int32_t)(jss + km))];
                        }
                    }
                }
            }
            __syncthreads();
        }
        RS_TICK(5);

        // 4. write back as dwords from the dword-aligned start; adler partials
        const uint32_t head = rp & 3u;
        const uint32_t nd = (head + B + 3u) >> 2;
        const uint32_t rd0 = (rp - head) >> 2;
        uint32_t* dstw = (uint32_t*)(out + (pos - head));
        const uint32_t* ring32 = (const uint32_t*)ring;
        const uint32_t posm = (uint32_t)(pos % 65521u);
        for (uint32_t q = tid; q < nd; q += RS_THREADS) {
            uint32_t ri = rd0 + q;
            ri -= ri >= RS_R / 4 ? RS_R / 4 : 0;
            const uint32_t v = ring32[ri];
            if (q + 1 < nd || ((head + B) & 3u) == 0) dstw[q] = v;
            else for (uint32_t bb = 0; bb < ((head + B) & 3u); ++bb) ((uint8_t*)(dstw + q))[bb] = (uint8_t)(v >> (8 * bb));
            if (!gz) {
                const uint32_t blo = q == 0 ? head : 0u;
                const uint32_t bhi = q + 1 < nd ? 4u : (((head + B) & 3u) ? ((head + B) & 3u) : 4u);
                const uint32_t m = (bhi == 4u ? ~0u : (1u << (8 * bhi)) - 1u) & (~0u << (8 * blo));
                const uint32_t vm = v & m;
                // global index of byte 0 of this dword, mod 65521
                uint32_t gi = posm + 65521u + 4 * q - head;
                gi -= gi >= 65521u ? 65521u : 0u;
                gi -= gi >= 65521u ? 65521u : 0u;
                const uint32_t s4 = __builtin_amdgcn_udot4(vm, 0x01010101u, 0u, false);
                accS += s4;
                accT += (uint64_t)gi * s4 + __builtin_amdgcn_udot4(vm, 0x03020100u, 0u, false);
            }
        }
        RS_TICK(6);
        pos += B;
        rp = ridx((int32_t)(rp + B));
        base += ntk;
    }
    if (timed) for (int k = 0; k < 8; ++k) atomicAdd(&A.dbg[k], tacc[k]);
    // combine the adler partials of this round
    uint32_t S_all = 0, T_all = 0;
    if (!gz) {
        uint64_t a = accS, b = accT;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) { a += __shfl_xor(a, o); b += __shfl_xor(b, o); }
        if (lane == 0) { red[w][0] = a; red[w][1] = b; }
        __syncthreads();
        uint64_t tS = round ? R->s1 : 0, tT = round ? R->s2 : 0;
#pragma unroll
        for (int q = 0; q < RS_WAVES; ++q) { tS += mod65521(red[q][0]); tT += mod65521(red[q][1]); }
        S_all = mod65521(tS);
        T_all = mod65521(tT);
    }
    __syncthreads();                                     // R->s1 / s2 were read above
    if (tid == 0) { R->pos = pos; R->s1 = S_all; R->s2 = T_all; }
    if (flag != 1) return;
    // Inflater chunk-wise checksum (16 KiB chunks, adler32.ts NMAX quirk): only a final
    // chunk of 5552 or 11104 bytes differs from the plain adler32; then replay that
    // chunk from the state at its start, S and T of the bytes before it
    const uint32_t r = (uint32_t)(pos & 16383u);
    const bool quirk = !gz && (r == 5552u || r == 11104u);
    uint32_t snapS = S_all, snapT = T_all;
    if (quirk) {
        uint64_t a = 0, b = 0;
        const uint64_t c = pos - r;
        for (uint32_t k = tid; k < r; k += RS_THREADS) {
            const uint32_t v = out[c + k];
            a += v;
            b += (uint64_t)((c + k) % 65521u) * v;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) { a += __shfl_xor(a, o); b += __shfl_xor(b, o); }
        if (lane == 0) { red[w][0] = a; red[w][1] = b; }
        __syncthreads();
        uint64_t ta = 0, tb = 0;
#pragma unroll
        for (int q = 0; q < RS_WAVES; ++q) { ta += red[q][0]; tb += red[q][1]; }
        snapS = (uint32_t)((S_all + 65521u - mod65521(ta)) % 65521u);
        snapT = (uint32_t)((T_all + 65521u - mod65521(tb)) % 65521u);
    }
    if (tid != 0) return;
    // final: record + verdicts (sd-inflate.ts:134-179); gzip's crc32 comes from k_inflate_finalize
    sdz_inflate_record Rc;
    Rc.status = S->status;
    Rc.zmsg = S->zmsg;
    Rc.out_len = pos;
    uint64_t ib = S->bitpos;
    uint64_t ilen = A.in_len[sid];
    Rc.in_used = (ib + 7) >> 3;
    if (Rc.in_used > ilen) Rc.in_used = ilen;
    Rc.stored_checksum = S->stored_ck;
    bool have = pos > 0;                                  // Inflater.checksum stays undefined otherwise
    int32_t running = 0;
    if (!gz) {
        const uint64_t n = quirk ? pos - r : pos;
        const uint32_t nm = mod65521(n), Sx = quirk ? snapS : S_all, Tx = quirk ? snapT : T_all;
        const uint32_t a1 = (1u + Sx) % 65521u;
        const uint32_t a2 = (uint32_t)(((uint64_t)nm + (uint64_t)nm * Sx + 65521ull * 65521ull - Tx) % 65521u);
        if (quirk) running = adler_quirk_tail(out + (pos - r), r, a1, a2);
        else running = (int32_t)(a1 | (a2 << 16));
    }
    Rc.running_checksum = have ? running : 0;
    Rc.stored_size = S->stored_size;
    Rc.mtime = S->mtime;
    Rc.name_off = S->name_off;
    Rc.name_len = S->name_len;
    Rc.container = (uint8_t)S->container;
    bool complete = S->mode == LM_DONE && (S->status == SDZ_OK || S->status == SDZ_TRAILING);
    Rc.complete = complete ? 1 : 0;
    uint8_t cv = S->stored_ck == 0 ? SDZ_UNCHECKED : ((have && S->stored_ck == running) ? SDZ_MATCH : SDZ_MISMATCH);
    uint8_t sv = S->stored_size == 0 ? SDZ_UNCHECKED
               : ((int64_t)S->stored_size == (int64_t)pos ? SDZ_MATCH : SDZ_MISMATCH);
    Rc.checksum_verdict = cv;
    Rc.size_verdict = sv;
    Rc.success = (complete && cv != SDZ_MISMATCH && sv != SDZ_MISMATCH) ? 1 : 0;
    for (int k = 0; k < 11; ++k) Rc.reserved[k] = 0;
    A.rec[sid] = Rc;
}

// ------------------------------------------------------------------ gzip: crc32 + verdicts

__device__ uint32_t gf2_mul(uint32_t a, uint32_t b) {       // a * b mod P (reflected)
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
__device__ uint32_t gf2_xbytes(uint64_t n, const uint32_t* x2n) {   // x^(8n) mod P
    uint32_t p = 1u << 31;
    unsigned k = 3;
    while (n) {
        if (n & 1) p = gf2_mul(x2n[k & 31], p);
        n >>= 1;
        k++;
    }
    return p;
}

// one wave per finished gzip stream: crc32 of its output (64 lane chunks merged with
// polynomial shifts) and the checksum verdicts that depend on it
__global__ __launch_bounds__(64) void k_inflate_finalize(InflateArgs A) {
    __shared__ uint32_t tab[256];
    __shared__ uint32_t x2n[32];
    const uint32_t sid = blockIdx.x;
    if (sid >= A.n) return;
    sdz_inflate_record* rec = A.rec + sid;
    if (rec->container != SDZ_CONTAINER_GZIP) return;
    const uint32_t lane = threadIdx.x;
    for (uint32_t v = lane; v < 256; v += 64) {
        uint32_t c = v;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
        tab[v] = c;
    }
    if (lane == 0) {
        uint32_t p = 1u << 30;
        x2n[0] = p;
        for (int k = 1; k < 32; ++k) x2n[k] = p = gf2_mul(p, p);
    }
    __syncthreads();
    const uint8_t* p = A.out + A.out_off[sid];
    const uint64_t len = rec->out_len;
    const uint64_t chunk = (len + 63) / 64;
    const uint64_t b0 = (uint64_t)lane * chunk;
    const uint64_t b1 = b0 + chunk < len ? b0 + chunk : len;
    uint64_t l = b1 > b0 ? b1 - b0 : 0;
    uint32_t cr = 0xffffffffu;
    for (uint64_t i = b0; i < b1; ++i) cr = tab[(cr ^ p[i]) & 255] ^ (cr >> 8);
    uint32_t crc = ~cr;
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t rc = __shfl_down(crc, o);
        uint64_t rl = __shfl_down(l, o);
        if ((lane & (2 * o - 1)) == 0 && lane + o < 64) {
            crc = gf2_mul(gf2_xbytes(rl, x2n), crc) ^ rc;
            l += rl;
        }
    }
    if (lane != 0) return;
    const bool have = len > 0;
    const int32_t running = (int32_t)crc;
    rec->running_checksum = have ? running : 0;
    const uint8_t cv = rec->stored_checksum == 0 ? SDZ_UNCHECKED
                     : ((have && rec->stored_checksum == running) ? SDZ_MATCH : SDZ_MISMATCH);
    rec->checksum_verdict = cv;
    rec->success = (rec->complete && cv != SDZ_MISMATCH && rec->size_verdict != SDZ_MISMATCH) ? 1 : 0;
}

uint32_t resolve_block_threads() { return RS_THREADS; }
uint32_t resolve_streams_per_block() { return 1; }
void launch_inflate_finalize(const InflateArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_inflate_finalize, dim3(a.n), dim3(64), 0, s, a);
}

}  // namespace sdz
