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
#define RS_R 36864                    // ring bytes: 32 KiB window + one batch
#define RS_STAGE 4096                 // batch output budget
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

// batch byte x (>= 0) of a token: literal byte, or the source position it copies
// (self-overlapping matches fold into their first period)
__device__ __forceinline__ uint32_t owner_of(const uint32_t* bm, const uint16_t* bp, uint32_t x) {
    const uint32_t wd = bm[x >> 5];
    return (uint32_t)bp[x >> 5] + (uint32_t)__popc(wd << (31u - (x & 31u))) - 1u;
}

__global__ __launch_bounds__(RS_THREADS) void k_inflate_resolve(InflateArgs A, uint32_t round) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[RS_R];
    __shared__ __attribute__((aligned(16))) uint32_t btok[RS_THREADS];   // the batch's tokens
    __shared__ __attribute__((aligned(16))) uint16_t bstart[RS_THREADS]; // their output offsets
    __shared__ uint32_t bm[RS_STAGE / 32];               // bit x: a token starts at batch byte x
    __shared__ uint16_t bp[RS_STAGE / 32];               // tokens starting before word k
    __shared__ uint32_t red[RS_WAVES][4];

    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    const uint32_t sid = blockIdx.x;
    if (sid >= A.n) return;
    const uint32_t flag = A.flags[sid];
    if (flag == 2) return;
    RSave* R = (RSave*)A.rsave + sid;
    const DSave* S = (const DSave*)A.dsave + sid;
    const bool gz = S->container == SDZ_CONTAINER_GZIP;
    uint64_t pos;
    uint32_t s1, s2, snap1, snap2;
    if (round == 0) { pos = 0; s1 = 1; s2 = 0; snap1 = 1; snap2 = 0; }
    else { pos = R->pos; s1 = R->s1; s2 = R->s2; snap1 = R->snap1; snap2 = R->snap2; }
    uint8_t* out = A.out + A.out_off[sid];
    const uint32_t* tk = A.tokens + (uint64_t)sid * A.round_tokens;
    const uint32_t ntok = A.ntok[sid];
    const int64_t dl = S->dict_used && A.dict ? (A.dict_len > 32767 ? 32767 : A.dict_len) : 0;
    const uint8_t* dict = dl ? A.dict + (A.dict_len - dl) : nullptr;

    // the window: output bytes [pos - 32 KiB, pos), the dictionary / zeros before 0
    uint32_t rp = (uint32_t)(pos % RS_R);
    for (uint32_t k = tid; k < RS_WIN; k += RS_THREADS) {
        int64_t p = (int64_t)pos - RS_WIN + k;
        uint32_t b = 0;
        if (p >= 0) b = round ? out[p] : 0u;
        else if (p >= -dl) b = dict[dl + p];
        ring[ridx((int32_t)((int64_t)rp - RS_WIN + k))] = (uint8_t)b;
    }

    // every wave scans the whole batch itself (4 tokens per lane), so the batch
    // layout needs no cross-wave exchange; wave 0 publishes it for the byte phase
    uint32_t t4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) t4[k] = 4 * lane + k < ntok ? tk[4 * lane + k] : 0u;
    for (uint32_t base = 0; base < ntok;) {
        uint32_t l4[4], e4[4];
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t t = t4[k];
            const bool inr = base + 4 * lane + k < ntok;
            l4[k] = !inr ? 0u : (t >> 31) ? ((t >> 16) & 255u) + 3u : ((t >> 24) & 3u) + 1u;
            acc += l4[k];
            e4[k] = acc;                                 // inclusive, lane-local
        }
        const uint32_t lx = wave_incl_scan(acc) - acc;   // exclusive lane prefix
        // tokens taken: the longest prefix whose output fits the stage (>= 1 token)
        uint64_t fits = __ballot(lx + e4[3] <= RS_STAGE);
        const uint32_t fl = fits == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~fits);   // first lane not all-fitting
        uint32_t kin = 0;                                // tokens of lane fl that fit
        {
            const uint32_t lxf = (uint32_t)__shfl((int)lx, (int)(fl & 63u));
            uint32_t c = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t ek = (uint32_t)__shfl((int)e4[k], (int)(fl & 63u));
                c += lxf + ek <= RS_STAGE ? 1u : 0u;
            }
            kin = fl == 64u ? 0u : c;
        }
        uint32_t ntk = 4 * fl + kin;
        if (ntk == 0) ntk = 1;
        if (ntk > ntok - base) ntk = ntok - base;
        const uint32_t lastl = (ntk - 1) >> 2, lastk = (ntk - 1) & 3u;
        uint32_t ev = lastk == 0 ? e4[0] : lastk == 1 ? e4[1] : lastk == 2 ? e4[2] : e4[3];
        const uint32_t B = (uint32_t)__shfl((int)(lx + ev), (int)lastl);
        if (w == 0) {
            *(uint4*)&btok[4 * lane] = make_uint4(t4[0], t4[1], t4[2], t4[3]);
            uint32_t st0 = lx, st1 = lx + e4[0], st2 = lx + e4[1], st3 = lx + e4[2];
            *(uint2*)&bstart[4 * lane] = make_uint2(st0 | (st1 << 16), st2 | (st3 << 16));
            bm[lane] = 0;
            bm[lane + 64] = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t j = 4 * lane + k;
                const uint32_t st = k == 0 ? st0 : k == 1 ? st1 : k == 2 ? st2 : st3;
                if (j < ntk) atomicOr(&bm[st >> 5], 1u << (st & 31u));
            }
            const uint32_t c0 = (uint32_t)__popc(bm[2 * lane]), c1 = (uint32_t)__popc(bm[2 * lane + 1]);
            const uint32_t px = wave_incl_scan(c0 + c1) - (c0 + c1);
            bp[2 * lane] = (uint16_t)px;
            bp[2 * lane + 1] = (uint16_t)(px + c0);
        }
        // next batch's tokens
        const uint32_t nb = base + ntk;
#pragma unroll
        for (int k = 0; k < 4; ++k) t4[k] = nb + 4 * lane + k < ntok ? tk[nb + 4 * lane + k] : 0u;
        __syncthreads();

        // bytes: each thread builds whole output dwords; a byte chases in-batch
        // references back to a literal or to a byte before the batch
        const uint32_t head = rp & 3u;
        const uint32_t nd = (head + B + 3u) >> 2;
        const uint32_t rd0 = (rp - head) >> 2;
        uint32_t* dstw = (uint32_t*)(out + (pos - head));
        uint32_t* ring32 = (uint32_t*)ring;
        const uint64_t cut = ((pos + B) >> 14) << 14;
        const bool cross = (pos >> 14) != ((pos + B) >> 14);
        const uint32_t c = cross ? (uint32_t)(cut - pos) : 0u;
        uint32_t S1 = 0, W = 0, Sc = 0, Wc = 0;
        for (uint32_t q = tid; q < nd; q += RS_THREADS) {
            uint32_t ri = rd0 + q;
            ri -= ri >= RS_R / 4 ? RS_R / 4 : 0;
            uint32_t v = ring32[ri];                     // head bytes are final already
            const int32_t x0 = (int32_t)(4 * q) - (int32_t)head;
            int32_t cur[4];
            uint32_t val[4];
            uint32_t pend = 0;                           // bytes still chasing a reference
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                cur[b] = x0 + b;
                pend |= (cur[b] >= 0 && cur[b] < (int32_t)B) ? 1u << b : 0u;
                val[b] = (v >> (8 * b)) & 255u;
            }
            // branch-free per byte: every load is unconditional, every update a select
            do {
                int32_t kk[4], dd[4], ss[4];
                uint32_t tt[4];
                bool wrap = false;                       // some byte inside a self-overlapping match
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const uint32_t x = (pend >> b) & 1u ? (uint32_t)cur[b] : 0u;
                    const uint32_t j = owner_of(bm, bp, x);
                    tt[b] = btok[j];
                    ss[b] = (int32_t)bstart[j];
                    kk[b] = (int32_t)x - ss[b];
                    dd[b] = (int32_t)(tt[b] & 0x7fffu) + 1;
                    const int32_t len = (int32_t)((tt[b] >> 16) & 255u) + 3;
                    wrap |= ((tt[b] >> 31) != 0) & (kk[b] >= dd[b]) & (dd[b] < len);
                }
                if (__ballot(wrap)) {                    // fold into the first period: k mod dist
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const int32_t k = kk[b], d = dd[b];
                        int32_t r = k - (int32_t)((float)k * __builtin_amdgcn_rcpf((float)d)) * d;
                        r += r < 0 ? d : 0;
                        r -= r >= d ? d : 0;
                        kk[b] = ((tt[b] >> 31) != 0 && k >= d) ? r : k;
                    }
                }
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const bool lit = (tt[b] >> 31) == 0;
                    const int32_t src = ss[b] + kk[b] - dd[b];
                    uint32_t pre = ring[ridx((int32_t)rp + (src < 0 ? src : -1))];
                    asm volatile("" : "+v"(pre));            // keep the load unconditional (no branch)
                    const uint32_t r = lit ? (tt[b] >> (8 * ((uint32_t)kk[b] & 3u))) & 255u : pre;
                    const bool act = (pend >> b) & 1u;
                    const bool done = lit || src < 0;
                    val[b] = act && done ? r : val[b];
                    cur[b] = act && !done ? src : cur[b];
                    pend &= act && done ? ~(1u << b) : ~0u;
                }
            } while (__ballot(pend != 0));
            v = val[0] | (val[1] << 8) | (val[2] << 16) | (val[3] << 24);
            ring32[ri] = v;
            if (q + 1 < nd || ((head + B) & 3u) == 0) dstw[q] = v;
            else for (uint32_t bb = 0; bb < ((head + B) & 3u); ++bb) ((uint8_t*)(dstw + q))[bb] = (uint8_t)(v >> (8 * bb));
            if (!gz) {
                // bytes of this dword inside the batch: [lo, hi)
                const uint32_t j = (uint32_t)x0;                 // batch index of byte 0 (mod 2^32)
                const uint32_t lo = q == 0 ? head : 0u;
                const uint32_t hi = q + 1 < nd ? 4u : (((head + B) & 3u) ? ((head + B) & 3u) : 4u);
                const uint32_t m = (hi == 4u ? ~0u : (1u << (8 * hi)) - 1u) & (~0u << (8 * lo));
                const uint32_t vm = v & m;
                // sum b and sum (B - j - bb) b over the dword's bytes, via v_dot4_u32_u8
                const uint32_t s4 = __builtin_amdgcn_udot4(vm, 0x01010101u, 0u, false);
                S1 += s4;
                W += (B - j) * s4 - __builtin_amdgcn_udot4(vm, 0x03020100u, 0u, false);
                if (cross) {                                     // bytes before the 16 KiB cut
                    const uint32_t cl = c - j;
                    const uint32_t mc = (int32_t)cl <= 0 ? 0u : cl >= 4u ? ~0u : (1u << (8 * cl)) - 1u;
                    const uint32_t vc = vm & mc;
                    const uint32_t c4 = __builtin_amdgcn_udot4(vc, 0x01010101u, 0u, false);
                    Sc += c4;
                    Wc += (c - j) * c4 - __builtin_amdgcn_udot4(vc, 0x03020100u, 0u, false);
                }
            }
        }
        if (!gz) {
            S1 = wave_sum(S1);
            W = wave_sum(W) % 65521u;
            Sc = wave_sum(Sc);
            Wc = wave_sum(Wc) % 65521u;
            if (lane == 0) { red[w][0] = S1; red[w][1] = W; red[w][2] = Sc; red[w][3] = Wc; }
        }
        __syncthreads();
        if (!gz) {
            uint64_t tS = 0, tW = 0, tSc = 0, tWc = 0;
#pragma unroll
            for (int q = 0; q < RS_WAVES; ++q) { tS += red[q][0]; tW += red[q][1]; tSc += red[q][2]; tWc += red[q][3]; }
            if (cross) {
                snap1 = (uint32_t)(((uint64_t)s1 + tSc) % 65521u);
                snap2 = (uint32_t)(((uint64_t)s2 + (uint64_t)c * s1 + tWc) % 65521u);
            }
            s2 = (uint32_t)(((uint64_t)s2 + (uint64_t)B * s1 + tW) % 65521u);
            s1 = (uint32_t)(((uint64_t)s1 + tS) % 65521u);
        }
        pos += B;
        rp = ridx((int32_t)(rp + B));
        base = nb;
    }
    if (tid == 0) {
        R->pos = pos; R->s1 = s1; R->s2 = s2; R->snap1 = snap1; R->snap2 = snap2;
    }
    if (flag != 1 || tid != 0) return;
    __threadfence_block();
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
        uint32_t r = (uint32_t)(pos & 16383u);
        if (r == 5552u || r == 11104u) running = adler_quirk_tail(out + (pos - r), r, snap1, snap2);
        else running = (int32_t)(s1 | (s2 << 16));
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
