// k_resolve.hip -- batched DEFLATE decoder, phase 2: tokens -> bytes, adler32, and the
// Inflater verdicts (src/sd-inflate.ts:134-179); k_inflate_finalize adds crc32 for gzip.
//
// One WORKGROUP of RS_WAVES waves per stream, four streams per CU.  The stream's LZ77
// window lives in LDS: a 35.5 KiB ring holds the last 32 KiB of output plus the bytes in
// flight, so back-references never leave the CU.
//
// Waves 0 .. RS_EW-1 (the emitters) form a pipeline without block barriers.  The round's
// tokens are cut into GROUPS of 64 (one per lane); emitter w takes groups w, w + RS_EW,
// ...  Per group:
//   1. lengths and a DPP wave scan give the group's byte count T; the group's start S
//      comes from its predecessor through a one-word LDS chain (tag, end), and S + T
//      is passed on at once, so starts run ahead of the copying;
//   2. rounds: every token whose source bytes are final is written -- literals and plain
//      copies as masked dword read-modify-writes (emit_msk), the rest by emit_tokens.
//      "Final" means below the stream-wide frontier Wf, or marked in the finality map;
//   3. the group publishes Wf = S + T once Wf reached S (in order).
// The last wave (the writer) copies final bytes to HBM in output-aligned 1 KiB chunks,
// folds them into adler32 (S = sum b, T = sum i b as whole-output sums) and publishes Wwb
// (bytes written back, which frees their ring slots).  The emitters issue no global
// stores, so the wait for their token prefetch never covers write-back stores.
// A head group (Wf == S) publishes its finished prefix as it goes, so a large group
// never waits on its own ring space.  Ring-space rule: writing byte p needs
// p < Wf + (R - 32 KiB) (no reader needs byte p - R any more) and p < Wwb + R (byte
// p - R is in HBM).  Every wait is bounded (SDZ_INTERNAL if a bound trips).
// Positions before the output start read the preset dictionary or zeros.
#include "inflate_state.h"
#include "crc32_dev.h"
#include <algorithm>
#include <type_traits>

namespace sdz {

#ifndef RS_WAVES
#define RS_WAVES 8
#endif
#define RS_EW (RS_WAVES - 1)           // emitter waves; the last wave writes back
#define RS_THREADS (64 * RS_WAVES)
#define RS_WIN 32768
#ifndef RS_R
#define RS_R 36352                    // ring bytes: 32 KiB window + bytes in flight
#endif
#define RS_SLACK (RS_R - RS_WIN)
#ifndef RS_WPE
#define RS_WPE RS_WAVES               // waves per SIMD the register budget is sized for
#endif
#ifndef RS_NAP
#define RS_NAP 12                     // s_sleep units (64 clocks) between polls (8: C2 resolve +0.5 ms, distinct +0.2 ms)
#endif
#ifndef RS_BM
#define RS_BM 4096                    // finality map bytes (a power of 2 >= RS_SLACK; lap = position / RS_BM)
#endif
#define RS_SPIN_LIMIT (1u << 22)      // watchdog: polls per wait (~0.4 s)

template <uint32_t RR>
__device__ __forceinline__ uint32_t ridx_t(int32_t x) {          // x in (-R, 2R)
    x += x < 0 ? (int32_t)RR : 0;
    x -= x >= (int32_t)RR ? (int32_t)RR : 0;
    return (uint32_t)x;
}
__device__ __forceinline__ uint32_t ridx(int32_t x) { return ridx_t<RS_R>(x); }

// inclusive wave scan with DPP row shifts and row broadcasts (gfx9)
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
// lane & 7, recomputed where it is used (volatile: not hoisted out of a loop and kept live, which made
// the register allocator spill the LDS addresses built from it to scratch)
__device__ __forceinline__ uint32_t lane_lo8() {
    uint32_t r;
    asm volatile("v_and_b32 %0, 7, %1" : "=v"(r) : "v"(threadIdx.x));
    return r;
}
__device__ __forceinline__ uint32_t tid_fresh() {
    uint32_t r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(threadIdx.x));
    return r;
}
// inclusive prefix max over lanes 0..7 (row 0): lane 7 holds the max of lanes 0..7
__device__ __forceinline__ uint32_t dpp_max8(uint32_t x) {
    uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x = x > y ? x : y;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);            // row_shr:2
    x = x > y ? x : y;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);            // row_shr:4
    return x > y ? x : y;
}
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint32_t lane_at(uint32_t x, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l);
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

// LDS-only ordering for the frontier words (no wait on outstanding HBM stores)
__device__ __forceinline__ void lds_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local"); }
__device__ __forceinline__ void lds_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); }
__device__ __forceinline__ uint32_t lds_get(uint32_t* p) {
    return uni(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ uint64_t lds_get64(uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_put(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <uint32_t RR>
__device__ __forceinline__ uint32_t ridx64(int64_t p) {         // ring index of a (call-relative) position
    int64_t x = p % (int64_t)RR;
    return (uint32_t)(x < 0 ? x + RR : x);
}

// adler32.ts:34-105 over the r ring bytes from position p0, seeded with the chunk-start
// state (NMAX quirk: sum2 += BASE instead of a reduction after each 5552-byte block)
template <uint32_t RR>
__device__ int32_t adler_quirk_ring(const uint8_t* ring, int64_t p0, uint32_t r, uint32_t s1, uint32_t s2in) {
    uint64_t a = s1, s2 = s2in;
    int64_t off = p0;
    uint32_t len = r;
    while (len >= 5552) {
        len -= 5552;
        for (int i = 0; i < 5552; ++i) { a += ring[ridx64<RR>(off++)]; s2 += a; }
        a %= 65521u;
        s2 += 65521u;
    }
    if (len) {
        while (len--) { a += ring[ridx64<RR>(off++)]; s2 += a; }
        a %= 65521u;
        s2 %= 65521u;
    }
    return (int32_t)((uint32_t)a | ((uint32_t)s2 << 16));
}

// Write the bytes of the lanes' tokens into the ring and mark them in the finality map
// -- called by a whole wave; lanes with `act` set write their token (d, s: ring indices
// of destination and source; mp: map index of the destination, lb: its lap byte).
// Every LDS access is aligned (an unaligned ds_read_b32/ds_write_b32 costs ~10x an
// aligned one on gfx950: measured, tools/ubench/lds_cost.hip).  A token is written as
// head bytes up to a dword boundary, whole aligned dwords, tail bytes; a copy's source
// dwords are assembled from aligned reads with v_alignbyte.  Copies whose source cannot
// reach what a step writes (dist >= 8 or no self-overlap) move two dwords per step,
// all reads before the writes; the others go dword by dword.  Loops run to the wave's
// longest job; writes past a token's end go to the lane's dummy slot, so output is
// exact without divergent branches.  Tokens that cross the ring's (or the map's) end
// go byte-serial.  Ring bytes are stored before their map bytes (LDS operations of a
// wave complete in order), so a reader that sees the map byte sees the data.
#define RS_DUMMY (RR + 4u * (threadIdx.x & 63u))
#define RS_CBAR() asm volatile("" ::: "memory")
__device__ __forceinline__ uint32_t lap_next(uint32_t lb) { return (lb & 127u) + 1u; }
// the 4 bytes of a period-`dist` (1..3) pattern P starting at phase ph: byte j = P[(ph + j) mod dist]
__device__ __forceinline__ uint32_t rep4(uint32_t P, uint32_t dist, uint32_t ph) {
    // selector bytes (ph + j) mod dist = bytes ph..ph+3 of the sequence 0,1,2,0,1,2,0,1 (or 0,1,...)
    const uint32_t lo = dist == 3 ? 0x00020100u : dist == 2 ? 0x01000100u : 0u;
    const uint32_t hi = dist == 3 ? 0x01000201u : lo;
    return __builtin_amdgcn_perm(P, P, __builtin_amdgcn_alignbyte(hi, lo, ph));
}
// 4 bytes of source starting at ring index x, from two aligned reads
__device__ __forceinline__ uint32_t src_word(const uint32_t* ring32, uint32_t x) {
    return __builtin_amdgcn_alignbyte(ring32[(x >> 2) + 1], ring32[x >> 2], x & 3u);
}
template <uint32_t RR, bool MAP>
__device__ __forceinline__ void emit_tokens_body(uint8_t* ring, uint8_t* fmap, bool act, uint32_t t, uint32_t d,
                                                 uint32_t s, uint32_t len, uint32_t dist, uint32_t mp, uint32_t lb) {
    uint32_t* ring32 = (uint32_t*)ring;
    uint32_t* fmap32 = (uint32_t*)fmap;
    uint8_t* dum8 = ring + RS_DUMMY;
    uint16_t* dum16 = (uint16_t*)(ring + RS_DUMMY);
    uint32_t* dum32 = ring32 + RS_DUMMY / 4;
    const bool lit = (t >> 31) == 0;
    const bool slow = act && (d + len > RR || (!lit && (s + len > RR || s < 4u)) || (MAP && mp + len > RS_BM));
    const bool fast = act && !slow;
    const bool per = fast && !lit && dist < 4;
    const bool cp = fast && !lit && dist >= 4;
    const uint32_t kd = d & 3u;
    const uint32_t h0 = (4u - kd) & 3u;
    const uint32_t h = fast ? (len < h0 ? len : h0) : 0u;
    const uint32_t nf = fast ? (len - h) >> 2 : 0u;
    const uint32_t r = fast ? len - h - 4 * nf : 0u;
    const uint32_t e = d + h + 4 * nf;                   // tail start (aligned)
    const uint32_t lw = lb * 0x01010101u;
    // the first source word: head bytes of a copy, or a period's pattern
    uint32_t H = 0;
    if (__ballot(fast && !lit)) H = src_word(ring32, fast && !lit ? s : 0u);
    const uint32_t Vh = lit ? t : per ? rep4(H, dist, 0) : H;
    // head: bytes [d, d + h) -- b8 at d (odd d or one byte), b16 at the even position, and
    // the second byte of a 2-byte head at d = 1 mod 4
    {
        const bool w8 = h > 0 && ((kd & 1u) || h == 1);
        const bool w16 = h >= 2 && !(kd == 1 && h == 2);
        const uint32_t p16 = kd == 1 ? d + 1 : d;
        const uint32_t v16 = kd == 1 ? Vh >> 8 : Vh;
        *(w8 ? ring + d : dum8) = (uint8_t)Vh;
        *(w16 ? (uint16_t*)(ring + p16) : dum16) = (uint16_t)v16;
        RS_CBAR();
        if constexpr (MAP) {
            *(w8 ? fmap + mp : dum8) = (uint8_t)lb;
            *(w16 ? (uint16_t*)(fmap + (mp + (p16 - d))) : dum16) = (uint16_t)lw;
        }
        const bool w8b = kd == 1 && h == 2;
        if (__ballot(w8b)) {
            *(w8b ? ring + d + 1 : dum8) = (uint8_t)(Vh >> 8);
            RS_CBAR();
            if constexpr (MAP) {
                *(w8b ? fmap + mp + 1 : dum8) = (uint8_t)lb;
            }
        }
    }
    // body: whole aligned dwords
    const uint32_t db = (d + h) >> 2, mb = (mp + h) >> 2;   // dword indices of the first body dword
    const uint32_t ss = s + h, sa = ss >> 2, k = ss & 3u;    // source: aligned base, byte shift
    const bool wide = per || (cp && (dist >= 8 || dist >= len));
    const uint32_t na = wide ? nf : 0u, nb = cp && !wide ? nf : 0u;
    uint32_t ph = per ? (dist == 3 ? h % 3u : h & (dist - 1u)) : 0u;   // phase of body dword 0
    for (uint32_t q = 0; __ballot(q < na); q += 2) {
        uint32_t a[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) a[j] = ring32[cp && q + j <= na ? sa + q + j : 0u];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t v = per ? rep4(H, dist, ph) : __builtin_amdgcn_alignbyte(a[j + 1], a[j], k);
            ph = dist == 3 ? (ph == 2 ? 0u : ph + 1u) : ph;  // +4 mod 3 = +1; mod 2 and 1: unchanged
            *(q + j < na ? ring32 + db + q + j : dum32) = v;
        }
        RS_CBAR();
        if constexpr (MAP) {
#pragma unroll
            for (int j = 0; j < 2; ++j) *(q + j < na ? fmap32 + mb + q + j : dum32) = lw;
        }
    }
    for (uint32_t q = 0; __ballot(q < nb); ++q) {
        const bool a = q < nb;
        const uint32_t x0 = ring32[a ? sa + q : 0u], x1 = ring32[a ? sa + q + 1 : 0u];
        *(a ? ring32 + db + q : dum32) = __builtin_amdgcn_alignbyte(x1, x0, k);
        RS_CBAR();
        if constexpr (MAP) {
            *(a ? fmap32 + mb + q : dum32) = lw;
        }
    }
    // tail: bytes [e, e + r) -- b16 at e, b8 at e + r - 1 for odd r
    if (__ballot(r != 0)) {
        uint32_t T = 0;
        if (__ballot(cp && r)) T = src_word(ring32, cp && r ? s + h + 4 * nf : 0u);
        const uint32_t pt = dist == 3 ? (h + nf) % 3u : h & (dist - 1u);   // phase (h + 4 nf) mod dist
        const uint32_t Vt = lit ? t >> (8 * h) : per ? rep4(H, dist, pt) : T;
        const bool w16 = r >= 2, w8 = r & 1u;
        *(w16 ? (uint16_t*)(ring + e) : dum16) = (uint16_t)Vt;
        *(w8 ? ring + e + r - 1 : dum8) = (uint8_t)(Vt >> (8 * (r - 1)));
        RS_CBAR();
        if constexpr (MAP) {
            *(w16 ? (uint16_t*)(fmap + (mp + (e - d))) : dum16) = (uint16_t)lw;
            *(w8 ? fmap + (mp + (e - d) + r - 1) : dum8) = (uint8_t)lb;
        }
    }
    if (__ballot(slow)) {                                 // across the ring's / map's end: byte-serial
        for (uint32_t i = 0; __ballot(slow && i < len); ++i) {
            const bool a = slow && i < len;
            const uint32_t b = lit ? (t >> (8 * (i & 3u))) & 255u : ring[a && !lit ? ridx_t<RR>((int32_t)(s + i)) : 0u];
            ring[a ? ridx_t<RR>((int32_t)(d + i)) : RS_DUMMY] = (uint8_t)b;
            RS_CBAR();
            const uint32_t m = mp + i;
            if constexpr (MAP) {
                *(a ? fmap + (m & (RS_BM - 1)) : ring + RS_DUMMY) = (uint8_t)(m >= RS_BM ? lap_next(lb) : lb);
            }
        }
    }
}

template <uint32_t RR, bool MAP>
__device__ __noinline__ void emit_tokens(uint8_t* ring, uint8_t* fmap, bool act, uint32_t t, uint32_t d,
                                            uint32_t s, uint32_t len, uint32_t dist, uint32_t mp, uint32_t lb) {
    emit_tokens_body<RR, MAP>(ring, fmap, act, t, d, s, len, dist, mp, lb);
}

template <int J, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (J < N) {
        f(std::integral_constant<int, J>{});
        static_for<J + 1, N>(f);
    }
}
// LDS masked write of dword i + J (J a compile-time word offset): bytes selected by `mask`
// take those of v; an atomic read-modify-write (ds_mskor_b32: D = (D & ~mask) | (v & mask)),
// so lanes writing different bytes of one dword in the same instruction are all kept
typedef __attribute__((address_space(3))) uint32_t lds_u32;
template <int J>
__device__ __forceinline__ void lds_mskor_at(uint32_t* base32, uint32_t i, uint32_t mask, uint32_t v) {
    const uint32_t a = (uint32_t)(uintptr_t)(lds_u32*)(base32 + i);
    asm volatile("ds_mskor_b32 %0, %1, %2 offset:%3" :: "v"(a), "v"(mask), "v"(v & mask), "i"(4 * J) : "memory");
}

// The lanes' tokens with few instructions (measured 2.3x fewer cycles than emit_tokens,
// tools/ubench/emit.hip): every token is written as dwords v_j = alignbyte(x[j+1], x[j], k)
// masked to its bytes -- a copy's x are its source dwords (aligned reads, all issued before
// the writes), a literal's are its 1-3 bytes placed so that the same formula lands them at
// d -- RS_MW dwords per step (tokens up to 4 RS_MW - 3 bytes take one step), each followed
// by the same mask on the finality map (map index = ring index mod 4).  Masked writes
// outside a token are no-ops.  Copies that overlap themselves (periods included), and
// tokens across the ring's end, go through emit_tokens (across the map's end: wrapped here).
#ifndef RS_MW
#define RS_MW 2
#endif
#ifndef RS_READ_ALL
#define RS_READ_ALL 1
#endif
#ifndef RS_MAP2
#define RS_MAP2 1                     // finality-map check: two map dwords per loop pass
#endif
// GEN: 0 -- no lane needs the general path (the caller routed them elsewhere); 1 -- through the
// out-of-line emit_tokens; 2 -- emit_tokens inlined (one call site per kernel: no callee-saved
// registers forced around a call)
template <uint32_t RR, bool MAP, int MW, int GEN = 1>
__device__ __forceinline__ void emit_msk(uint8_t* ring, uint8_t* fmap, bool act, uint32_t t, uint32_t d,
                                         uint32_t s, uint32_t len, uint32_t dist, uint32_t mp, uint32_t lb) {
    uint32_t* ring32 = (uint32_t*)ring;
    uint32_t* fmap32 = (uint32_t*)fmap;
    const uint32_t dumi = RR / 4 + (threadIdx.x & 31u);     // reads run MW dwords on
    const bool lit = (t >> 31) == 0;
    // (a token across the map's end stays here: its map dwords wrap, with the next lap's byte)
    const bool slow = act && (d + len > RR || (!lit && (s + len > RR || s < 4u)));
    const bool gen = act && (slow || (!lit && dist < len));  // periods and self-overlapping copies too
    if constexpr (GEN == 1) {
        if (__ballot(gen)) emit_tokens<RR, MAP>(ring, fmap, gen, t, d, s, len, dist, mp, lb);
    } else if constexpr (GEN == 2) {
        if (__ballot(gen)) emit_tokens_body<RR, MAP>(ring, fmap, gen, t, d, s, len, dist, mp, lb);
    }
    const bool one = act && !gen;
    const uint32_t kd = d & 3u, D0 = d >> 2, M0 = mp >> 2;
    const uint32_t sx = s - kd, k = sx & 3u;
    const uint32_t xa = one && !lit ? sx >> 2 : dumi;
    const uint32_t e = one ? kd + len : 0u;               // token end, in bytes from dword D0
    const uint32_t lw = lb * 0x01010101u;
    // a literal: x0 = t (kd = 0), or x0 = 0, x1 = t with shift 4 - kd
    const uint32_t kk = lit ? (4u - kd) & 3u : k;
    uint32_t x[MW + 1], r[MW + 1];
#pragma unroll
    for (int j = 0; j <= MW; ++j) r[j] = ring32[xa + (uint32_t)j];
#if RS_READ_ALL
    // every lane reads (a literal lane its dummy dwords): without this the compiler sank the
    // reads under `if (!lit)`, an exec-mask save / branch / restore around each of them
    if constexpr (MW == 2) asm volatile("" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]));
#endif
#pragma unroll
    for (int j = 0; j <= MW; ++j)
        x[j] = !lit ? r[j] : j == 0 ? (kd ? 0u : t) : j == 1 ? (kd ? t : 0u) : 0u;
    const uint32_t lom = 0xffffffffu << (8 * kd);
    static_for<0, MW>([&](auto jc) {                   // each dword's data, then its finality
        constexpr int j = decltype(jc)::value;
        const int32_t hb = (int32_t)e - 4 * j;            // bytes of the token in dword j: up to hb
        const uint32_t h = hb >= 4 ? 0xffffffffu : hb <= 0 ? 0u : (1u << (8 * hb)) - 1u;
        const uint32_t mk = j == 0 ? h & lom : h;
        lds_mskor_at<j>(ring32, D0, mk, __builtin_amdgcn_alignbyte(x[j + 1], x[j], kk));
        if constexpr (MAP) {
            const uint32_t mi = M0 + (uint32_t)j;            // map dword, wrapped (dword-aligned end)
            const bool wr = mi >= RS_BM / 4u;
            lds_mskor_at<0>(fmap32, wr ? mi - RS_BM / 4u : mi, mk, wr ? lap_next(lb) * 0x01010101u : lw);
        }
    });
    // later steps of copies longer than 4 RS_MW - 3 bytes
    for (uint32_t w0 = MW; __ballot(e > 4u * w0); w0 += MW) {
        const bool on = e > 4u * w0;
#pragma unroll
        for (int j = 0; j <= MW; ++j) x[j] = ring32[on ? xa + w0 + (uint32_t)j : dumi + (uint32_t)j];
#pragma unroll
        for (int j = 0; j < MW; ++j) {
            const int32_t hb = (int32_t)e - 4 * (int32_t)(w0 + j);
            const uint32_t mw = !on || hb <= 0 ? 0u : hb >= 4 ? 0xffffffffu : (1u << (8 * hb)) - 1u;
            lds_mskor_at<0>(ring32, D0 + w0 + (uint32_t)j, mw, __builtin_amdgcn_alignbyte(x[j + 1], x[j], k));
            if constexpr (MAP) {
                const uint32_t mi = M0 + w0 + (uint32_t)j;
                const bool wr = mi >= RS_BM / 4u;
                lds_mskor_at<0>(fmap32, wr ? mi - RS_BM / 4u : mi, mw, wr ? lap_next(lb) * 0x01010101u : lw);
            }
        }
    }
}

__device__ __forceinline__ uint32_t mod65521(uint64_t x) { return (uint32_t)(x % 65521u); }

// wait (bounded) until *p >= v; false if the watchdog tripped (or another wave's did)
__device__ __forceinline__ bool wait_ge(uint32_t* p, uint32_t v, uint32_t* fail) {
    for (uint32_t n = 0;; ++n) {
        if (lds_get(p) >= v) { lds_acquire(); return true; }
        if (n > RS_SPIN_LIMIT || lds_get(fail)) {
            if (!lds_get(fail)) lds_put(fail, 2u | (v << 4));   // site | position, for diagnosis
            return false;
        }
        __builtin_amdgcn_s_sleep(RS_NAP);
    }
}

// Finality map over the bytes in flight: map byte (g mod RS_BM) holds the lap byte
// ((g / RS_BM) & 127) + 1 of global position g once byte g is in the ring.  A stale value
// is a different lap, so nothing is ever cleared; a map byte overwritten by a later lap
// belongs to a byte already below Wf (RS_SLACK <= RS_BM), where the check is skipped.
// Wave-uniform loop over the aligned map dwords of [lo, hi) (low 32 bits of global
// positions) of each active lane.
__device__ __forceinline__ uint32_t lap_of(uint32_t g) { return ((g / RS_BM) & 127u) + 1u; }
__device__ __forceinline__ bool map_all(const uint8_t* fmap, bool act, uint32_t lo, uint32_t hi) {
    const uint32_t* fmap32 = (const uint32_t*)fmap;
    uint32_t miss = 0;                                    // VGPR accumulation: no lane-mask (SALU) ops
    const uint32_t n = act ? hi - lo : 0u;               // modulo 2^32: positions are low bits
    const uint32_t m0 = lo >> 2, nw = n ? ((lo & 3u) + n + 3u) >> 2 : 0u;
    const uint32_t bt = ((lo + n - 1u) & 3u) + 1u;       // bytes used of the last dword
#if RS_READ_ALL
    // byte masks without selects or branches: lanes past their last dword read map dword 0 and
    // mask it out (the compiler had turned the selects around the read into an exec-mask branch)
    const uint32_t lm = ~0u << (8 * (lo & 3u));          // the first dword's bytes
    const uint32_t hm = bt == 4u ? ~0u : (1u << (8 * bt)) - 1u;   // the last dword's
#if RS_MAP2
    // two dwords per pass (the loop's test, ballot and counters once per pair)
    for (uint32_t i = 0; __ballot(i < nw); i += 2) {
        const uint32_t m = m0 + i, m1 = m + 1u;
        const uint32_t in = (uint32_t)((int32_t)(i - nw) >> 31);        // i < nw
        const uint32_t in1 = (uint32_t)((int32_t)(i + 1u - nw) >> 31);  // i + 1 < nw
        const uint32_t in2 = (uint32_t)((int32_t)(i + 2u - nw) >> 31);  // i + 2 < nw
        const uint32_t mask = in & (in1 | hm) & (i == 0 ? lm : ~0u);
        const uint32_t mask1 = in1 & (in2 | hm);
        uint32_t v = fmap32[m & (RS_BM / 4 - 1) & in], v1 = fmap32[m1 & (RS_BM / 4 - 1) & in1];
        asm volatile("" : "+v"(v), "+v"(v1));
        miss |= ((v ^ (lap_of(4 * m) * 0x01010101u)) & mask) | ((v1 ^ (lap_of(4 * m1) * 0x01010101u)) & mask1);
    }
#else
    for (uint32_t i = 0; __ballot(i < nw); ++i) {
        const uint32_t m = m0 + i;
        const uint32_t in = (uint32_t)((int32_t)(i - nw) >> 31);        // i < nw
        const uint32_t more = (uint32_t)((int32_t)(i + 1u - nw) >> 31); // i + 1 < nw
        const uint32_t mask = in & (more | hm) & (i == 0 ? lm : ~0u);
        uint32_t v = fmap32[m & (RS_BM / 4 - 1) & in];
        asm volatile("" : "+v"(v));
        miss |= (v ^ (lap_of(4 * m) * 0x01010101u)) & mask;
    }
#endif
#else
    for (uint32_t i = 0; __ballot(i < nw); ++i) {
        const uint32_t m = m0 + i;
        const uint32_t bl = i == 0 ? lo & 3u : 0u, bh = i + 1 == nw ? bt : 4u;
        const uint32_t mask = i < nw ? (bh == 4u ? ~0u : (1u << (8 * bh)) - 1u) & (~0u << (8 * bl)) : 0u;
        const uint32_t v = fmap32[i < nw ? m & (RS_BM / 4 - 1) : 0u];
        miss |= (v ^ (lap_of(4 * m) * 0x01010101u)) & mask;
    }
#endif
    return miss == 0;
}
#ifndef RS_WAKE
#define RS_WAKE 0                     // s_wakeup after each publish: sleeping waves poll at once
#endif
__device__ __forceinline__ void rs_wake() {
#if RS_WAKE
    asm volatile("s_wakeup" ::: "memory");
#endif
}
__device__ __forceinline__ void publish_wf(uint32_t* wf, uint32_t v1) {
    lds_release();
    if ((threadIdx.x & 63u) == 0) lds_put(wf, v1);
    rs_wake();
}

// The ring's window at the start of a round (all threads; a barrier must follow): output bytes
// [pos0 - 32 KiB, pos0); before position 0 of this call, the window saved by the previous call
// (incremental mode), else the dictionary / zeros.  Position p sits at ring index p mod RR.
template <uint32_t RR, uint32_t NT>
__device__ __forceinline__ void ring_window_init(uint8_t* ring, const InflateArgs& A, uint32_t sid, uint32_t round,
                                                 uint64_t pos0, const uint8_t* out, int64_t dl, const uint8_t* dict) {
    // the window: output bytes [pos0 - 32 KiB, pos0); before position 0 of this call, the
    // window saved by the previous call (incremental mode), else the dictionary / zeros
    const uint32_t tid = threadIdx.x;
    const uint32_t rp0 = (uint32_t)(pos0 % RR);
    RSave* R = (RSave*)A.rsave + sid;
    const uint8_t* hist = A.streaming && R->hist ? A.window + (uint64_t)sid * IS_WIN : nullptr;
    static_assert((RR - RS_WIN) % 16 == 0 && IS_WIN == RS_WIN, "ring window start must be 16-aligned");
    if (pos0 == 0 && hist) {
        // ring bytes [RR - RS_WIN, RR) hold positions [-32 KiB, 0)
        for (uint32_t k = tid; k < RS_WIN / 16; k += NT)
            ((uint4*)(ring + (RR - RS_WIN)))[k] = ((const uint4*)hist)[k];
    } else if (pos0 == 0 && dl == 0) {
        // a stream's first round without a dictionary: zeros
        for (uint32_t k = tid; k < RS_WIN / 16; k += NT)
            ((uint4*)(ring + (RR - RS_WIN)))[k] = make_uint4(0, 0, 0, 0);
    } else if (round && pos0 >= RS_WIN) {
        // a later round: the 32 KiB before pos0 from the output, 4 loads in flight per thread
        for (uint32_t k = 4 * tid; k < RS_WIN; k += 4 * NT) {
            const uint8_t* q = out + pos0 - RS_WIN + k;
            const uint32_t b0 = q[0], b1 = q[1], b2 = q[2], b3 = q[3];
            const int32_t r = (int32_t)rp0 - RS_WIN + (int32_t)k;
            ring[ridx_t<RR>(r)] = (uint8_t)b0; ring[ridx_t<RR>(r + 1)] = (uint8_t)b1;
            ring[ridx_t<RR>(r + 2)] = (uint8_t)b2; ring[ridx_t<RR>(r + 3)] = (uint8_t)b3;
        }
    } else {
        for (uint32_t k = tid; k < RS_WIN; k += NT) {
            const int64_t p = (int64_t)pos0 - RS_WIN + k;
            uint32_t b = 0;
            if (p >= 0) b = round ? out[p] : 0u;
            else if (hist) b = hist[RS_WIN + p];
            else if (p >= -dl) b = dict[dl + p];
            ring[ridx_t<RR>((int32_t)rp0 - RS_WIN + (int32_t)k)] = (uint8_t)b;
        }
    }
}

// The end of a round, shared by the resolve kernels (all threads of the workgroup): the adler32
// partials combined, RSave updated, and on the stream's last round of the call the record and the
// Inflater verdicts (sd-inflate.ts:134-179), plus the incremental mode's window and carry.
// pos: output bytes of this call resolved so far (or, with chainp, pos0 + the low word of *chainp,
// read after the barrier); failp: the watchdog word (0 = none).
template <uint32_t RR, int NW>
__device__ __forceinline__ void resolve_finish(const InflateArgs& A, uint32_t round, uint32_t sid, uint32_t flag, bool fin0,
                                               bool gz, uint64_t pos0, uint64_t pos, const uint64_t* chainp,
                                               const uint32_t* failp, const uint8_t* ring, uint32_t accS, uint64_t accT,
                                               uint64_t* red) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    RSave* R = (RSave*)A.rsave + sid;
    DSave* S = (DSave*)A.dsave + sid;
    // combine the adler partials of this round
    __syncthreads();
    const uint32_t fail = *(const volatile uint32_t*)failp;
    if (chainp) pos = pos0 + (uint64_t)(uint32_t)*(const volatile uint64_t*)chainp;   // end of the last group
    const bool failed = fail != 0 || (round && R->ck != 0);   // sticky across rounds
    uint32_t S_all = 0, T_all = 0;
    if (!gz) {
        uint64_t a = accS, b = accT;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) { a += __shfl_xor(a, o); b += __shfl_xor(b, o); }
        if (lane == 0) { red[2 * w] = a; red[2 * w + 1] = b; }
        __syncthreads();
        uint64_t tS = round ? R->s1 : 0, tT = round ? R->s2 : 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) { tS += mod65521(red[2 * q]); tT += mod65521(red[2 * q + 1]); }
        S_all = mod65521(tS);
        T_all = mod65521(tT);
    }
    __syncthreads();                                     // R->s1 / s2 were read above
    if (tid == 0) { R->pos = pos; R->s1 = S_all; R->s2 = T_all; R->ck = failed ? 1 : 0; }
    const bool fin = flag == 1 || flag == 3 || fin0;    // the stream's last round of this call
    if (!fin) return;
    const uint64_t bitpos = S->bitpos;
    const uint64_t ilen = A.in_len[sid];
    uint32_t carry_n = 0;
    uint64_t keep_end = 0;
    bool carry_over = false;
    if (A.streaming && flag == 3) {
        // stalled: keep the window (the 32 KiB before the next call's output) and the input
        // from the unit in progress on (the bits the reference holds in its bit buffer)
        uint8_t* win = A.window + (uint64_t)sid * IS_WIN;
        const uint32_t wb = (uint32_t)((pos % RR + RR - RS_WIN) % RR);   // ring index of pos - 32 KiB
        for (uint32_t k = tid; k < RS_WIN; k += 64 * NW) win[k] = ring[(wb + k) % RR];
        // out of input: all of it from the unit's first byte; out of room: only the carried
        // bytes -- the caller passes its own unconsumed bytes again (from in_used on)
        const uint64_t cb = bitpos >> 3;
        const uint64_t nc = R->carry_len;
        keep_end = S->stall == 2 ? (cb > nc ? cb : nc) : ilen;
        carry_n = (uint32_t)(keep_end - cb);
        carry_over = keep_end - cb > SDZ_INFLATE_CARRY;
        if (!carry_over) {
            const uint8_t* src = A.in + A.in_off[sid] + cb;
            uint8_t* dst = A.carry + (uint64_t)sid * SDZ_INFLATE_CARRY;
            for (uint32_t k = tid; k < carry_n; k += 64 * NW) dst[k] = src[k];
        }
    }
    // Inflater.checksum (sd-inflate.ts:136-146): adler32 over 16 KiB output chunks counted
    // from the start of each append()'s output (abase), with the NMAX quirk (adler32.ts:67):
    // a final chunk of 5552 or 11104 bytes leaves sum2 unreduced.  Every other chunk ends
    // reduced, so the value is the plain adler32 state except after such a chunk, which is
    // replayed from the state at its start -- recovered from the plain state at its end and
    // its bytes (the last <= 11104 output bytes are in the ring).
    const bool cont_next = A.streaming && flag == 3 && S->stall == 2;   // this append continues
    const uint64_t T0 = A.streaming ? R->total : 0, T1 = T0 + pos;
    const uint64_t abase = A.streaming ? R->abase : 0;
    const uint32_t rr = (uint32_t)((T1 - abase) & 16383u);
    const bool quirk = !gz && !failed && !cont_next && (rr == 5552u || rr == 11104u);
    uint64_t qa = 0, qb = 0;                              // sum b_j, sum (rr - j) b_j of that chunk
    if (quirk) {
        for (uint32_t k = tid; k < rr; k += 64 * NW) {
            const uint32_t v = ring[ridx64<RR>((int64_t)pos - rr + k)];
            qa += v;
            qb += (uint64_t)(rr - k) * v;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) { qa += __shfl_xor(qa, o); qb += __shfl_xor(qb, o); }
        if (lane == 0) { red[2 * w] = qa; red[2 * w + 1] = qb; }
        __syncthreads();
        qa = 0; qb = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) { qa += red[2 * q]; qb += red[2 * q + 1]; }
    }
    __syncthreads();                                      // window / carry copies done
    if (tid != 0) return;
    if (carry_over) { S->mode = LM_DONE; S->status = SDZ_CARRY_OVERFLOW; S->zmsg = 0; }
    // final: record + verdicts (sd-inflate.ts:134-179); gzip's crc32 comes from k_inflate_finalize
    sdz_inflate_record Rc;
    Rc.status = failed ? SDZ_INTERNAL : S->status;
    Rc.zmsg = failed ? (int32_t)fail : S->zmsg;      // watchdog: site | position << 4
    Rc.out_len = pos;
    uint64_t used = (bitpos + 7) >> 3;
    if (used > ilen) used = ilen;
    // incremental: the stream offset up to which input is consumed or held by the device
    Rc.in_used = A.streaming ? R->in_base + (flag == 3 && !carry_over ? keep_end : used) : used;
    Rc.stored_checksum = S->stored_ck;
    const uint64_t total = T1;
    bool have = total > 0;                                // Inflater.checksum stays undefined otherwise
    int32_t running = 0;
    uint32_t a1 = A.streaming ? R->a1 : 1u, a2 = A.streaming ? R->a2 : 0u;   // state at T0 (exact)
    if (!gz) {
        if (pos) {                                        // no output keeps the exact (quirky) state
            const uint32_t nm = mod65521(pos);
            const uint32_t b1 = (uint32_t)(((uint64_t)a1 + S_all) % 65521u);
            const uint32_t b2 = (uint32_t)(((uint64_t)a2 + (uint64_t)nm * a1 + (uint64_t)nm * S_all +
                                            65521ull * 65521ull - T_all) % 65521u);
            a1 = b1;
            a2 = b2;
        }
        if (quirk) {
            uint32_t s1s, s2s;                            // state at the final chunk's start
            if (T1 - rr == abase) {
                s1s = A.streaming ? R->a1s : 1u;
                s2s = A.streaming ? R->a2s : 0u;
            } else {
                s1s = (uint32_t)((a1 + 65521u - mod65521(qa)) % 65521u);
                s2s = (uint32_t)(((uint64_t)a2 + 65521ull * 65521ull - (uint64_t)rr * s1s - mod65521(qb)) % 65521u);
            }
            running = adler_quirk_ring<RR>(ring, (int64_t)pos - rr, rr, s1s, s2s);
        } else {
            running = (int32_t)(a1 | (a2 << 16));
        }
    }
    Rc.running_checksum = have ? running : 0;
    Rc.stored_size = S->stored_size;
    Rc.mtime = S->mtime;
    Rc.name_off = S->name_off;
    Rc.name_len = S->name_len;
    Rc.container = (uint8_t)S->container;
    bool complete = !failed && S->mode == LM_DONE && (S->status == SDZ_OK || S->status == SDZ_TRAILING);
    Rc.complete = complete ? 1 : 0;
    uint8_t cv = S->stored_ck == 0 ? SDZ_UNCHECKED : ((have && S->stored_ck == running) ? SDZ_MATCH : SDZ_MISMATCH);
    uint8_t sv = S->stored_size == 0 ? SDZ_UNCHECKED
               : ((int64_t)S->stored_size == (int64_t)total ? SDZ_MATCH : SDZ_MISMATCH);
    Rc.checksum_verdict = cv;
    Rc.size_verdict = sv;
    Rc.success = (complete && cv != SDZ_MISMATCH && sv != SDZ_MISMATCH) ? 1 : 0;
    Rc.out_full = S->mode != LM_DONE && S->stall == 2 ? 1 : 0;
    if (!complete && Rc.status == SDZ_OK) Rc.status = SDZ_TRUNCATED;   // incremental: needs more input
    for (int k = 0; k < 10; ++k) Rc.reserved[k] = 0;
    A.rec[sid] = Rc;
    if (A.streaming) {                                    // state for the next call
        R->total = total;
        if (!gz && have) { R->a1 = (uint32_t)running & 0xffffu; R->a2 = (uint32_t)running >> 16; }
        if (flag == 3 && !carry_over) {
            R->in_base += bitpos >> 3;
            R->carry_len = carry_n;
            R->hist = 1;
            S->bitpos = bitpos & 7;
        } else {
            R->carry_len = 0;
        }
    }
}

// One write-back chunk of the writer (or finisher) wave: output bytes [ab, ab + m) from ring index Wr
// to HBM as coalesced dwords (an output-aligned KiB as 4 full dwords per lane), folded into the
// lane's adler32 sums; gm = ab mod 65521.
__device__ __forceinline__ void rs_write_chunk(uint8_t* out, const uint32_t* ring32, bool gz, uint64_t ab, uint32_t m,
                                               uint32_t Wr, uint32_t gm, uint32_t& accS, uint64_t& accT) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t h = (uint32_t)(ab & 3u);
    const uint32_t gi0 = gm + 65521u - h;                // index of byte 0 of dword 0, mod 65521 (+ 65521)
    if (m == 1024u) {
        uint32_t* dstw = (uint32_t*)(out + ab);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t q = lane + 64u * k;
            const uint32_t v = ring32[ridx((int32_t)Wr + 4 * (int32_t)q) >> 2];
            dstw[q] = v;
            if (!gz) {
                const uint32_t s4 = __builtin_amdgcn_udot4(v, 0x01010101u, 0u, false);
                accS += s4;
                accT += (uint64_t)(gi0 + 4 * q) * s4 + __builtin_amdgcn_udot4(v, 0x03020100u, 0u, false);
            }
        }
    } else {
        const uint32_t nq = (uint32_t)(((ab + m + 3u) >> 2) - (ab >> 2));
        uint32_t* dstw = (uint32_t*)(out + (ab - h));
        const int32_t rb0 = (int32_t)Wr - (int32_t)h;    // ring index of the first dword (4-aligned)
        const uint32_t tl = (uint32_t)((ab + m) & 3u);
        for (uint32_t q = lane; q < nq; q += 64) {
            const uint32_t v = ring32[ridx(rb0 + 4 * (int32_t)q) >> 2];
            const uint32_t blo = q == 0 ? h : 0u;
            const uint32_t bhi = q + 1 < nq || tl == 0 ? 4u : tl;
            if (blo == 0 && bhi == 4) dstw[q] = v;
            else for (uint32_t bb = blo; bb < bhi; ++bb) ((uint8_t*)(dstw + q))[bb] = (uint8_t)(v >> (8 * bb));
            if (!gz) {
                const uint32_t mk = (bhi == 4u ? ~0u : (1u << (8 * bhi)) - 1u) & (~0u << (8 * blo));
                const uint32_t vm = v & mk;
                const uint32_t s4 = __builtin_amdgcn_udot4(vm, 0x01010101u, 0u, false);
                accS += s4;
                accT += (uint64_t)(gi0 + 4 * q) * s4 + __builtin_amdgcn_udot4(vm, 0x03020100u, 0u, false);
            }
        }
    }
}

__global__ __launch_bounds__(RS_THREADS) __attribute__((amdgpu_waves_per_eu(RS_WPE, RS_WPE))) void k_inflate_resolve(InflateArgs A, uint32_t round) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[RS_R + 256];   // + per-lane dummies
    __shared__ uint64_t chain;                           // (tag of the last started group) << 32 | its end
    __shared__ uint32_t wf, wwb, fail, edone;            // frontiers: final bytes, written-back bytes; emitters done
    __shared__ __attribute__((aligned(16))) uint8_t fmap[RS_BM];   // finality map of the bytes in flight

    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    const uint32_t sid = blockIdx.x;
    if (sid >= A.n) return;
    const uint32_t flag = A.flags[sid];
    // incremental mode: a stream that finished in an earlier call still gets its record
    const bool fin0 = A.streaming && round == 0 && flag == 2;
    if (flag == 2 && !fin0) return;
    RSave* R = (RSave*)A.rsave + sid;
    DSave* S = (DSave*)A.dsave + sid;
    const bool gz = S->container == SDZ_CONTAINER_GZIP;
    const uint64_t pos0 = round == 0 ? 0 : R->pos;
    uint8_t* out = A.out + A.out_off[sid];
    const uint32_t* tk = A.tokens + (uint64_t)sid * A.round_tokens;
    const uint32_t ntok = A.ntok[sid];
    const int64_t dl = S->dict_used && A.dict ? (A.dict_len > 32767 ? 32767 : A.dict_len) : 0;
    const uint8_t* dict = dl ? A.dict + (A.dict_len - dl) : nullptr;

    const uint32_t rp0 = (uint32_t)(pos0 % RS_R);
    const uint32_t pm0 = (uint32_t)(pos0 % 65521u);
    ring_window_init<RS_R, RS_THREADS>(ring, A, sid, round, pos0, out, dl, dict);
    if (tid == 0) { chain = 0xffffffff00000000ull; wf = 0; wwb = 0; fail = 0; edone = 0; }
    for (uint32_t k = tid; k < RS_BM / 4; k += RS_THREADS) ((uint32_t*)fmap)[k] = 0;
    __syncthreads();

    // adler32 as sums over the whole output: s1 = 1 + S, s2 = n + n S - T (mod 65521),
    // S = sum b_i, T = sum i b_i -- per-lane partials, combined once per round
    uint32_t accS = 0;
    uint64_t accT = 0;                                    // < 2^47 per lane and round: reduced once at the end
#ifdef SDZ_TIMING
    const bool timed = A.dbg && sid < 8 && lane == 0;
#else
    const bool timed = false;
#endif
    unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tlast = timed ? clock64() : 0;
#define RS_TICK(k) do { if (timed) { unsigned long long tn = clock64(); tacc[k] += tn - tlast; tlast = tn; } } while (0)
    const uint32_t ngroups = (ntok + 63u) >> 6;
    // Control flow below is kept wave-uniform (values read from LDS go through
    // readfirstlane, lane predicates are selects): the scalar unit, shared by the CU's
    // four SIMDs, is the busiest resource of this kernel (an extra SALU per copy round
    // costs ~3 SIMD cycles, measured), so divergent ifs and their exec-mask juggling
    // are avoided on the hot path.  `fail` is polled once per 64 waits only.
    const uint32_t wu = uni(w);
    const uint32_t g32 = (uint32_t)pos0;
    // emitter waves: no global stores, so the token prefetch is their only vector-memory
    // traffic and its wait does not cover write-back stores
    uint32_t tnext = tk[wu * 64u + lane < ntok ? wu * 64u + lane : 0u];
    bool bad = false;                                     // this wave's watchdog tripped
    for (uint32_t g = wu; wu < RS_EW && g < ngroups; g += RS_EW) {
        const uint32_t ti = g * 64u + lane;
        const bool valid = ti < ntok;
        const uint32_t t = tnext;
        tnext = tk[ti + 64u * RS_EW < ntok ? ti + 64u * RS_EW : 0u];
        const bool ism = (int32_t)t < 0;
        const uint32_t len = !valid ? 0u : ism ? ((t >> 16) & 255u) + 3u : ((t >> 24) & 3u) + 1u;
        const uint32_t dist = ism ? (t & 0x7fffu) + 1u : 0u;
        const uint32_t incl = wave_incl_scan(len);
        const uint32_t T = lane_at(incl, 63);
        const uint32_t off = incl - len;
        RS_TICK(0);

        // 1. the group's start from its predecessor; pass ours on
        uint32_t Sg = 0;
        for (uint32_t n = 1;; ++n) {
            const uint64_t c = lds_get64(&chain);
            if (uni((uint32_t)(c >> 32)) == g - 1u) { Sg = uni((uint32_t)c); break; }
            if ((n & 63u) == 0 && (n > RS_SPIN_LIMIT || lds_get(&fail))) {
                if (!lds_get(&fail)) lds_put(&fail, 1u | (g << 4));
                bad = true;
                break;
            }
            __builtin_amdgcn_s_sleep(RS_NAP);
        }
        if (bad) break;
        if (lane == 0) __hip_atomic_store(&chain, ((uint64_t)g << 32) | (Sg + T), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
        rs_wake();
        RS_TICK(1);

        // 2. copy rounds
        const uint32_t sr = uni((rp0 + Sg) % RS_R);                    // ring index of byte Sg (u32: Sg < 2^26)
        const uint32_t dst = Sg + off, dend = dst + len;
        const int32_t src = (int32_t)dst - (int32_t)dist;             // round-relative (may be < 0)
        const int32_t need = ism ? src + (int32_t)(len < dist ? len : dist) : INT32_MIN;
        const uint32_t d = ridx((int32_t)(sr + off));
        const uint32_t s = ridx((int32_t)(sr + off) - (int32_t)dist);
        const uint32_t gd = (uint32_t)pos0 + dst;                       // low bits of the global position
        const uint32_t mp = gd & (RS_BM - 1), lb = lap_of(gd);
        bool done = len == 0;
        uint64_t nd = __ballot(!done);
        for (uint32_t n = 1; nd; ++n) {
            const uint32_t pre = lane_at(off, (uint32_t)__builtin_ctzll(nd));   // finished prefix
            uint32_t cwf = lds_get(&wf);
            const uint32_t cwb = lds_get(&wwb);
            if (cwf >= Sg && cwf < Sg + pre) {            // head: publish our finished prefix
                publish_wf(&wf, Sg + pre);
                cwf = Sg + pre;
            }
            const bool room = !done && dend <= cwf + RS_SLACK && dend <= cwb + RS_R;
            const bool inwin = need <= (int32_t)cwf;
            const uint32_t blo = src > (int32_t)cwf ? (uint32_t)src : cwf;
            const bool chk = room && !inwin;
            bool ok = true;
            if (__ballot(chk)) ok = map_all(fmap, chk, g32 + blo, g32 + (uint32_t)need);
#ifdef RS_ABL_ONE
            const bool rdy = room;                        // development: sources never waited for (output wrong)
#else
            const bool rdy = room && (inwin || ok);
#endif
            const uint64_t rm = __ballot(rdy);
            if (rm) {
                RS_CBAR();
                emit_msk<RS_R, true, RS_MW>(ring, fmap, rdy, t, d, s, len, dist, mp, lb);
                done = done || rdy;
                nd &= ~rm;
                n = 0;
                if (timed) tacc[6]++;
            } else {
                if (timed) tacc[7]++;
                if ((n & 63u) == 0 && (n > RS_SPIN_LIMIT || lds_get(&fail))) {
                    if (!lds_get(&fail)) lds_put(&fail, 3u | (Sg << 4));
                    bad = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(RS_NAP);
            }
        }
        if (bad) break;
        RS_TICK(2);
        // 3. finality, in group order: publish now if we are the head (no one else can
        // move wf past Sg), else once the frontier reaches us
        for (uint32_t n = 1;; ++n) {
            if (lds_get(&wf) >= Sg) { lds_acquire(); break; }
            if ((n & 63u) == 0 && (n > RS_SPIN_LIMIT || lds_get(&fail))) {
                if (!lds_get(&fail)) lds_put(&fail, 2u | (Sg << 4));
                bad = true;
                break;
            }
            __builtin_amdgcn_s_sleep(RS_NAP);
        }
        if (bad) break;
        publish_wf(&wf, Sg + T);
        RS_TICK(4);
    }
    const uint32_t* ring32 = (const uint32_t*)ring;
    if (wu < RS_EW) {
        lds_release();
        if (lane == 0) __hip_atomic_fetch_add(&edone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
        // the writer wave: final bytes -> HBM in output-aligned 1 KiB chunks, folded into the
        // adler32 sums; publishes wwb, which frees ring slots
        uint32_t WB = 0, Wr = rp0, gm = pm0;              // written back (round-relative), its ring index, (pos0 + WB) mod 65521
        for (uint32_t n = 1;; ++n) {
            const bool fi = lds_get(&edone) == RS_EW;     // every group published: wf is the round's end
            lds_acquire();
            const uint32_t Fv = lds_get(&wf);
            const uint64_t ab = pos0 + WB;
            const uint32_t nk = 1024u - (uint32_t)(ab & 1023u);
            uint32_t m;
            if (Fv - WB >= nk) m = nk;
            else if (fi) {
                if (Fv == WB) break;
                m = Fv - WB;
            } else {
                if ((n & 63u) == 0 && (n > RS_SPIN_LIMIT || lds_get(&fail))) {
                    if (!lds_get(&fail)) lds_put(&fail, 4u | (WB << 4));
                    break;
                }
                __builtin_amdgcn_s_sleep(RS_NAP);
                continue;
            }
            n = 0;
            rs_write_chunk(out, ring32, gz, ab, m, Wr, gm, accS, accT);
            WB += m;
            Wr += m;
            Wr -= Wr >= RS_R ? RS_R : 0u;
            gm += m;
            gm -= gm >= 65521u ? 65521u : 0u;
            lds_release();                                // our ring reads are complete
            if (lane == 0) lds_put(&wwb, WB);
            rs_wake();
        }
    }
    if (timed) for (int k = 0; k < 8; ++k) atomicAdd(&A.dbg[k], tacc[k]);

    // (the adler partials' reduction reuses the finality map, which no one reads any more)
    resolve_finish<RS_R, RS_WAVES>(A, round, sid, flag, fin0, gz, pos0, 0, &chain, &fail, ring, accS, accT, (uint64_t*)fmap);
}

// ------------------------------------------------------------------ gzip: crc32 + verdicts

// one wave per finished gzip stream: crc32 of its output (crc32_dev.h) and the checksum
// verdicts that depend on it
// Long outputs are cut into chunks whose crc32 k_gzip_crc_parts computes one block each (4
// waves, 64 lanes each over a quarter); k_inflate_finalize chains them in order with x^(8 n)
// shifts (crc32 of a concatenation).  parts[sid * maxc + c]: chunk c of stream sid.
__global__ __launch_bounds__(256) void k_gzip_crc_parts(InflateArgs A, uint64_t chunk, uint32_t maxc, uint32_t* parts) {
    __shared__ CrcTables ct;
    __shared__ uint32_t wc[4];
    const uint32_t sid = blockIdx.y, c = blockIdx.x;
    if (sid >= A.n) return;
    const sdz_inflate_record* rec = A.rec + sid;
    const uint64_t len = rec->out_len;
    if (rec->container != SDZ_CONTAINER_GZIP || len <= chunk || (uint64_t)c * chunk >= len) return;
    crc_tables_init(ct);
    __syncthreads();
    const uint64_t a = (uint64_t)c * chunk, n = len - a < chunk ? len - a : chunk;
    const uint64_t q = ((n + 3) / 4 + 7) & ~7ull;        // a quarter per wave (8-byte multiples)
    const uint32_t w = threadIdx.x >> 6;
    const uint64_t b0 = (uint64_t)w * q < n ? (uint64_t)w * q : n, b1 = b0 + q < n ? b0 + q : n;
    const uint32_t cr = crc32_wave(A.out + A.out_off[sid] + a + b0, b1 - b0, ct);
    if ((threadIdx.x & 63u) == 0) wc[w] = cr;
    __syncthreads();
    if (threadIdx.x != 0) return;
    uint32_t crc = 0;
    for (uint32_t k = 0; k < 4; ++k) {
        const uint64_t lo = (uint64_t)k * q < n ? (uint64_t)k * q : n, hi = lo + q < n ? lo + q : n;
        crc = gf2_mulmod(gf2_xbytes(hi - lo, ct.x2n), crc) ^ wc[k];
    }
    parts[(uint64_t)sid * maxc + c] = crc;
}

__global__ __launch_bounds__(64) void k_inflate_finalize(InflateArgs A, uint64_t chunk, uint32_t maxc,
                                                         const uint32_t* parts) {
    __shared__ CrcTables ct;
    const uint32_t sid = blockIdx.x;
    if (sid >= A.n) return;
    sdz_inflate_record* rec = A.rec + sid;
    if (rec->container != SDZ_CONTAINER_GZIP) return;    // block-uniform: no table build for zlib / raw
    crc_tables_init(ct);
    __syncthreads();
    const uint64_t len = rec->out_len;
    uint32_t crc = 0;
    if (len <= chunk) {
        crc = crc32_wave(A.out + A.out_off[sid], len, ct);
        if (threadIdx.x != 0) return;
    } else {
        if (threadIdx.x != 0) return;
        for (uint64_t a = 0, c = 0; a < len; a += chunk, ++c) {
            const uint64_t n = len - a < chunk ? len - a : chunk;
            crc = gf2_mulmod(gf2_xbytes(n, ct.x2n), crc) ^ parts[(uint64_t)sid * maxc + c];
        }
    }
    RSave* R = (RSave*)A.rsave + sid;
    bool have = len > 0;
    if (A.streaming) {
        // crc32(chunk, seed) chains: crc(A B) = crc(A) x^(8 |B|) + crc(B) mod P
        crc = gf2_mulmod(gf2_xbytes(len, ct.x2n), R->crc) ^ crc;
        R->crc = crc;
        have = R->total > 0;
    }
    const int32_t running = (int32_t)crc;
    rec->running_checksum = have ? running : 0;
    const uint8_t cv = rec->stored_checksum == 0 ? SDZ_UNCHECKED
                     : ((have && rec->stored_checksum == running) ? SDZ_MATCH : SDZ_MISMATCH);
    rec->checksum_verdict = cv;
    rec->success = (rec->complete && cv != SDZ_MISMATCH && rec->size_verdict != SDZ_MISMATCH) ? 1 : 0;
}

uint32_t resolve_block_threads() { return RS_THREADS; }
uint32_t resolve_streams_per_block() { return 1; }
void launch_inflate_resolve(const InflateArgs& a, uint32_t round, dim3 grid, hipStream_t s) {
    hipLaunchKernelGGL(k_inflate_resolve, grid, dim3(RS_THREADS), 0, s, a, round);
}
// parts: scratch for the chunk crcs (a.tokens: the token rings are free once the rounds are
// done; >= 1024 entries per stream); chunks of >= 256 KiB, <= 1024 per stream and <= 4 Mi
// blocks in all
void launch_inflate_finalize(const InflateArgs& a, hipStream_t s) {
    uint64_t mx = 0;
    uint64_t chunk = 256 << 10;
    uint32_t maxc = 1;
    unsigned long long* slot = (unsigned long long*)a.tokens;
    uint32_t* parts = a.tokens + 64;
    // the largest output slot sizes the chunked crc32 grid: from the host when it has the slots
    // (no device read and wait), else one device reduction
    const bool known = a.host_cap_max != 0;
    if (known) mx = a.host_cap_max;
    if ((known || device_max_u64(a.out_cap, a.n, slot, &mx, s) == 0) && mx > chunk) {
        uint64_t c = (mx + chunk - 1) / chunk;
        const uint64_t lim = std::min<uint64_t>(1024, std::max<uint64_t>(1, (4ull << 20) / a.n));
        if (c > lim) { c = lim; chunk = ((mx + c - 1) / c + 7) & ~7ull; }
        maxc = (uint32_t)c;
        if ((uint64_t)maxc * a.n + 64 <= (uint64_t)a.round_tokens * a.n)
            hipLaunchKernelGGL(k_gzip_crc_parts, dim3(maxc, a.n), dim3(256), 0, s, a, chunk, maxc, parts);
        else
            chunk = ~0ull;                               // (no room: one wave per stream)
    }
    hipLaunchKernelGGL(k_inflate_finalize, dim3(a.n), dim3(64), 0, s, a, chunk, maxc, (const uint32_t*)parts);
}

}  // namespace sdz
