// k_inflate.hip -- batched DEFLATE decoder for gfx950 (MI355X), phase 1 + round driver.
//
// Replaces the serial hot path of @stardazed/zlib's inflate:
//   Inflate.inflate container FSM   src/inflate.ts:132-473
//   InfBlocks.proc block FSM        src/infblocks.ts:123-628
//   InfCodes inflate_fast / proc    src/infcodes.ts:62-676
//   huft_build + tree builders      src/inftree.ts:95-392
//   Inflater.append/finish verdicts src/sd-inflate.ts:87-179 (finished in k_resolve.hip)
//
// Two phases per round:
//  PHASE 1  k_inflate_decode (this file) -- one LANE per stream.  Huffman decoding is
//    serial per stream, so a wave decodes 64 streams in lock-step.  Decoding is
//    table-free in registers: the 15 left-justified limits of a tree are compared
//    with the 15 bit-reversed peek bits and a depth-4 select tree picks a packed
//    per-length word (rank offset, literal threshold, shift).  Only the rank->symbol
//    bytes live in LDS (324 B/stream).  The lane emits 32-bit tokens (up to 3
//    literals, or a length/distance pair), staged in LDS and flushed to HBM as
//    128-byte lines.  No window reads, no output writes.
//  PHASE 2  k_inflate_resolve (k_resolve.hip) -- turns the tokens into bytes.
// The host runs rounds (phase 1 fills up to T tokens per stream, phase 2 drains
// them) until every stream is finished.
//
// Reference quirks mirrored: root-bits "need" at end of
// input (infcodes.ts:368-387), huft_build's MANY=1400 table budget, incomplete
// single-code trees, the gzip FEXTRA mode that never advances (inflate.ts:343-345).
#include <vector>
#include "inflate_state.h"
#include <type_traits>

namespace sdz {

// IL_STREAMS streams per workgroup, IL_WAVE_LANES of them per wave: with 32, a workgroup
// has twice the waves, each with half its lanes active -- the same streams and LDS per CU,
// two instruction streams per SIMD to hide each other's latency
#ifndef IL_WAVE_LANES
#define IL_WAVE_LANES 64
#endif
#define IL_STREAMS 256
#ifndef IL_STOP_SHIFT
#define IL_STOP_SHIFT 0               // a hot epoch runs until every lane needs block-level work
                                      // (since cold_run is inlined: distinct decode 11.25 -> 11.09 ms;
                                      // 1, half the lanes, and 2, a quarter: 11.25 / 11.41 ms; C2 equal)
                                      // (1/8: 4 % slower on distinct streams, C2 equal)
#endif
#define IL_THREADS (IL_STREAMS * 64 / IL_WAVE_LANES)
#define IL_TSTAGE 32                  // tokens staged in LDS per stream (one 128 B line)
#ifndef IL_UNIFORM_FLUSH
#define IL_UNIFORM_FLUSH 1            // the symbol loop writes staged tokens at its ring step
#endif
#define IL_TSTRIDE 136                // LDS bytes per stream for the token stage (8-aligned)
#define IL_BAD_IDX 300                // rank selected by codes past lim[15]
#ifndef IL_PEEK_PAR
#define IL_PEEK_PAR 1                 // peek from the pre-refill words beside the refill's compare
#endif

// LDS: per-stream symbol tables, then per-stream token stages (file scope, so the
// non-inlined hot and cold functions address it as LDS, not through flat pointers)
__device__ __forceinline__ uint32_t lane_slot() {   // this lane's stream slot in the workgroup
    return IL_WAVE_LANES == 64 ? threadIdx.x : (threadIdx.x >> 6) * IL_WAVE_LANES + (threadIdx.x & (IL_WAVE_LANES - 1));
}
__shared__ __attribute__((aligned(16))) uint8_t g_region[IL_STREAMS * IL_REGION];
__shared__ __attribute__((aligned(16))) uint32_t g_stage[IL_STREAMS * (IL_TSTRIDE / 4)];
__device__ __forceinline__ uint8_t* lane_region() { return g_region + lane_slot() * IL_REGION; }
#ifndef IL_REFILL2
#define IL_REFILL2 1                  // symbol loop: one refill of up to 2 dwords per step (br_refill2)
#endif
#ifndef IL_RING32
#define IL_RING32 1                   // ... its ring step loads 32 B at a time (ring_step2)
#endif
#if IL_REFILL2
#define IL_RING_DW 32                 // input ring dwords per lane (128 B + 8 B pad)
#else
#define IL_RING_DW 16                 // (64 B + 8 B pad)
#endif
#define IL_RING_STRIDE (IL_RING_DW + 2)
__shared__ __attribute__((aligned(16))) uint32_t g_ring[IL_STREAMS * IL_RING_STRIDE];
__device__ __forceinline__ uint32_t* lane_stage() { return g_stage + lane_slot() * (IL_TSTRIDE / 4); }
__device__ __forceinline__ uint32_t* lane_ring() { return g_ring + lane_slot() * IL_RING_STRIDE; }

__constant__ uint8_t c_border[19] = { 16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15 };

#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(1))) const uint4 g_uint4;   // global_load, not flat_load
#define GLB __attribute__((address_space(1)))
#else
#define GLB
typedef const uint4 g_uint4;
#endif

// decoder state shared by the hot symbol loop and the cold block-level code
struct Core {
    // 64-bit window w1:w0 of which bo bits are consumed (bo < 32 after a refill)
    uint32_t w0, w1, bo;
    int32_t avail;                    // input bits from bit 0 of w0 (saturated at 2^30)
    int32_t avail0;                   // avail when the reader was positioned
    uint64_t base_bit;                // stream bit index of w0's bit 0 at that time
    uint32_t room, room0;             // output bytes still allowed (saturated), at positioning
    uint64_t pos0;                    // output position at positioning
    int mode, last, status, zmsg;
    // token output
    uint32_t* tb;                     // this stream's token ring in HBM
    uint32_t* ts;                     // LDS stage
    uint32_t ntok, tcap;
    uint32_t litw, nlit;
    bool full;
#ifdef IL_HOT_CHECK
    // development: the readable input span and the stream, for bounds checks
    const uint8_t* chk_lo;
    const uint8_t* chk_hi;
    uint32_t chk_id;
#endif
};
// The symbol loop's input: w2 (next dword) is fed from a per-lane 64-byte LDS ring.
// Once per 4 loop iterations -- a wave-uniform point -- each lane commits the 16-32
// bytes it loaded one group earlier and issues the next loads.  Per-lane register
// prefetch would not do: some lane's load would always be in flight into the
// registers every lane reads, and the wave would wait on it at each refill.
struct Hot : Core {
    uint32_t w2, nx;                  // next dword, and the ring dword after it (read ahead)
    uint32_t nx2;                     // (IL_REFILL2) and the one after that
    uint32_t arp;                     // (IL_REFILL2) avail + 8 * rpos: the loop keeps avail implicit
    uint32_t rpos, wpos;              // ring bytes consumed / committed (mod 2^32)
    uint4 s0, s1;                     // loads in flight, committed at the next group
    uint32_t ns;
    uint32_t nfl;                     // tokens in HBM (IL_UNIFORM_FLUSH: a multiple of 16)
    g_uint4* vp;                      // next 16 input bytes to load
    g_uint4* vend;                    // first 16-byte chunk past the input
    uint32_t* ring;
};
#ifdef IL_HOT_CHECK
// a hot-path access outside its bounds: reported once per lane, the access skipped and the
// lane stopped (status BAD_RECORD), so the run ends without a fault
// (one out-of-line report: printf expanded at every inlined check site made the build take hours)
__device__ __noinline__ void hot_check_fail(int what, uint32_t id, unsigned long long a, unsigned long long b,
                                            unsigned long long lo, unsigned long long hi) {
    printf("IL_HOT_CHECK site %d stream %u lane %u: %llx %llx lo %llx hi %llx\n", what, id, threadIdx.x, a, b, lo, hi);
}
#define HOT_CHECK(L, cond, what, a, b)                                                            \
    (!(cond) ? (hot_check_fail(what, (L).chk_id, (unsigned long long)(a), (unsigned long long)(b), \
                               (unsigned long long)(L).chk_lo, (unsigned long long)(L).chk_hi),   \
                (L).mode = LM_DONE, (L).status = SDZ_BAD_RECORD, (L).full = true, false) : true)
#else
#define HOT_CHECK(L, cond, what, a, b) true
#endif
// ... and the cold code: a plain reader plus the block-level state
struct Lane : Core {
    const uint32_t* dp;               // next input dword
    int container, fixed, nl, nd;
    int32_t stored_ck, stored_size, mtime;
    uint32_t name_off, name_len, stored_left;
    int dict_used;
    uint8_t* lens;                    // global scratch for code lengths
    // end of input: one-shot streams end TRUNCATED; incremental ones (streaming) are parked
    // at the start of the unit in progress (ubit) and stall until the next call
    uint64_t ubit;
    int streaming, stall;
};

// ------------------------------------------------------------------ bit reader

__device__ __forceinline__ uint32_t br_peek32(const Core& L) { return __builtin_amdgcn_alignbit(L.w1, L.w0, L.bo); }
__device__ __forceinline__ int32_t br_avail(const Core& L) { return L.avail - (int32_t)L.bo; }
__device__ __forceinline__ uint64_t br_consumed(const Core& L) {
    return L.base_bit + (uint64_t)(int64_t)(L.avail0 - L.avail) + L.bo;
}
__device__ __forceinline__ void br_drop(Core& L, uint32_t n) { L.bo += n; }
__device__ __forceinline__ void br_setavail(Core& L, uint64_t bitpos, uint64_t total_bits) {
    L.base_bit = bitpos - L.bo;
    uint64_t av = total_bits - L.base_bit;
    L.avail = (int32_t)(av > (1ull << 30) ? (1ull << 30) : av);
    L.avail0 = L.avail;
}

__device__ __forceinline__ void br_refill(Lane& L) {
    if (L.bo >= 32) {
        if (!HOT_CHECK(L, (const uint8_t*)L.dp >= L.chk_lo && (const uint8_t*)(L.dp + 1) <= L.chk_hi, 4,
                       (uintptr_t)L.dp, 0)) { L.bo = 0; L.avail = 0; return; }
        L.w0 = L.w1; L.w1 = *L.dp++; L.bo -= 32; L.avail -= 32;
    }
}
// read n <= 24 bits; returns false (stall) if the input does not hold them
__device__ __forceinline__ bool br_get(Lane& L, int n, uint32_t& v) {
    br_refill(L);
    if (br_avail(L) < n) return false;
    v = br_peek32(L) & ((1u << n) - 1u);
    L.bo += (uint32_t)n;
    return true;
}
// position the reader at bit `bitpos` of the stream starting at p
__device__ __forceinline__ void br_init(Lane& L, const uint8_t* p, uint64_t bitpos, uint64_t total_bits) {
    uintptr_t addr = (uintptr_t)(p + (bitpos >> 3));
    L.dp = (const uint32_t*)(addr & ~(uintptr_t)3);
#ifdef IL_HOT_CHECK
    if (!HOT_CHECK(L, bitpos <= total_bits && (const uint8_t*)L.dp >= L.chk_lo && (const uint8_t*)(L.dp + 2) <= L.chk_hi, 7,
                   bitpos, total_bits)) {
        L.dp = (const uint32_t*)L.chk_lo;
        bitpos = 0;
        addr = (uintptr_t)L.chk_lo;
    }
#endif
    L.w0 = L.dp[0];
    L.w1 = L.dp[1];
    L.dp += 2;
    L.bo = (uint32_t)(8 * (addr & 3) + (bitpos & 7));
    br_setavail(L, bitpos, total_bits);
}

// branch-free: the ring dword that becomes w2 was read one refill earlier (nx), and
// the next one is read unconditionally, so no refill waits on an LDS read
__device__ __forceinline__ void br_refill(Hot& L) {
    bool c = L.bo >= 32;
    L.w0 = c ? L.w1 : L.w0;
    L.w1 = c ? L.w2 : L.w1;
    L.w2 = c ? L.nx : L.w2;
    L.rpos += c ? 4u : 0u;
    L.avail -= c ? 32 : 0;
    L.bo &= 31u;
    L.nx = L.ring[(L.rpos >> 2) & 15u];
}
// the refill and the peek after it, with the peek taken from the pre-refill words in parallel
// with the refill's compare (one dependent operation less on the bit position's chain)
__device__ __forceinline__ uint32_t br_refill_peek(Hot& L) {
#if IL_PEEK_PAR
    const bool c = L.bo >= 32;
    const uint32_t pa = __builtin_amdgcn_alignbit(L.w1, L.w0, L.bo);   // alignbit uses bo & 31
    const uint32_t pb = __builtin_amdgcn_alignbit(L.w2, L.w1, L.bo);
    br_refill(L);
    return c ? pb : pa;
#else
    br_refill(L);
    return br_peek32(L);
#endif
}
__device__ __forceinline__ void tok_flush_hot(Hot& L);
// the wave-uniform ring step (see struct Hot); keeps >= 24 bytes in the ring,
// enough for the 4 iterations of up to 48 bits each that follow
__device__ __forceinline__ void ring_step(Hot& L) {
    if (L.ns) {
        uint32_t k = (L.wpos >> 2) & 15u;
        *(uint2*)(L.ring + k) = make_uint2(L.s0.x, L.s0.y);
        *(uint2*)(L.ring + k + 2) = make_uint2(L.s0.z, L.s0.w);
        L.wpos += 16;
        if (L.ns == 2) {
            k = (L.wpos >> 2) & 15u;
            *(uint2*)(L.ring + k) = make_uint2(L.s1.x, L.s1.y);
            *(uint2*)(L.ring + k + 2) = make_uint2(L.s1.z, L.s1.w);
            L.wpos += 16;
        }
        L.ns = 0;
    }
#if !IL_FLUSH_LATE
    tok_flush_hot(L);
#endif
    uint32_t lvl = L.wpos - L.rpos;
    if (lvl <= 48 && L.vp < L.vend) {
        if (!HOT_CHECK(L, (const uint8_t*)L.vp >= L.chk_lo && (const uint8_t*)(L.vp + 2) <= L.chk_hi, 1,
                       (uintptr_t)L.vp, (uintptr_t)L.vend)) return;
        L.s0 = *L.vp++;
        L.ns = 1;
        if (lvl <= 32 && L.vp < L.vend) { L.s1 = *L.vp++; L.ns = 2; }
    }
#if IL_FLUSH_LATE
    tok_flush_hot(L);
#endif
}
// the same ring step for the wave decoder (k_inflate_wdec), whose tokens have their own stage
__device__ __forceinline__ void ring_step_wd(Hot& L) {
    if (L.ns) {
        uint32_t k = (L.wpos >> 2) & 15u;
        *(uint2*)(L.ring + k) = make_uint2(L.s0.x, L.s0.y);
        *(uint2*)(L.ring + k + 2) = make_uint2(L.s0.z, L.s0.w);
        L.wpos += 16;
        if (L.ns == 2) {
            k = (L.wpos >> 2) & 15u;
            *(uint2*)(L.ring + k) = make_uint2(L.s1.x, L.s1.y);
            *(uint2*)(L.ring + k + 2) = make_uint2(L.s1.z, L.s1.w);
            L.wpos += 16;
        }
        L.ns = 0;
    }
    uint32_t lvl = L.wpos - L.rpos;
    if (lvl <= 48 && L.vp < L.vend) {
        L.s0 = *L.vp++;
        L.ns = 1;
        if (lvl <= 32 && L.vp < L.vend) { L.s1 = *L.vp++; L.ns = 2; }
    }
}
__device__ __forceinline__ void br_init(Hot& L, const uint8_t* p, uint64_t bitpos, uint64_t total_bits,
                                        uint32_t* ring) {
    uintptr_t addr = (uintptr_t)(p + (bitpos >> 3));
    g_uint4* vp = (g_uint4*)(addr & ~(uintptr_t)15);
    uint4 c0 = vp[0], c1 = vp[1], c2 = vp[2], c3 = vp[3];
    L.ring = ring;
    // ring rows are 8-byte aligned (72-byte stride): written as pairs of uint2
    *(uint2*)(ring + 0) = make_uint2(c0.x, c0.y); *(uint2*)(ring + 2) = make_uint2(c0.z, c0.w);
    *(uint2*)(ring + 4) = make_uint2(c1.x, c1.y); *(uint2*)(ring + 6) = make_uint2(c1.z, c1.w);
    *(uint2*)(ring + 8) = make_uint2(c2.x, c2.y); *(uint2*)(ring + 10) = make_uint2(c2.z, c2.w);
    *(uint2*)(ring + 12) = make_uint2(c3.x, c3.y); *(uint2*)(ring + 14) = make_uint2(c3.z, c3.w);
    L.vp = vp + 4;
    L.wpos = 64;
    uint32_t k = (uint32_t)((addr >> 2) & 3);
    L.w0 = ring[k];
    L.w1 = ring[k + 1];
    L.w2 = ring[k + 2];
    L.nx = ring[k + 3];
    L.rpos = 4 * (k + 3);
    L.ns = 0;
    L.bo = (uint32_t)(8 * (addr & 3) + (bitpos & 7));
    br_setavail(L, bitpos, total_bits);
}

#if IL_REFILL2
// The lane decoder's reader (IL_REFILL2): a step refills once, by 0, 1 or 2 dwords, and takes a
// 64-bit peek, so that a length code's distance code is read from the same peek instead of after
// a second refill.  The ring (32 dwords) holds two read-ahead dwords (nx, nx2).  Invariant: at a
// ring step, after its commit, lvl = wpos - rpos >= 32 bytes, so every read-ahead of the next 4
// steps (at most 6 dwords of advance, + nx2) reads committed bytes: with loads of 32 B at lvl <= 64
// and 16 B at lvl <= 96, committed one ring step later, lvl drops by at most 24 B per 4 steps.
__device__ __forceinline__ void br_init2(Hot& L, const uint8_t* p, uint64_t bitpos, uint64_t total_bits,
                                         uint32_t* ring) {
    uintptr_t addr = (uintptr_t)(p + (bitpos >> 3));
    g_uint4* vp = (g_uint4*)(addr & ~(uintptr_t)15);
    uint4 c0 = vp[0], c1 = vp[1], c2 = vp[2], c3 = vp[3];
    L.ring = ring;
    *(uint2*)(ring + 0) = make_uint2(c0.x, c0.y); *(uint2*)(ring + 2) = make_uint2(c0.z, c0.w);
    *(uint2*)(ring + 4) = make_uint2(c1.x, c1.y); *(uint2*)(ring + 6) = make_uint2(c1.z, c1.w);
    *(uint2*)(ring + 8) = make_uint2(c2.x, c2.y); *(uint2*)(ring + 10) = make_uint2(c2.z, c2.w);
    *(uint2*)(ring + 12) = make_uint2(c3.x, c3.y); *(uint2*)(ring + 14) = make_uint2(c3.z, c3.w);
    ring[IL_RING_DW] = c0.x;                          // the mirror of dword 0 (see br_refill2)
    L.vp = vp + 4;
    L.wpos = 64;
    uint32_t k = (uint32_t)((addr >> 2) & 3);
    L.w0 = ring[k];
    L.w1 = ring[k + 1];
    L.w2 = ring[k + 2];
    L.nx = ring[k + 3];
    L.nx2 = ring[k + 4];
    L.rpos = 4 * (k + 3);                             // lvl = 64 - rpos >= 40
    L.ns = 0;
    L.bo = (uint32_t)(8 * (addr & 3) + (bitpos & 7));
    br_setavail(L, bitpos, total_bits);
    L.arp = (uint32_t)L.avail + 8u * L.rpos;
}
// input bits from the current position, and the explicit avail the cold code and br_consumed use
__device__ __forceinline__ int32_t br_avail2(const Hot& L) { return (int32_t)(L.arp - 8u * L.rpos) - (int32_t)L.bo; }
__device__ __forceinline__ void br_sync2(Hot& L) { L.avail = (int32_t)(L.arp - 8u * L.rpos); }
// bo < 96 (a step leaves it below 32 + 48)
__device__ __forceinline__ void br_refill2(Hot& L) {
    const uint32_t bo = L.bo;
    const bool c1 = bo >= 32, c2 = bo >= 64;
    const uint32_t w0 = L.w0, w1 = L.w1, w2 = L.w2, nx = L.nx, nx2 = L.nx2;
    L.w0 = c2 ? w2 : (c1 ? w1 : w0);
    L.w1 = c2 ? nx : (c1 ? w2 : w1);
    L.w2 = c2 ? nx2 : (c1 ? nx : w2);
    L.rpos += (bo >> 3) & ~3u;                        // 4 bytes per dword moved in
    L.bo = bo & 31u;
    // nx and nx2 in one ds_read2_b32: dword IL_RING_DW mirrors dword 0
    const uint32_t* q = (const uint32_t*)((const uint8_t*)L.ring + (L.rpos & (4u * IL_RING_DW - 4u)));
    L.nx = q[0];
    L.nx2 = q[1];
}
__device__ __forceinline__ void ring_step2(Hot& L) {
#if IL_RING32
    // loads of 32 B only, at lvl <= 80 (committed one ring step later: lvl stays >= 32 and below
    // 112 + 16); wpos stays a multiple of 32, so only a load's first 16 B can land on dword 0.  The
    // second chunk may lie past the input's last 16-B chunk: inside the 64 readable bytes the C-ABI
    // asks for after a stream (include/sdz.h), and never consumed (the bit count ends before it)
    if (L.ns) {
        const uint32_t k = (L.wpos >> 2) & (IL_RING_DW - 1);
        *(uint2*)(L.ring + k) = make_uint2(L.s0.x, L.s0.y);
        *(uint2*)(L.ring + k + 2) = make_uint2(L.s0.z, L.s0.w);
        *(uint2*)(L.ring + k + 4) = make_uint2(L.s1.x, L.s1.y);
        *(uint2*)(L.ring + k + 6) = make_uint2(L.s1.z, L.s1.w);
        L.ring[k == 0 ? IL_RING_DW : IL_RING_DW + 1] = L.s0.x;   // mirror of dword 0 (else the pad)
        L.wpos += 32;
        L.ns = 0;
    }
    tok_flush_hot(L);
    if (L.wpos - L.rpos <= 80 && L.vp < L.vend) {
        if (!HOT_CHECK(L, (const uint8_t*)L.vp >= L.chk_lo && (const uint8_t*)(L.vp + 2) <= L.chk_hi, 1,
                       (uintptr_t)L.vp, (uintptr_t)L.vend)) return;
        L.s0 = L.vp[0];
        L.s1 = L.vp[1];
        L.vp += 2;
        L.ns = 2;
    }
#else
    if (L.ns) {
        uint32_t k = (L.wpos >> 2) & (IL_RING_DW - 1);
        *(uint2*)(L.ring + k) = make_uint2(L.s0.x, L.s0.y);
        *(uint2*)(L.ring + k + 2) = make_uint2(L.s0.z, L.s0.w);
        L.ring[k == 0 ? IL_RING_DW : IL_RING_DW + 1] = L.s0.x;   // mirror of dword 0 (else the pad)
        L.wpos += 16;
        if (L.ns == 2) {
            k = (L.wpos >> 2) & (IL_RING_DW - 1);
            *(uint2*)(L.ring + k) = make_uint2(L.s1.x, L.s1.y);
            *(uint2*)(L.ring + k + 2) = make_uint2(L.s1.z, L.s1.w);
            L.ring[k == 0 ? IL_RING_DW : IL_RING_DW + 1] = L.s1.x;
            L.wpos += 16;
        }
        L.ns = 0;
    }
    tok_flush_hot(L);
    uint32_t lvl = L.wpos - L.rpos;
    if (lvl <= 96 && L.vp < L.vend) {
        if (!HOT_CHECK(L, (const uint8_t*)L.vp >= L.chk_lo && (const uint8_t*)(L.vp + 2) <= L.chk_hi, 1,
                       (uintptr_t)L.vp, (uintptr_t)L.vend)) return;
        L.s0 = *L.vp++;
        L.ns = 1;
        if (lvl <= 64 && L.vp < L.vend) { L.s1 = *L.vp++; L.ns = 2; }
    }
#endif
}
#endif

// ------------------------------------------------------------------ canonical trees

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

// packed word for the code (rank offset / threshold / shift) whose 15-bit bit-reversed
// prefix is rc: pk[1 + #{k : rc >= lim[k]}], as a depth-4 select tree (limits ascend)
// The selects use VGPR masks (all ones where rc >= lim[k]) and v_bfi_b32, written as
// inline asm so they stay VALU-only: compare-into-SGPR + v_cndmask pairs serialise on
// one SGPR pair with wait states between them (gfx950), 15 times per tree.
__device__ __forceinline__ uint32_t ge_mask(uint32_t rc, uint32_t lim) {   // lim, rc <= 32768
    uint32_t m;
    asm("v_sub_u32 %0, %1, %2\n\tv_ashrrev_i32 %0, 31, %0" : "=&v"(m) : "v"(lim - 1u), "v"(rc));
    return m;
}
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) {   // m ? a : b, bitwise
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t tsel(const HTree& T, uint32_t rc) {
    uint32_t g1 = ge_mask(rc, T.lim[1]), g2 = ge_mask(rc, T.lim[2]), g3 = ge_mask(rc, T.lim[3]);
    uint32_t g4 = ge_mask(rc, T.lim[4]), g5 = ge_mask(rc, T.lim[5]), g6 = ge_mask(rc, T.lim[6]);
    uint32_t g7 = ge_mask(rc, T.lim[7]), g8 = ge_mask(rc, T.lim[8]), g9 = ge_mask(rc, T.lim[9]);
    uint32_t g10 = ge_mask(rc, T.lim[10]), g11 = ge_mask(rc, T.lim[11]), g12 = ge_mask(rc, T.lim[12]);
    uint32_t g13 = ge_mask(rc, T.lim[13]), g14 = ge_mask(rc, T.lim[14]), g15 = ge_mask(rc, T.lim[15]);
    uint32_t a1 = bfi(g1, T.pk[2], T.pk[1]), a3 = bfi(g3, T.pk[4], T.pk[3]);
    uint32_t a5 = bfi(g5, T.pk[6], T.pk[5]), a7 = bfi(g7, T.pk[8], T.pk[7]);
    uint32_t a9 = bfi(g9, T.pk[10], T.pk[9]), a11 = bfi(g11, T.pk[12], T.pk[11]);
    uint32_t a13 = bfi(g13, T.pk[14], T.pk[13]), a15 = bfi(g15, T.pk[16], T.pk[15]);
    uint32_t b1 = bfi(g2, a3, a1), b5 = bfi(g6, a7, a5), b9 = bfi(g10, a11, a9), b13 = bfi(g14, a15, a13);
    uint32_t c1 = bfi(g4, b5, b1), c9 = bfi(g12, b13, b9);
    return bfi(g8, c9, c1);
}
#ifndef IL_BSEARCH
#define IL_BSEARCH 1                      // binary-search tree select (C2 decode -3 %)
#endif
#if IL_BSEARCH
// the same word by a 4-step binary search over the (non-decreasing) limits: c = #{k : rc >=
// lim[k]} bit by bit, with the pk select tree cut by the top bit first so that only its last
// level waits for the last compare (34 VALU against 45)
__device__ __forceinline__ uint32_t ge_mask_m1(uint32_t rc, uint32_t limm1) {   // rc >= limm1 + 1
    uint32_t m;
    asm("v_sub_u32 %0, %1, %2\n\tv_ashrrev_i32 %0, 31, %0" : "=&v"(m) : "v"(limm1), "v"(rc));
    return m;
}
// M1: the tree's limits are stored minus one (the hot loop's register copy, hot_epoch)
template <bool M1 = false>
__device__ __forceinline__ uint32_t tsel_bs(const HTree& T, uint32_t rc) {
    auto ge = [&](uint32_t x) { return M1 ? ge_mask_m1(rc, x) : ge_mask(rc, x); };
    const uint32_t m1 = ge(T.lim[8]);
    // pk[1 + c]: level 1 by m1 (c >= 8)
    const uint32_t p1 = bfi(m1, T.pk[9], T.pk[1]), p2 = bfi(m1, T.pk[10], T.pk[2]);
    const uint32_t p3 = bfi(m1, T.pk[11], T.pk[3]), p4 = bfi(m1, T.pk[12], T.pk[4]);
    const uint32_t p5 = bfi(m1, T.pk[13], T.pk[5]), p6 = bfi(m1, T.pk[14], T.pk[6]);
    const uint32_t p7 = bfi(m1, T.pk[15], T.pk[7]), p8 = bfi(m1, T.pk[16], T.pk[8]);
    const uint32_t l1 = bfi(m1, T.lim[9], T.lim[1]), l3 = bfi(m1, T.lim[11], T.lim[3]);
    const uint32_t l5 = bfi(m1, T.lim[13], T.lim[5]), l7 = bfi(m1, T.lim[15], T.lim[7]);
    const uint32_t l2 = bfi(m1, T.lim[10], T.lim[2]), l6 = bfi(m1, T.lim[14], T.lim[6]);
    const uint32_t m2 = ge(bfi(m1, T.lim[12], T.lim[4]));
    const uint32_t q1 = bfi(m2, p5, p1), q2 = bfi(m2, p6, p2), q3 = bfi(m2, p7, p3), q4 = bfi(m2, p8, p4);
    const uint32_t k1 = bfi(m2, l5, l1), k3 = bfi(m2, l7, l3);
    const uint32_t m3 = ge(bfi(m2, l6, l2));
    const uint32_t r1 = bfi(m3, q3, q1), r2 = bfi(m3, q4, q2);
    const uint32_t m4 = ge(bfi(m3, k3, k1));
    return bfi(m4, r2, r1);
}
#ifndef IL_TSEL_ASM
#define IL_TSEL_ASM 1
#endif
#if IL_TSEL_ASM
// tsel_bs<true> as one asm block: as separate statements the compiler put an s_nop between an asm
// statement and the next one reading its result (it cannot see inside them), 7 per distance decode
__device__ __forceinline__ uint32_t tsel_hot_asm(const HTree& T, uint32_t rc) {
    uint32_t r, m, lx, p1, p2, p3, p4, p5, p6, p7, p8, a1, a2, a3, a5, a6, a7;
    asm("v_sub_u32 %[m], %[L8], %[rc]\n\t"
        "v_ashrrev_i32 %[m], 31, %[m]\n\t"
        "v_bfi_b32 %[lx], %[m], %[L12], %[L4]\n\t"
        "v_bfi_b32 %[p1], %[m], %[P9], %[P1]\n\t"
        "v_bfi_b32 %[p2], %[m], %[P10], %[P2]\n\t"
        "v_bfi_b32 %[p3], %[m], %[P11], %[P3]\n\t"
        "v_bfi_b32 %[p4], %[m], %[P12], %[P4]\n\t"
        "v_bfi_b32 %[p5], %[m], %[P13], %[P5]\n\t"
        "v_bfi_b32 %[p6], %[m], %[P14], %[P6]\n\t"
        "v_bfi_b32 %[p7], %[m], %[P15], %[P7]\n\t"
        "v_bfi_b32 %[p8], %[m], %[P16], %[P8]\n\t"
        "v_bfi_b32 %[a1], %[m], %[L9], %[L1]\n\t"
        "v_bfi_b32 %[a2], %[m], %[L10], %[L2]\n\t"
        "v_bfi_b32 %[a3], %[m], %[L11], %[L3]\n\t"
        "v_bfi_b32 %[a5], %[m], %[L13], %[L5]\n\t"
        "v_bfi_b32 %[a6], %[m], %[L14], %[L6]\n\t"
        "v_bfi_b32 %[a7], %[m], %[L15], %[L7]\n\t"
        "v_sub_u32 %[m], %[lx], %[rc]\n\t"          // level 2
        "v_ashrrev_i32 %[m], 31, %[m]\n\t"
        "v_bfi_b32 %[p1], %[m], %[p5], %[p1]\n\t"
        "v_bfi_b32 %[p2], %[m], %[p6], %[p2]\n\t"
        "v_bfi_b32 %[p3], %[m], %[p7], %[p3]\n\t"
        "v_bfi_b32 %[p4], %[m], %[p8], %[p4]\n\t"
        "v_bfi_b32 %[lx], %[m], %[a6], %[a2]\n\t"
        "v_bfi_b32 %[a1], %[m], %[a5], %[a1]\n\t"
        "v_bfi_b32 %[a3], %[m], %[a7], %[a3]\n\t"
        "v_sub_u32 %[m], %[lx], %[rc]\n\t"          // level 3
        "v_ashrrev_i32 %[m], 31, %[m]\n\t"
        "v_bfi_b32 %[lx], %[m], %[a3], %[a1]\n\t"
        "v_bfi_b32 %[p1], %[m], %[p3], %[p1]\n\t"
        "v_bfi_b32 %[p2], %[m], %[p4], %[p2]\n\t"
        "v_sub_u32 %[m], %[lx], %[rc]\n\t"          // level 4
        "v_ashrrev_i32 %[m], 31, %[m]\n\t"
        "v_bfi_b32 %[r], %[m], %[p2], %[p1]"
        : [r] "=&v"(r), [m] "=&v"(m), [lx] "=&v"(lx), [p1] "=&v"(p1), [p2] "=&v"(p2), [p3] "=&v"(p3),
          [p4] "=&v"(p4), [p5] "=&v"(p5), [p6] "=&v"(p6), [p7] "=&v"(p7), [p8] "=&v"(p8), [a1] "=&v"(a1),
          [a2] "=&v"(a2), [a3] "=&v"(a3), [a5] "=&v"(a5), [a6] "=&v"(a6), [a7] "=&v"(a7)
        : [rc] "v"(rc), [L1] "v"(T.lim[1]), [L2] "v"(T.lim[2]), [L3] "v"(T.lim[3]), [L4] "v"(T.lim[4]),
          [L5] "v"(T.lim[5]), [L6] "v"(T.lim[6]), [L7] "v"(T.lim[7]), [L8] "v"(T.lim[8]), [L9] "v"(T.lim[9]),
          [L10] "v"(T.lim[10]), [L11] "v"(T.lim[11]), [L12] "v"(T.lim[12]), [L13] "v"(T.lim[13]),
          [L14] "v"(T.lim[14]), [L15] "v"(T.lim[15]), [P1] "v"(T.pk[1]), [P2] "v"(T.pk[2]), [P3] "v"(T.pk[3]),
          [P4] "v"(T.pk[4]), [P5] "v"(T.pk[5]), [P6] "v"(T.pk[6]), [P7] "v"(T.pk[7]), [P8] "v"(T.pk[8]),
          [P9] "v"(T.pk[9]), [P10] "v"(T.pk[10]), [P11] "v"(T.pk[11]), [P12] "v"(T.pk[12]),
          [P13] "v"(T.pk[13]), [P14] "v"(T.pk[14]), [P15] "v"(T.pk[15]), [P16] "v"(T.pk[16]));
    return r;
}
#define tsel tsel_bs<false>
#define tsel_hot tsel_hot_asm
#else
#define tsel tsel_bs<false>
#define tsel_hot tsel_bs<true>
#endif
#else
#define tsel_hot tsel
#endif
__device__ __forceinline__ int32_t pk_rank(uint32_t v, uint32_t rc) {
    return (int32_t)(v >> 16) + (int32_t)(rc >> (v & 31u)) - 32768;   // bit 4 is 0: v_lshrrev's own mask
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
#define TREE_NEED(T, len, rank) \
    dec_need((T).c[0], (T).c[1], (T).c[2], (T).c[3], (T).c[4], (T).l, (T).kmin, (T).g, (T).left, (len), (rank))

// limits and packed words from the counts; hs = per-length literal threshold
// (packed like the counts) or null for the distance tree
template <bool LIT>
__device__ __forceinline__ void finish_tree(Tree& T, const uint32_t (&hs)[5]) {
    uint32_t code = 0;
    int32_t idx = 0;
#pragma unroll
    for (int L = 1; L <= 15; ++L) {
        uint32_t cl = cnt_get(T.c, L);
        T.lim[L] = (code + cl) << (15 - L);
        int32_t off = idx - (int32_t)code;
        uint32_t h = LIT ? cnt_get(hs, L) : 511u;
        T.pk[L] = ((uint32_t)(off + 32768) << 16) | (h << 5) | (uint32_t)(15 - L);
        idx += (int32_t)cl;
        code = (code + cl) << 1;
    }
    T.lim[0] = 0;
    T.pk[0] = 0;
    T.pk[16] = ((uint32_t)(IL_BAD_IDX + 32768) << 16) | 15u;   // threshold 0: never a literal
}

// f(s, lens[s]) for s in [0, n), the lengths read 16 at a time: a lane's byte loads from its HBM
// scratch each waited a round trip (a dynamic header's two passes over ~300 lengths: ~130 us of a
// block's block-level work).  The scratch is 16-byte aligned and kInflateScratchPerStream (320) a
// multiple of 16, so the aligned chunks around [lens, lens + n) stay inside the stream's scratch.
template <class F>
__device__ __forceinline__ void for_lens(const uint8_t* lens, int n, F f) {
    const uintptr_t a = (uintptr_t)lens, a0 = a & ~(uintptr_t)15;
    const int lead = (int)(a - a0);
    for (int b = 0; b < n + lead; b += 16) {
        const uint4 w = *(const uint4*)(a0 + (uintptr_t)b);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const uint32_t wj = j < 4 ? w.x : j < 8 ? w.y : j < 12 ? w.z : w.w;
            const int s = b + j - lead;
            if (s >= 0 && s < n) f(s, (int)((wj >> (8 * (j & 3))) & 255u));
        }
    }
}

// counts + Kraft remainder for n lengths read from global memory
__device__ __forceinline__ void count_lens(Tree& T, const uint8_t* lens, int n, int root) {
    T.c[0] = T.c[1] = T.c[2] = T.c[3] = T.c[4] = 0;
    for_lens(lens, n, [&](int, int len) { if (len) cnt_add(T.c, len, 1u); });
    int left = 1, kmin = 16, g = 0;
#pragma unroll
    for (int L = 1; L <= 15; ++L) {
        int cl = (int)cnt_get(T.c, L);
        left = 2 * left - cl;
        if (cl) { kmin = kmin > L ? L : kmin; g = L; }
    }
    T.kmin = kmin;
    T.g = g;
    T.left = left;
    int l = root;
    if (g != 0) { if (l < kmin) l = kmin; if (l > g) l = g; }
    T.l = l;
}

// rank -> symbol bytes in canonical order; returns the per-length literal thresholds
// (lit/len: symbols >= 256 are stored as sym - 256 after the literals of their length)
__device__ __forceinline__ void place_syms(const Tree& T, const uint8_t* lens, int n, uint8_t* out,
                                           uint32_t (&hs)[5]) {
    uint32_t nx[5] = { 0, 0, 0, 0, 0 };
    uint32_t idx = 0;
#pragma unroll
    for (int L = 1; L <= 15; ++L) { cnt_add(nx, L, idx); idx += cnt_get(T.c, L); }
    int nlit = n < 256 ? n : 256;
    for_lens(lens, nlit, [&](int s, int len) {
        if (len) { out[cnt_get(nx, len)] = (uint8_t)s; cnt_add(nx, len, 1u); }
    });
    hs[0] = nx[0]; hs[1] = nx[1]; hs[2] = nx[2]; hs[3] = nx[3]; hs[4] = nx[4];
    if (n > nlit)
        for_lens(lens + nlit, n - nlit, [&](int s, int len) {
            if (len) { out[cnt_get(nx, len)] = (uint8_t)s; cnt_add(nx, len, 1u); }   // s = symbol - 256
        });
}

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
__device__ __forceinline__ void with_dummies(const Tree& T, uint32_t (&c)[5]) {
    c[0] = T.c[0]; c[1] = T.c[1]; c[2] = T.c[2]; c[3] = T.c[3]; c[4] = T.c[4];
    if (T.g != 0 && T.left > 0) cnt_add(c, T.g, (uint32_t)(T.left >> (15 - T.g)));
}

// ------------------------------------------------------------------ tokens

// token: bit31=0 -> literals: bits 24-25 = count-1 (1..3 bytes in bits 0-23)
//        bit31=1 -> match: bits 16-23 = length-3, bits 0-14 = distance-1
// 32 staged tokens -> HBM.  Some lane of the wave fills its stage at most steps (64 lanes,
// one flush per 32 tokens each), so this block runs nearly every step: all LDS reads are
// issued before the first store (one wait, not one per 16 bytes).
__device__ __forceinline__ void tok_flush_stage(Core& L) {
    if (!HOT_CHECK(L, L.ntok >= IL_TSTAGE && L.ntok <= L.tcap && (L.ntok & (IL_TSTAGE - 1)) == 0, 5,
                   L.ntok, L.tcap)) return;
    const uint2* s = (const uint2*)L.ts;
    GLB uint4* d = (GLB uint4*)(L.tb + (L.ntok - IL_TSTAGE));
    uint2 v[IL_TSTAGE / 2];
#pragma unroll
    for (int k = 0; k < IL_TSTAGE / 2; ++k) v[k] = s[k];
#pragma unroll
    for (int k = 0; k < IL_TSTAGE / 4; ++k) d[k] = make_uint4(v[2 * k].x, v[2 * k].y, v[2 * k + 1].x, v[2 * k + 1].y);
}
// The stage is a ring of the last 32 tokens.  The cold code flushes each 32-token line as it
// fills; the symbol loop (IL_UNIFORM_FLUSH) only stages, and writes 16-token chunks at its
// wave-uniform ring step (tok_flush_hot): a push site then has no flush branch, which some
// lane of a wave of distinct streams took at nearly every step.
template <class C>
__device__ __forceinline__ void tok_push(C& L, uint32_t t) {
    uint32_t k = L.ntok & (IL_TSTAGE - 1);
    L.ts[k] = t;
    L.ntok++;
    if constexpr (!(IL_UNIFORM_FLUSH && std::is_same<C, Hot>::value))
        if (k == IL_TSTAGE - 1) tok_flush_stage(L);
}
template <class C>
__device__ __forceinline__ void tok_flush_lits(C& L) {
    if (L.nlit) {
        tok_push(L, ((L.nlit - 1u) << 24) | L.litw);
        L.nlit = 0;
        L.litw = 0;
    }
}
#ifndef IL_FULL_AT_RING
#define IL_FULL_AT_RING 1                 // token room checked at the ring step (C2 decode -2 %, distinct -3 %)
#endif
#ifndef IL_TWO_LOOPS
#define IL_TWO_LOOPS 1                    // the unchecked 4-step loop, then the checked one (hot_epoch)
#endif
#ifndef IL_UNCHECKED_RUN
#define IL_UNCHECKED_RUN 1                // 4 steps without bit / room checks when the ring step allows
#endif
#ifndef IL_BF_TOKENS
#define IL_BF_TOKENS 1
#endif
#ifndef IL_OPEN_SLOT
#define IL_OPEN_SLOT 1                    // symbol loop: the open literal token kept in its stage slot
#endif
template <class C>
__device__ __forceinline__ void tok_lit(C& L, uint32_t b) {
    L.litw |= b << (8 * L.nlit);
    if constexpr (IL_OPEN_SLOT && IL_UNIFORM_FLUSH && std::is_same<C, Hot>::value) {
        // the token of the pending literals is stored in slot ntok & 31 as it grows (not yet
        // counted, so no flush takes it); the third literal counts it, and a match only counts it
        L.ts[L.ntok & (IL_TSTAGE - 1)] = (L.nlit << 24) | L.litw;
        const bool full = ++L.nlit == 3;
        L.ntok += full ? 1u : 0u;
        L.litw = full ? 0u : L.litw;
        L.nlit = full ? 0u : L.nlit;
    } else if constexpr (IL_BF_TOKENS && IL_UNIFORM_FLUSH && std::is_same<C, Hot>::value) {
        // symbol loop: no branch -- a store that does not push goes to the stage's spare slot
        const bool full = ++L.nlit == 3;
        L.ts[full ? (L.ntok & (IL_TSTAGE - 1)) : IL_TSTAGE] = (2u << 24) | L.litw;
        L.ntok += full ? 1u : 0u;
        L.litw = full ? 0u : L.litw;
        L.nlit = full ? 0u : L.nlit;
    } else {
        if (++L.nlit == 3) tok_flush_lits(L);
    }
}
template <class C>
__device__ __forceinline__ void tok_match(C& L, uint32_t len, uint32_t dist) {
    if constexpr (IL_OPEN_SLOT && IL_UNIFORM_FLUSH && std::is_same<C, Hot>::value) {
        L.ntok += L.nlit != 0 ? 1u : 0u;                  // (its token is in its slot: tok_lit)
        L.ts[L.ntok & (IL_TSTAGE - 1)] = 0x80000000u | ((len - 3u) << 16) | (dist - 1u);
        L.ntok++;
        L.nlit = 0;
        L.litw = 0;
    } else if constexpr (IL_BF_TOKENS && IL_UNIFORM_FLUSH && std::is_same<C, Hot>::value) {
        const bool hl = L.nlit != 0;
        L.ts[hl ? (L.ntok & (IL_TSTAGE - 1)) : IL_TSTAGE] = ((L.nlit - 1u) << 24) | L.litw;
        L.ntok += hl ? 1u : 0u;
        L.ts[L.ntok & (IL_TSTAGE - 1)] = 0x80000000u | ((len - 3u) << 16) | (dist - 1u);
        L.ntok++;
        L.nlit = 0;
        L.litw = 0;
    } else {
        tok_flush_lits(L);
        tok_push(L, 0x80000000u | ((len - 3u) << 16) | (dist - 1u));
    }
}
// symbol loop: the next 16 staged tokens to HBM once there are (at most 2 tokens per step,
// 4 steps between calls: at most 23 unwritten, within the 32-token ring)
__device__ __forceinline__ void tok_flush_hot(Hot& L) {
    if (!IL_UNIFORM_FLUSH) return;
    const bool f = L.ntok - L.nfl >= 16u;
    if (__ballot(f)) {
        if (f && HOT_CHECK(L, L.nfl + 16u <= L.tcap && L.nfl + 16u <= L.ntok && (L.nfl & 15u) == 0, 2,
                           L.nfl, ((uint64_t)L.ntok << 32) | L.tcap)) {
            const uint2* st = (const uint2*)(L.ts + (L.nfl & (IL_TSTAGE - 1)));
            GLB uint4* d = (GLB uint4*)(L.tb + L.nfl);
            uint2 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = st[k];
#pragma unroll
            for (int k = 0; k < 4; ++k) d[k] = make_uint4(v[2 * k].x, v[2 * k].y, v[2 * k + 1].x, v[2 * k + 1].y);
            L.nfl += 16u;
        }
    }
}
__device__ __forceinline__ void tok_finish(Core& L) {
    tok_flush_lits(L);
    if (!HOT_CHECK(L, L.ntok <= L.tcap, 6, L.ntok, L.tcap)) return;
    uint32_t k = L.ntok & (IL_TSTAGE - 1), b = L.ntok - k;
    for (uint32_t j = 0; j < k; ++j) L.tb[b + j] = L.ts[j];
}

__device__ __forceinline__ void lane_fail(Core& L, int status, int zmsg) {
    L.status = status;
    L.zmsg = zmsg;
    L.mode = LM_DONE;
}
// The unit that started at bit L.ubit (a header, block header, symbol, stored byte or
// trailer) cannot finish: out of input (why 1) or of output room (why 2).  A one-shot
// stream ends there; an incremental one (Inflater.append across calls) is parked at
// the unit's start and waits for the next call -- the reference stops its output at the
// same place, holding the unit's bits in its bit buffer (infcodes.ts:367-387 need rule).
// cold_run stops at once and parks the stream at L.ubit.
__device__ __forceinline__ void lane_stall(Lane& L, int why) {
    if (!L.streaming) { lane_fail(L, why == 1 ? SDZ_TRUNCATED : SDZ_OUT_OVERFLOW, 0); return; }
    L.stall = why;
}

// ------------------------------------------------------------------ block setup

__device__ __forceinline__ void setup_fixed(Lane& L, Tree& LL, Tree& DD, uint8_t* region) {
    // ranks: 256..279 (7 bits) | 0..143, 280..287 (8 bits) | 144..255 (9 bits)
    int k = 0;
    for (int s = 0; s < 24; ++s) region[k++] = (uint8_t)s;
    for (int s = 0; s < 144; ++s) region[k++] = (uint8_t)s;
    for (int s = 24; s < 32; ++s) region[k++] = (uint8_t)s;
    for (int s = 144; s < 256; ++s) region[k++] = (uint8_t)s;
    for (int s = 0; s < 30; ++s) region[IL_DSYM + s] = (uint8_t)s;
    LL.c[0] = LL.c[1] = LL.c[2] = LL.c[3] = LL.c[4] = 0;
    cnt_add(LL.c, 7, 24); cnt_add(LL.c, 8, 152); cnt_add(LL.c, 9, 112);
    LL.l = 9; LL.kmin = 7; LL.g = 9; LL.left = 0;
    DD.c[0] = DD.c[1] = DD.c[2] = DD.c[3] = DD.c[4] = 0;
    cnt_add(DD.c, 5, 30);
    DD.l = 5; DD.kmin = 5; DD.g = 5; DD.left = 2 << 10;
    uint32_t hs[5] = { 0, 0, 0, 0, 0 };                  // literal thresholds: 0 | 168 | 288
    cnt_add(hs, 8, 168); cnt_add(hs, 9, 288);
    finish_tree<true>(LL, hs);
    finish_tree<false>(DD, hs);
    L.fixed = 1;
}

// infblocks.ts:334-551 + inftree.ts:313-379.  Returns false when the lane stopped
// (error or stall); L.status/zmsg say which.
__device__ __forceinline__ bool setup_dynamic(Lane& L, Tree& LL, Tree& DD, uint8_t* region) {
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
        uint32_t rc = __builtin_bitreverse32(br_peek32(L)) >> 25;
        int len = 1;
        int32_t off = off7[1];
#pragma unroll
        for (int k = 1; k < 7; ++k) { bool ge = rc >= lim7[k]; len = ge ? k + 1 : len; off = ge ? off7[k + 1] : off; }
        // g7 == 1 with one code: both patterns read the last entry written (inftree.ts:265-267)
        uint32_t c = cls[(g7 == 1 && left > 0) ? 0 : (off + (int32_t)(rc >> (7 - len)))];
        if (g7 == 1 && left > 0) len = 1;
        br_drop(L, (uint32_t)len);
        if (!HOT_CHECK(L, idx < (int)kInflateScratchPerStream, 8, idx, total)) return false;
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
    count_lens(LL, L.lens, nl, 9);
    if (LL.left < 0) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_LL_OVERSUB; return false; }
    count_lens(DD, L.lens + nl, nd, 6);
    bool llzero = LL.g == 0, ddzero = DD.g == 0;
    int ent_ll = 0, ent_d = 0;
    uint32_t tl[5], td[5];
    with_dummies(LL, tl);
    with_dummies(DD, td);
    bool exact = false;
    if (!llzero) ent_ll = table_bound(tl, LL.l, LL.g);
    if (!ddzero && DD.left >= 0) ent_d = table_bound(td, DD.l, DD.g);
    if (ent_ll + ent_d > 1400) {
        exact = true;
        int dummy;
        if (!llzero) ent_ll = huft_replay(tl[0], tl[1], tl[2], tl[3], tl[4], LL.kmin, LL.g, LL.l, -1, &dummy);
    }
    if (!llzero && ent_ll > 1400) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_LL_OVERSUB; return false; }
    if (llzero || (LL.left > 0 && LL.g != 1)) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_LL_INCOMPLETE; return false; }
    // distance tree (inftree.ts:359-376)
    if (DD.left < 0) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_D_OVERSUB; return false; }
    if (exact && !ddzero) {
        int dummy;
        ent_d = huft_replay(td[0], td[1], td[2], td[3], td[4], DD.kmin, DD.g, DD.l, -1, &dummy);
    }
    if (!ddzero && ent_ll + ent_d > 1400) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_D_OVERSUB; return false; }
    if (!ddzero && DD.left > 0 && DD.g != 1) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_D_INCOMPLETE; return false; }
    if (ddzero && nl > 257) { L.status = SDZ_DATA_ERROR; L.zmsg = ZM_D_EMPTY; return false; }
    uint32_t hs[5], hd[5];
    place_syms(LL, L.lens, nl, region, hs);
    place_syms(DD, L.lens + nl, nd, region + IL_DSYM, hd);
    finish_tree<true>(LL, hs);
    finish_tree<false>(DD, hd);
    L.nl = nl; L.nd = nd;
    L.fixed = 0;
    return true;
}

// one block-level step for a lane that is not decoding symbols
__device__ __forceinline__ void block_step(Lane& L, Tree& LL, Tree& DD, uint8_t* region) {
    if (L.mode == LM_TYPE) {
        uint32_t t;
        if (!br_get(L, 3, t)) { lane_stall(L, 1); return; }
        L.last = (int)(t & 1);
        uint32_t bt = t >> 1;
        if (bt == 0) {                                   // stored (infblocks.ts:184-196, 243-277)
            uint64_t cons = br_consumed(L);
            br_drop(L, (uint32_t)((8 - (cons & 7)) & 7));
            uint32_t lo, hi;
            if (!br_get(L, 16, lo) || !br_get(L, 16, hi)) { lane_stall(L, 1); return; }
            if ((~hi & 0xffffu) != lo) { lane_fail(L, SDZ_DATA_ERROR, ZM_STORED_LENS); return; }
            L.stored_left = lo;
            L.mode = lo ? LM_STORED : (L.last ? LM_TRAILER : LM_TYPE);
        } else if (bt == 1) {
            setup_fixed(L, LL, DD, region);
            L.mode = LM_CODES;
        } else if (bt == 2) {
            if (!setup_dynamic(L, LL, DD, region)) {
                if (L.status == SDZ_TRUNCATED) { L.status = SDZ_OK; lane_stall(L, 1); }
                else L.mode = LM_DONE;
                return;
            }
            L.mode = LM_CODES;
        } else {
            lane_fail(L, SDZ_DATA_ERROR, ZM_BLOCK_TYPE);
        }
        return;
    }
    if (L.mode == LM_STORED) {                            // infblocks.ts:278-333, resumable
        while (L.stored_left && !L.full) {
            uint32_t b;
            if (L.streaming) L.ubit = br_consumed(L);
            if (!br_get(L, 8, b)) { lane_stall(L, 1); return; }
            if (L.room == 0) { lane_stall(L, 2); return; }
            tok_lit(L, b);
            L.room--;
            L.stored_left--;
            if (L.ntok + 3 > L.tcap) L.full = true;
        }
        if (!L.stored_left) L.mode = L.last ? LM_TRAILER : LM_TYPE;
        return;
    }
    if (L.mode == LM_TRAILER) {                          // inflate.ts:403-463
        uint64_t cons = br_consumed(L);
        br_refill(L);
        br_drop(L, (uint32_t)((8 - (cons & 7)) & 7));   // WASH + blocks.reset()
        if (L.container == SDZ_CONTAINER_ZLIB) {
            uint32_t v = 0;
            for (int k = 0; k < 4; ++k) {
                uint32_t b;
                if (!br_get(L, 8, b)) { lane_stall(L, 1); return; }
                v = (v << 8) | b;
            }
            L.stored_ck = (int32_t)v;
        } else if (L.container == SDZ_CONTAINER_GZIP) {
            uint32_t v = 0, z = 0;
            for (int k = 0; k < 4; ++k) {
                uint32_t b;
                if (!br_get(L, 8, b)) { lane_stall(L, 1); return; }
                v = (v >> 8) | (b << 24);
            }
            L.stored_ck = (int32_t)v;
            for (int k = 0; k < 4; ++k) {
                uint32_t b;
                if (!br_get(L, 8, b)) { lane_stall(L, 1); return; }
                z = (z >> 8) | (b << 24);
            }
            L.stored_size = (int32_t)z;
        }
        L.mode = LM_DONE;
        L.status = br_avail(L) > 0 ? SDZ_TRAILING : SDZ_OK;
        return;
    }
}

// length symbol (1..29 = sym - 256) -> base length and extra bits (infcodes.ts:27-35)
// (selects only: a nested conditional here compiled to an exec-mask branch)
__device__ __forceinline__ uint32_t len_base(uint32_t li, uint32_t& e) {
    const uint32_t k = li - 1u;                           // 0..28
    e = k - 8u < 20u ? (k - 4u) >> 2 : 0u;                // 8..27: 1..5
    const uint32_t sh = ((4u + (k & 3u)) << e) + 3u;      // (k = 4..7, e = 0: k + 3)
    const uint32_t b = k < 4u ? k + 3u : sh;
    return k == 28u ? 258u : b;
}
// distance symbol 0..29 -> base distance and extra bits (infcodes.ts:37-46)
__device__ __forceinline__ uint32_t dist_base(uint32_t ds, uint32_t& e) {
    e = ds < 4u ? 0u : (ds - 2u) >> 1;
    return ds < 4u ? ds + 1u : ((2u + (ds & 1u)) << e) + 1u;
}

// decode one literal/length symbol (+ its distance): the fast path, taken while at
// least 64 input bits remain (one step reads at most 48)
// CHK = false: the caller has checked for the next 4 steps what the room checks test (room for 4
// matches), so a step has none (IL_UNCHECKED_RUN)
template <bool CHK = true>
__device__ __forceinline__ void fast_step(Hot& L, const HTree& LL, const HTree& DD, const uint8_t* region) {
    uint32_t pw = br_refill_peek(L);
    uint32_t rc = __builtin_bitreverse32(pw) >> 17;
    uint32_t v = tsel_hot(LL, rc);
    int32_t idx = pk_rank(v, rc);
    uint32_t len = 15u - (v & 15u);
    uint32_t b = region[idx];
    L.bo += len;
    if (idx < (int32_t)((v >> 5) & 511u)) {               // literal
        if (CHK && L.room == 0) { lane_fail(L, SDZ_OUT_OVERFLOW, 0); return; }
        L.room--;
        tok_lit(L, b);
        return;
    }
    if (b - 1u >= 29u || idx >= 288) {                    // end of block, or invalid code
        if (b == 0 && idx < 288) L.mode = L.last ? LM_TRAILER : LM_TYPE;
        else lane_fail(L, SDZ_DATA_ERROR, ZM_INVALID_LITLEN);
        return;
    }
    uint32_t e;
    uint32_t mlen = len_base(b, e);
    mlen += (pw >> len) & ((1u << e) - 1u);
    L.bo += e;
    pw = br_refill_peek(L);
    rc = __builtin_bitreverse32(pw) >> 17;
    v = tsel_hot(DD, rc);
    idx = pk_rank(v, rc);
    len = 15u - (v & 15u);
    uint32_t ds = region[IL_DSYM + idx];
    if (idx >= (int32_t)((v >> 5) & 511u)) { lane_fail(L, SDZ_DATA_ERROR, ZM_INVALID_DIST); return; }
    uint32_t dist = dist_base(ds, e);
    dist += (pw >> len) & ((1u << e) - 1u);
    L.bo += len + e;
    if (CHK && L.room < mlen) { lane_fail(L, SDZ_OUT_OVERFLOW, 0); return; }
    L.room -= mlen;
    tok_match(L, mlen, dist);
}
#if IL_REFILL2
// fast_step on the IL_REFILL2 reader: one refill, a 64-bit peek (lo, hi) at the symbol's first
// bit; the length's extra bits (<= 15 + 5 bits in) and the distance code with its extra bits
// (<= 15 + 13 bits from its start) come from it
// A failure in the symbol loop sets the mode and the message only (zm 0: output overflow); the
// status follows from them when the epoch ends (hot_fix_status): one value less to merge per step.
__device__ __forceinline__ void hot_fail(Hot& L, int zm) { L.mode = LM_DONE; L.zmsg = zm; }
__device__ __forceinline__ void hot_fix_status(Hot& L) {
    if (L.mode == LM_DONE && L.status == SDZ_OK) L.status = L.zmsg ? SDZ_DATA_ERROR : SDZ_OUT_OVERFLOW;
}
template <bool CHK = true>
__device__ __forceinline__ void fast_step2(Hot& L, const HTree& LL, const HTree& DD, const uint8_t* region) {
    br_refill2(L);
    const uint32_t lo = __builtin_amdgcn_alignbit(L.w1, L.w0, L.bo);
    const uint32_t hi = __builtin_amdgcn_alignbit(L.w2, L.w1, L.bo);
    uint32_t rc = __builtin_bitreverse32(lo) >> 17;
    uint32_t v = tsel_hot(LL, rc);
    const int32_t idx = pk_rank(v, rc);
    const uint32_t len = 15u - (v & 15u);
    const uint32_t b = region[idx];
    if (idx < (int32_t)((v >> 5) & 511u)) {               // literal
        L.bo += len;
        if (CHK && L.room == 0) { hot_fail(L, 0); return; }
        L.room--;
        tok_lit(L, b);
        return;
    }
    // a length code -- or the end of block or an invalid code, tested once with the distance
    // code's validity below (the distance decode of those is discarded)
    uint32_t e;
    uint32_t mlen = len_base(b, e);
    mlen += (lo >> len) & ((1u << e) - 1u);
    const uint32_t s = len + e;                           // <= 20
    const uint32_t pd = __builtin_amdgcn_alignbit(hi, lo, s);
    rc = __builtin_bitreverse32(pd) >> 17;
    v = tsel_hot(DD, rc);
    const int32_t dx = pk_rank(v, rc);
    const uint32_t dlen = 15u - (v & 15u);
    const uint32_t ds = region[IL_DSYM + dx];
    uint32_t de;
    uint32_t dist = dist_base(ds, de);
    dist += (pd >> dlen) & ((1u << de) - 1u);
    const bool badl = b - 1u >= 29u || idx >= 288;
    if (badl || dx >= (int32_t)((v >> 5) & 511u)) {
        if (!badl) { L.bo += s; hot_fail(L, ZM_INVALID_DIST); return; }
        L.bo += len;
        if (b == 0 && idx < 288) L.mode = L.last ? LM_TRAILER : LM_TYPE;
        else hot_fail(L, ZM_INVALID_LITLEN);
        return;
    }
    L.bo += s + dlen + de;
    if (CHK && L.room < mlen) { hot_fail(L, 0); return; }
    L.room -= mlen;
    tok_match(L, mlen, dist);
}
#define IL_FAST_STEP fast_step2
#define IL_RING_STEP ring_step2
#define IL_BR_INIT br_init2
#else
#define IL_FAST_STEP fast_step
#define IL_RING_STEP ring_step
#define IL_BR_INIT br_init
#endif

// the same with the reference's end-of-input behaviour: every read checks the
// bits available, and a code is only resolved once the reference's table walk
// would have had the bits it asks for (infcodes.ts:367-387)
__device__ __forceinline__ void slow_step(Lane& L, const Tree& LL, const Tree& DD, const uint8_t* region) {
    br_refill(L);
    uint32_t pw = br_peek32(L);
    uint32_t rc = __builtin_bitreverse32(pw) >> 17;
    uint32_t v = tsel(LL, rc);
    bool bad = rc >= LL.lim[15];
    int32_t idx = bad ? (int32_t)(LL.pk[15] >> 16) - 32768 + (int32_t)rc : pk_rank(v, rc);
    int len = bad ? 15 : 15 - (int)(v & 15u);
    if (br_avail(L) < TREE_NEED(LL, len, idx)) { lane_stall(L, 1); return; }
    if (bad) { lane_fail(L, SDZ_DATA_ERROR, ZM_INVALID_LITLEN); return; }
    uint32_t b = region[idx];
    L.bo += (uint32_t)len;
    if (idx < (int32_t)((v >> 5) & 511u)) {
        if (L.room == 0) { lane_stall(L, 2); return; }
        L.room--;
        tok_lit(L, b);
        return;
    }
    if (b == 0) { L.mode = L.last ? LM_TRAILER : LM_TYPE; return; }
    if (b > 29) { lane_fail(L, SDZ_DATA_ERROR, ZM_INVALID_LITLEN); return; }
    uint32_t e;
    uint32_t mlen = len_base(b, e);
    if (br_avail(L) < (int)e) { lane_stall(L, 1); return; }
    mlen += (pw >> len) & ((1u << e) - 1u);
    L.bo += e;
    br_refill(L);
    pw = br_peek32(L);
    rc = __builtin_bitreverse32(pw) >> 17;
    v = tsel(DD, rc);
    bad = rc >= DD.lim[15];
    idx = bad ? (int32_t)(DD.pk[15] >> 16) - 32768 + (int32_t)rc : pk_rank(v, rc);
    len = bad ? 15 : 15 - (int)(v & 15u);
    if (br_avail(L) < TREE_NEED(DD, len, idx)) { lane_stall(L, 1); return; }
    if (bad) { lane_fail(L, SDZ_DATA_ERROR, ZM_INVALID_DIST); return; }
    uint32_t ds = region[IL_DSYM + idx];
    L.bo += (uint32_t)len;
    uint32_t dist = dist_base(ds, e);
    if (br_avail(L) < (int)e) { lane_stall(L, 1); return; }
    dist += (pw >> len) & ((1u << e) - 1u);
    L.bo += e;
    if (L.room < mlen) { lane_stall(L, 2); return; }
    L.room -= mlen;
    tok_match(L, mlen, dist);
}

// container header (inflate.ts:142-401; sd-inflate.ts:194-207 for AUTO)
__device__ __forceinline__ void parse_container(Lane& L, int32_t format, int32_t has_dict,
                                                int32_t dict_adler, uint64_t ilen) {
    bool raw = format == SDZ_FMT_RAW;
    if (format == SDZ_FMT_AUTO) {
        if (ilen < 2) { lane_fail(L, SDZ_TOO_SMALL, 0); return; }
        br_refill(L);
        uint32_t pw = br_peek32(L);
        uint32_t b0 = pw & 255u, b1 = (pw >> 8) & 255u;
        bool ident = (b0 == 0x78 && ((b0 << 8) + b1) % 31 == 0) || (b0 == 0x1f && b1 == 0x8b);
        raw = !ident;
    }
    if (raw) return;
    uint32_t b = 0, method = 0, flg = 0, v = 0;
    bool gz = false;
    if (!br_get(L, 8, b)) { lane_stall(L, 1); return; }
    if (b == 0x1f) {
        if (!br_get(L, 8, b)) { lane_stall(L, 1); return; }
        if (b != 0x8b) { lane_fail(L, SDZ_DATA_ERROR, ZM_INVALID_GZIP_ID); return; }
        gz = true;
        if (!br_get(L, 8, method)) { lane_stall(L, 1); return; }
    } else {
        method = b;
    }
    if ((method & 0xf) != 8) { lane_fail(L, SDZ_DATA_ERROR, ZM_UNKNOWN_METHOD); return; }
    if ((method >> 4) + 8 > 15) { lane_fail(L, SDZ_DATA_ERROR, ZM_INVALID_WINDOW); return; }
    if (!br_get(L, 8, flg)) { lane_stall(L, 1); return; }
    if (gz) {
        L.container = SDZ_CONTAINER_GZIP;
        uint32_t mt = 0;
        for (int k = 0; k < 4; ++k) {
            if (!br_get(L, 8, v)) { lane_stall(L, 1); return; }
            mt = (mt >> 8) | (v << 24);
        }
        L.mtime = (int32_t)mt;
        for (int k = 0; k < 2; ++k)
            if (!br_get(L, 8, v)) { lane_stall(L, 1); return; }
        if (flg & 4) { lane_fail(L, SDZ_TRUNCATED, 0); return; }   // inflate.ts:333-346 (EXTRA0 never advances): final
        if (flg & 8) {
            L.name_off = (uint32_t)(br_consumed(L) >> 3);
            for (;;) {
                if (!br_get(L, 8, v)) { lane_stall(L, 1); return; }
                if (v == 0) break;
                L.name_len++;
            }
        }
        if (flg & 16) {
            for (;;) {
                if (!br_get(L, 8, v)) { lane_stall(L, 1); return; }
                if (v == 0) break;
            }
        }
        if (flg & 2)
            for (int k = 0; k < 2; ++k)
                if (!br_get(L, 8, v)) { lane_stall(L, 1); return; }
    } else {
        L.container = SDZ_CONTAINER_ZLIB;
        if (((method << 8) + flg) % 31 != 0) { lane_fail(L, SDZ_DATA_ERROR, ZM_HEADER_CHECK); return; }
        if (flg & 0x20) {
            uint32_t id = 0;
            for (int k = 0; k < 4; ++k) {
                if (!br_get(L, 8, v)) { lane_stall(L, 1); return; }
                id = (id << 8) | v;
            }
            if (!has_dict) { lane_fail(L, SDZ_NEED_DICT, ZM_NEED_DICT); return; }
            if ((int32_t)id != dict_adler) { lane_fail(L, SDZ_DICT_MISMATCH, 0); return; }
            L.dict_used = 1;
        }
    }
}

// ------------------------------------------------------------------ cold path

// Everything but the symbol loop -- container header, block headers and tree
// building, stored blocks, the careful end-of-input symbol path -- on the state
// parked in the stream's DSave.  Returns when the lane can use the fast path
// again, has finished, or has filled its token ring.  Not inlined: its registers
// are its own, so the symbol loop keeps a small register footprint.
// MODE: 0 one-shot; 1 incremental (Inflater.append across calls: stall at the end of the
// input); 2 segment (block-parallel decode of a long stream, k_split.hip: start at a
// candidate block start, stop at a block boundary that is a candidate, or at the trailer)
struct SegStop {
    uint64_t start;                   // the segment's start bit
    const uint64_t* cand;             // its stream's sorted candidate block starts
    uint32_t ncand;
};
__device__ __forceinline__ bool seg_is_cand(const SegStop& G, uint64_t bit) {
    uint32_t lo = 0, hi = G.ncand;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (G.cand[mid] < bit) lo = mid + 1; else hi = mid;
    }
    return lo < G.ncand && G.cand[lo] == bit;
}

// n dwords src -> dst by one lane, 16 loads in flight: the lane-serial copies of a stream's symbol
// region and open token line between HBM and LDS waited one round trip per dword (~50 us of
// every k_inflate_wcold launch)
__device__ __forceinline__ void copy_dw(uint32_t* dst, const uint32_t* src, uint32_t n) {
    for (uint32_t k = 0; k < n; k += 16) {
        uint32_t v[16];
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) v[j] = k + j < n ? src[k + j] : 0u;
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j)
            if (k + j < n) dst[k + j] = v[j];
    }
}
__shared__ __attribute__((aligned(16))) uint8_t wd_region[IL_REGION];   // the wave decoder's symbol bytes
__shared__ Tree wd_LL, wd_DD;                     // ... and trees (from the stream's state)
// force_slow: decode the current block's symbols with the exact slow step to its end (the wave
// decoder's hand-back for errors, output room, tables past its LDS budget and the last input bits)
template <int MODE>
// inlined into its callers (k_inflate_decode's epochs, k_inflate_wcold): as a call it saved and
// restored ~180 VGPRs through scratch around every block-level step (832 B of scratch per lane);
// inlined, C2 decode 52.2 -> 51.5 ms and the 1,024-stream wave batch 3.19 -> 3.08 ms
// (tools/dbg/wdec_variant.sh).  IL_COLD_NOINLINE restores the call.
#ifdef IL_COLD_NOINLINE
#define IL_COLD_ATTR __noinline__
#else
#define IL_COLD_ATTR __forceinline__
#endif
__device__ IL_COLD_ATTR void cold_run(DSave* S, const uint8_t* inp, uint64_t ilen, uint64_t cap,
                                      uint32_t* tb, uint32_t tcap, uint8_t* lens, int32_t format, int32_t has_dict,
                                      int32_t dict_adler, uint32_t init, SegStop G, int force_slow = 0) {
    Lane L;
    Tree LL, DD;
    uint8_t* region = lane_region();
    L.ts = lane_stage();
    L.tb = tb; L.tcap = tcap; L.lens = lens;
#ifdef IL_HOT_CHECK
    L.chk_lo = (const uint8_t*)((uintptr_t)inp & ~(uintptr_t)15);
    L.chk_hi = inp + ilen + 64;
    L.chk_id = blockIdx.x * IL_STREAMS + lane_slot();
#endif
    L.streaming = MODE == 1; L.stall = 0; L.ubit = 0;
    if (init) {
        L.mode = LM_TYPE; L.last = 0; L.status = SDZ_OK; L.zmsg = 0; L.container = SDZ_CONTAINER_RAW;
        L.fixed = 0; L.nl = L.nd = 0; L.stored_ck = 0; L.stored_size = 0; L.mtime = 0;
        L.name_off = 0; L.name_len = 0; L.stored_left = 0; L.dict_used = 0;
        L.ntok = 0; L.litw = 0; L.nlit = 0; L.full = false;
        LL.l = DD.l = 0; LL.g = DD.g = 0; LL.kmin = DD.kmin = 1; LL.left = DD.left = 0;
        L.pos0 = 0;
        if (MODE == 2 && G.start) {
            br_init(L, inp, G.start, ilen * 8);           // a candidate block start: raw blocks
        } else {
            br_init(L, inp, 0, ilen * 8);
            parse_container(L, format, has_dict, dict_adler, ilen);
            if (L.stall) L.mode = LM_INIT;               // incremental: header not complete yet
        }
    } else {
        L.mode = S->mode; L.last = S->last; L.status = S->status; L.zmsg = S->zmsg;
        L.container = S->container; L.fixed = S->fixed; L.nl = S->nl; L.nd = S->nd;
        L.stored_ck = S->stored_ck; L.stored_size = S->stored_size; L.mtime = S->mtime;
        L.name_off = S->name_off; L.name_len = S->name_len; L.stored_left = S->stored_left;
        L.dict_used = S->dict_used;
        L.ntok = S->ntok; L.litw = S->litw; L.nlit = S->nlit; L.full = S->full != 0;
        br_init(L, inp, S->bitpos, ilen * 8);
        L.pos0 = S->pos;
        LL = S->LL; DD = S->DD;
    }
    uint64_t r = cap - L.pos0;
    L.room = L.room0 = (uint32_t)(r > 0x7fffffffull ? 0x7fffffffull : r);
    for (;;) {
        if (L.full || L.mode == LM_DONE || L.stall) break;
        if (MODE) L.ubit = br_consumed(L);
        if (MODE == 2) {                                  // a segment ends at the trailer, or at a candidate
            if (L.mode == LM_TRAILER) { L.stall = SEG_FINAL; break; }
            if (L.mode == LM_TYPE && L.ubit != G.start && seg_is_cand(G, L.ubit)) { L.stall = SEG_HANDOVER; break; }
        }
        if (L.mode == LM_CODES) {
            if (!force_slow && br_avail(L) >= 64 && (MODE != 1 || L.room >= 258)) break;   // hot_ready's preconditions
            slow_step(L, LL, DD, region);
            if (L.ntok + 3 > L.tcap) L.full = true;
        } else {
            force_slow = 0;                               // (the block it applied to has ended)
            block_step(L, LL, DD, region);
            if (L.avail0 - L.avail > (1 << 28)) L.full = true;   // keeps the saturated counter exact
        }
    }
    S->bitpos = L.stall ? L.ubit : br_consumed(L); S->pos = L.pos0 + (L.room0 - L.room);
    S->mode = L.mode; S->last = L.last; S->status = L.status; S->zmsg = L.zmsg;
    S->container = L.container; S->fixed = L.fixed; S->nl = L.nl; S->nd = L.nd;
    S->stored_ck = L.stored_ck; S->stored_size = L.stored_size; S->mtime = L.mtime;
    S->name_off = L.name_off; S->name_len = L.name_len; S->stored_left = L.stored_left;
    S->dict_used = L.dict_used;
    S->ntok = L.ntok; S->litw = L.litw; S->nlit = L.nlit; S->full = L.full ? 1 : 0;
    S->stall = L.stall;
    S->LL = LL; S->DD = DD;
}

// ------------------------------------------------------------------ hot path

__device__ __forceinline__ void hot_load(Hot& H, HTree& LL, HTree& DD, const DSave* S,
                                         const uint8_t* inp, uint64_t ilen, uint64_t cap) {
#ifdef IL_HOT_CHECK
    H.chk_lo = (const uint8_t*)((uintptr_t)inp & ~(uintptr_t)15);
    H.chk_hi = inp + ilen + 64;                           // the batch's readable slack
    H.chk_id = blockIdx.x * IL_STREAMS + lane_slot();
    {
        const uint8_t* a = (const uint8_t*)(((uintptr_t)(inp + (S->bitpos >> 3))) & ~(uintptr_t)15);
        if (!HOT_CHECK(H, S->bitpos <= ilen * 8 && a >= H.chk_lo && a + 64 <= H.chk_hi + 16, 3,
                       S->bitpos, ilen)) {
            H.mode = LM_DONE;
            return;
        }
    }
#endif
    IL_BR_INIT(H, inp, S->bitpos, ilen * 8, lane_ring());
    H.vend = (g_uint4*)(((uintptr_t)(inp + ilen) + 15) & ~(uintptr_t)15);
    H.pos0 = S->pos;
    uint64_t r = cap - H.pos0;
    H.room = H.room0 = (uint32_t)(r > 0x7fffffffull ? 0x7fffffffull : r);
    H.mode = S->mode; H.last = S->last; H.status = S->status; H.zmsg = S->zmsg;
    H.ntok = S->ntok; H.litw = S->litw; H.nlit = S->nlit; H.full = S->full != 0;
    H.nfl = H.ntok & ~(IL_TSTAGE - 1u);                   // (the stage holds the open line)
    LL = (const HTree&)S->LL;
    DD = (const HTree&)S->DD;
}
__device__ __forceinline__ void hot_save(const Hot& H, DSave* S) {
    S->bitpos = br_consumed(H); S->pos = H.pos0 + (H.room0 - H.room);
    S->mode = H.mode; S->last = H.last; S->status = H.status; S->zmsg = H.zmsg;
    S->ntok = H.ntok; S->litw = H.litw; S->nlit = H.nlit; S->full = H.full ? 1 : 0;
}
// one symbol step reads at most 48 bits and writes at most 258 bytes; below either
// bound the cold path's exact end-of-input / end-of-room handling takes over.  The room
// bound applies to incremental streams only (STREAM: 258 bytes), which must stop at a
// symbol's start when out_cap is reached; a one-shot stream (or segment) keeps the last
// symbols of an exactly sized output slot in the hot loop, whose own room check ends it
// OUT_OVERFLOW.  (Leaving those symbols to the cold code too, so that the loop needs no room
// checks, was measured: the extra cold epoch at every stream's end cost 3 ms of the
// distinct streams' 14.)
#if IL_REFILL2
#define IL_HOT_AVAIL br_avail2
#else
#define IL_HOT_AVAIL br_avail
#endif
template <bool STREAM>
__device__ __forceinline__ bool hot_ready(const Hot& H) {
    return H.mode == LM_CODES && !H.full && IL_HOT_AVAIL(H) >= 64 && (!STREAM || H.room >= 258);
}
template <int MODE>
__device__ __forceinline__ bool can_hot(const DSave* S, uint64_t tbits, uint64_t cap) {
    return S->mode == LM_CODES && !S->full && tbits - S->bitpos >= 64 && (MODE == 0 || !S->stall) &&
           (MODE != 1 || cap - S->pos >= 258);
}

// one epoch of the symbol loop: every lane with `hot` set decodes until no more
// than `stop` lanes of the wave can continue.  Not inlined, so that its register
// allocation is not shaped by the cold call in the caller's loop.  IL_HOT_INLINE inlines it
// (development variant).
#ifdef IL_HOT_INLINE
#define IL_HOT_ATTR __forceinline__
#else
#define IL_HOT_ATTR __noinline__
#endif
template <bool STREAM>
__device__ IL_HOT_ATTR void hot_epoch(DSave* S, const uint8_t* inp, uint64_t ilen, uint64_t cap,
                                       uint32_t* tb, uint32_t tcap, bool hot, int stop) {
    Hot H;
    HTree LL, DD;
    const uint8_t* region = lane_region();
    // lanes without a stream in this epoch: every field the loop body may touch is defined
    // (mode DONE and full keep them out of the symbol steps; ring_step is not run for them)
    H.mode = LM_DONE; H.full = true; H.ntok = 0; H.nfl = 0; H.tcap = tcap; H.tb = tb; H.ts = lane_stage();
    H.avail = 0; H.bo = 0; H.avail0 = 0; H.base_bit = 0; H.room = H.room0 = 0; H.pos0 = 0;
    H.last = 0; H.status = SDZ_OK; H.zmsg = 0; H.litw = 0; H.nlit = 0;
    H.w0 = H.w1 = H.w2 = H.nx = H.nx2 = 0; H.rpos = H.wpos = 0; H.ns = 0; H.arp = 0;
    H.s0 = H.s1 = make_uint4(0u, 0u, 0u, 0u);
    H.vp = H.vend = (g_uint4*)inp; H.ring = lane_ring();
#ifdef IL_HOT_CHECK
    H.chk_lo = H.chk_hi = nullptr; H.chk_id = ~0u;
#endif
    if (hot) {
        hot_load(H, LL, DD, S, inp, ilen, cap);
#if IL_OPEN_SLOT && IL_UNIFORM_FLUSH
        // literals left pending by the cold code: their token into its slot (see tok_lit)
        if (H.nlit) H.ts[H.ntok & (IL_TSTAGE - 1)] = ((H.nlit - 1u) << 24) | H.litw;
#endif
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) { LL.lim[k] = DD.lim[k] = 0; }
#pragma unroll
        for (int k = 0; k < 17; ++k) { LL.pk[k] = DD.pk[k] = 0; }
    }
#if IL_BSEARCH
#pragma unroll
    for (int k = 1; k <= 15; ++k) { LL.lim[k] -= 1u; DD.lim[k] -= 1u; }   // tsel_hot's form
#endif
#ifndef IL_REP_UNROLL
#define IL_REP_UNROLL 4                   // the 4 steps between ring steps, unrolled (C2 decode -3 %)
#endif
    // every lane runs the ring step: an idle lane's (vp == vend, ns 0, no tokens) changes
    // nothing.  Under `if (hot)` its reader fields were dead on the idle path, which LLVM then
    // fed as undef into the loop's phis (seen in the IR of the hot_epoch-inlined variant that
    // faulted in round 4); here every value the loop reads is defined for every lane
#if IL_UNCHECKED_RUN && IL_FULL_AT_RING && IL_TWO_LOOPS
    // Two loops in sequence: the first runs 4 steps without their bit and room checks as long as
    // every lane that can step has the input bits and the output room for 4 steps of up to 48 bits
    // and 258 bytes each (a step then only tests that its lane is still in the block); once some lane
    // has not, the rest of the epoch runs checked steps.  (One loop with both bodies merged their
    // values at its back edge: ~20 register copies per 4 steps.)
    // the exit test's count against a scalar (`stop` arrives in a VGPR: the loop's exit was a
    // divergent-looking test with exec-mask bookkeeping), and the readiness it computes is the next
    // run's (the ring step changes none of its inputs; the token-room check moves before it)
    const int stop_s = __builtin_amdgcn_readfirstlane(stop);
    bool more = true;
    if (H.ntok + 3u + 8u > H.tcap) H.full = true;         // token room, once per 4 steps: <= 2 tokens per step
    bool rdy = hot_ready<STREAM>(H);
    for (;;) {
        IL_RING_STEP(H);
        if (__ballot(rdy && !(IL_HOT_AVAIL(H) >= 64 + 3 * 48 && H.room >= 4u * 258u))) break;
#pragma unroll
        for (int rep = 0; rep < 4; ++rep)
            if (rdy && H.mode == LM_CODES) IL_FAST_STEP<false>(H, LL, DD, region);
        if (H.ntok + 3u + 8u > H.tcap) H.full = true;
        rdy = hot_ready<STREAM>(H);
        if ((int)__popcll(__ballot(rdy)) <= stop_s) { more = false; break; }
    }
    while (more) {
#pragma unroll IL_REP_UNROLL
        for (int rep = 0; rep < 4; ++rep)
            if (hot_ready<STREAM>(H)) IL_FAST_STEP(H, LL, DD, region);
        if (H.ntok + 3u + 8u > H.tcap) H.full = true;
        if ((int)__popcll(__ballot(hot_ready<STREAM>(H))) <= stop_s) break;
        IL_RING_STEP(H);
    }
#else
    do {
        IL_RING_STEP(H);
#if IL_FULL_AT_RING
        // token room checked once per 4 steps: at most 2 tokens per step
        if (H.ntok + 3u + 8u > H.tcap) H.full = true;
#endif
#if IL_UNCHECKED_RUN && IL_FULL_AT_RING
        // when every lane that can step has the input bits and the output room for 4 steps of up
        // to 48 bits and 258 bytes each, the 4 steps run without their bit and room checks; a
        // step then only tests that its lane is still in the block (an end of block or an error
        // in an earlier step ends it)
        const bool rdy = hot_ready<STREAM>(H);
        if (!__ballot(rdy && !(IL_HOT_AVAIL(H) >= 64 + 3 * 48 && H.room >= 4u * 258u))) {
#pragma unroll
            for (int rep = 0; rep < 4; ++rep)
                if (rdy && H.mode == LM_CODES) IL_FAST_STEP<false>(H, LL, DD, region);
        } else
#endif
        {
#pragma unroll IL_REP_UNROLL
        for (int rep = 0; rep < 4; ++rep) {
            if (hot_ready<STREAM>(H)) {
                IL_FAST_STEP(H, LL, DD, region);
#if !IL_FULL_AT_RING
                if (H.ntok + 3 > H.tcap) H.full = true;
#endif
            }
        }
        }
    } while (__popcll(__ballot(hot_ready<STREAM>(H))) > stop);
#endif
    // back to the cold code's invariant: everything below the open 32-token line in HBM
    // (nfl >= ntok - 15 after this, and a multiple of 16)
    tok_flush_hot(H);
#if IL_REFILL2
    br_sync2(H);
    hot_fix_status(H);
#endif
    if (hot) hot_save(H, S);
}

template <int MODE>
__device__ __forceinline__ void epochs(const InflateArgs& A, DSave* S, const uint8_t* inp, uint64_t ilen,
                                       uint64_t cap, uint32_t* tb, uint32_t tcap, uint8_t* lens, bool live,
                                       SegStop G) {
    const uint64_t tbits = ilen * 8;
#ifdef SDZ_TIMING
    // development: wave clocks of the cold (block-level) and hot (symbol) parts, waves of the
    // first 8 workgroups (dbg[8..11]: cold cycles, hot cycles, cold runs, hot epochs)
    const bool timed = A.dbg && blockIdx.x < 8 && (threadIdx.x & 63u) == 0;
    unsigned long long tc = 0, th = 0, nc = 0, nh = 0, t0 = timed ? clock64() : 0;
#endif
    for (;;) {
        bool hot = live && can_hot<MODE>(S, tbits, cap);
        bool cold = live && !S->full && S->mode != LM_DONE && !hot && (MODE == 0 || !S->stall);
        if (__ballot(cold)) {
            if (cold)
                cold_run<MODE>(S, inp, ilen, cap, tb, tcap, lens, A.format, A.dict != nullptr, dict_id_of(A.dict_adler, A.dict_adler_dev),
                               MODE == 1 && S->mode == LM_INIT ? 1u : 0u, G);
            hot = live && can_hot<MODE>(S, tbits, cap);
#ifdef SDZ_TIMING
            if (timed) { const unsigned long long t = clock64(); tc += t - t0; t0 = t; ++nc; }
#endif
        }
        uint64_t hm = __ballot(hot);
        if (hm == 0) break;
        int nhot = __popcll(hm);
        hot_epoch<MODE == 1>(S, inp, ilen, cap, tb, tcap, hot, nhot - (nhot >= 16 ? nhot >> IL_STOP_SHIFT : 1));
#ifdef SDZ_TIMING
        if (timed) { const unsigned long long t = clock64(); th += t - t0; t0 = t; ++nh; }
#endif
    }
#ifdef SDZ_TIMING
    if (timed) { atomicAdd(&A.dbg[8], tc); atomicAdd(&A.dbg[9], th); atomicAdd(&A.dbg[10], nc); atomicAdd(&A.dbg[11], nh); }
#endif
}

// One lane per stream; in segment mode (A.segmode, k_split.hip) one lane per segment of a
// long stream, in one round, into the segment's own token buffer.  Streams whose tokens
// the segments provide (A.split_state) are skipped: k_seg_feed fills their rounds.
__global__ __launch_bounds__(IL_THREADS, 1) void k_inflate_decode(InflateArgs A, uint32_t round) {
    uint8_t* region = lane_region();
    uint32_t* ts = lane_stage();
#ifdef IL_LDS_POISON
    {   // development: this lane's LDS (symbol region, token stage, input ring) starts as 0xA5 bytes, so a
        // read before a write sees the same value whatever ran on the CU before
        for (uint32_t k = 0; k < IL_REGION / 4; ++k) ((uint32_t*)region)[k] = 0xA5A5A5A5u;
        for (uint32_t k = 0; k < IL_TSTRIDE / 4; ++k) ts[k] = 0xA5A5A5A5u;
        for (uint32_t k = 0; k < IL_RING_STRIDE; ++k) lane_ring()[k] = 0xA5A5A5A5u;
    }
#endif
    uint32_t gid = blockIdx.x * IL_STREAMS + lane_slot();
    bool valid = gid < A.n && (threadIdx.x & 63u) < IL_WAVE_LANES;
    uint32_t sid = valid ? gid : 0u;
    if (valid && A.split_state) {                        // split streams: see split.h
        const uint32_t st = A.split_state[sid];
        valid = A.fallback_pass ? st == SPS_FALLBACK : (st == 0 || st == SPS_FALLBACK);
    }
    const uint32_t xid = A.segmode ? A.seg[sid].stream : sid;           // the stream of the input
    DSave* S = (DSave*)A.dsave + sid;
    uint32_t* tb = A.segmode ? A.segtok + A.seg[sid].tok : A.tokens + (uint64_t)sid * A.round_tokens;
    const uint32_t tcap = A.segmode ? A.seg[sid].cap : A.round_tokens;
    uint8_t* lens = A.scratch + (uint64_t)sid * kInflateScratchPerStream;
    SegStop G = { 0, nullptr, 0 };
    if (A.segmode) {
        const uint32_t k = A.seg[sid].split;
        const uint32_t nc = A.spinfo[k].ncand;
        G.start = A.seg[sid].bit;
        G.cand = A.cand + (uint64_t)k * SP_CAND_MAX;
        G.ncand = nc < SP_CAND_MAX ? nc : SP_CAND_MAX;
    }
    const uint8_t* inp = A.in;
    uint64_t ilen = 0, cap = 0;
    bool live = false;
    if (valid) {
        inp = A.in + A.in_off[xid];
        ilen = A.in_len[xid];
        cap = A.out_cap[xid];
        // a call's first round starts a stream (one-shot, or an incremental stream whose
        // header is still incomplete) or resumes it (later rounds; incremental calls)
        const bool resume = round > 0 || (A.streaming && S->mode != LM_INIT);
        if (round == 0 && (A.out_off[xid] & 7)) {
            S->mode = LM_DONE; S->status = SDZ_BAD_RECORD; S->zmsg = 0; S->bitpos = 0; S->pos = 0;
            S->container = SDZ_CONTAINER_RAW; S->stored_ck = 0; S->stored_size = 0; S->mtime = 0;
            S->name_off = 0; S->name_len = 0; S->dict_used = 0; S->ntok = 0; S->litw = 0;
            S->nlit = 0; S->full = 0; S->stall = 0;
        } else if (!resume) {
            live = true;
            if (A.streaming) cold_run<1>(S, inp, ilen, cap, tb, tcap, lens, A.format,
                                         A.dict != nullptr, dict_id_of(A.dict_adler, A.dict_adler_dev), 1u, G);
            else if (A.segmode) cold_run<2>(S, inp, ilen, cap, tb, tcap, lens, A.format,
                                            A.dict != nullptr, dict_id_of(A.dict_adler, A.dict_adler_dev), 1u, G);
            else cold_run<0>(S, inp, ilen, cap, tb, tcap, lens, A.format,
                             A.dict != nullptr, dict_id_of(A.dict_adler, A.dict_adler_dev), 1u, G);
        } else if (S->mode != LM_DONE && !(round > 0 && S->stall)) {
            live = true;
            copy_dw((uint32_t*)region, (const uint32_t*)S->region, IL_REGION / 4);
            S->ntok = 0; S->full = 0;
            if (round == 0) { S->pos = 0; S->stall = 0; }      // a new call: fresh output slot
        }
    }
    // epochs: lanes that need block-level work do it together (cold_run), then
    // every lane that can decodes symbols with register-resident state until all of them
    // have left the fast path (IL_STOP_SHIFT); state is parked in DSave in between
    if (A.streaming) epochs<1>(A, S, inp, ilen, cap, tb, tcap, lens, live, G);
    else if (A.segmode) epochs<2>(A, S, inp, ilen, cap, tb, tcap, lens, live, G);
    else epochs<0>(A, S, inp, ilen, cap, tb, tcap, lens, live, G);

    bool more = live && S->mode != LM_DONE && !S->stall;
    uint64_t mm = __ballot(more);                        // one counter update per wave
    if (mm && (threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(mm)) atomicAdd(A.active, (uint32_t)__popcll(mm));
    if (!live) {
        if (valid) { A.ntok[sid] = 0; A.flags[sid] = 2; }
        return;
    }
    {
        Core H;                                          // flush the token stage
        H.tb = tb; H.ts = ts; H.ntok = S->ntok; H.litw = S->litw; H.nlit = S->nlit; H.tcap = tcap;
#ifdef IL_HOT_CHECK
        H.chk_lo = H.chk_hi = nullptr; H.chk_id = sid;
#endif
        tok_finish(H);
        S->ntok = H.ntok; S->litw = 0; S->nlit = 0;
        A.ntok[sid] = H.ntok;
    }
    // 0: more rounds; 1: finished this round; 3+: stalled (incremental: done for this call;
    // segment: handed over or reached the trailer)
    A.flags[sid] = S->mode == LM_DONE ? 1u : S->stall ? 3u : 0u;
    if (S->mode != LM_DONE && !A.segmode)
        copy_dw((uint32_t*)S->region, (const uint32_t*)region, IL_REGION / 4);
}

// ------------------------------------------------------------------ wave decoder
//
// k_inflate_wdec: one WAVE per stream.  Huffman codes resynchronise: decoding a block from a
// bit offset that is not a symbol start falls onto the true symbol boundaries after a few
// symbols (on text: median 6, 99.9 % within 76 symbols / 1,058 bits, measured on
// paradiselost slices).  So an iteration cuts the current block's bits from the known
// position B0 into up to 64 chunks of C bits, and lane j decodes chunk j speculatively with
// the block's tables:
//   - lane j > 0 records the symbol starts of its first WD_W bits in an LDS bitmap and emits
//     one token per symbol there (so that the token index at a recorded start is the number
//     of recorded starts before it);
//   - past its chunk's end, lane j keeps decoding until it stands on a symbol start that
//     lane j + 1 recorded (SYNC): from there both decode the same symbols, so lane j stops
//     and lane j + 1's tokens from that index on are the true ones;
//   - a lane also stops at an end of block (EOB), an invalid code (ERR), its token capacity
//     (CAP), the last 64 input bits (END), or WD_W bits past its chunk without a sync (NOSYNC).
// Lane 0 starts on a true symbol start, so the lanes 0..J linked by SYNCs decode exactly the
// serial symbol sequence, J being the first lane that stopped otherwise; the stream goes on
// from J's stop position.  Their tokens are compacted (in place, downwards) to the stream's
// token ring, where k_inflate_resolve reads them as from k_inflate_decode.
// Everything that is not the symbol loop of a Huffman block -- container header, block
// headers and trees, stored blocks, trailer, the last input bits, and the exact handling of
// errors and output room (a room overflow or an ERR hands the block to the slow step from
// the iteration's start) -- is cold_run<0> in k_inflate_wcold, a lane per stream.
// Decoding uses two-level lookup tables in LDS (root 10 / 8 bits, built from the canonical
// trees by the whole wave) instead of the lane-per-stream decoder's table-free registers: a
// wave holds one stream, and its latency is hidden by the other waves on the SIMD.
#ifndef WD_W
#define WD_W 1024                 // bits of a lane's boundary map
#endif
#define WD_BMW (WD_W / 32)
#define WD_BMS (WD_BMW + 1)       // a lane's map stride: odd, so that lanes at one offset hit 32 banks
#ifndef WD_CAP
#define WD_CAP 512                // provisional tokens per lane and iteration
#endif
// the runtime sizes each stream's provisional slots (kWdProvTokens) for 64 lanes x WD_CAP tokens
// plus one dummy slot per lane (the compaction's masked-off stores)
static_assert(kWdProvTokens >= 64ull * WD_CAP + 64ull, "kWdProvTokens (sdz_internal.h) too small for WD_CAP");
#ifndef WD_LLR
#define WD_LLR 10                 // root bits of the literal/length table
#define WD_DR 8                   // ... of the distance table
#define WD_LLT 1536               // table entries (root + subtables)
#define WD_DT 736                 // (6 waves per CU: the LDS total stays below 160 KiB / 6)
#endif
#ifndef WD_CMAX
#define WD_CMAX 4096              // chunk bits
#endif
#define WD_CMIN 256
#define WD_MINSPEC 512            // bits past the last-64 reserve below which lane 0 runs the slow step
#define WD_TST 16                 // token stage per lane (LDS)
#define WD_INV 511u               // table symbol: invalid code
#ifndef WD_WPE
#define WD_WPE 2                  // waves per SIMD the register budget is sized for (<= 256 VGPRs)
#endif

__shared__ __attribute__((aligned(16))) uint32_t wd_tab[WD_LLT + WD_DT];   // literal/length, then distance
#define wd_ll wd_tab
#define wd_dt (wd_tab + WD_LLT)
__shared__ __attribute__((aligned(16))) uint32_t wd_bm[64 * WD_BMS];
__shared__ __attribute__((aligned(16))) uint32_t wd_ring[64 * 18];
// token stage: WD_TST slots + a dummy slot (stores that do not push) per lane; the odd stride puts
// the lanes' flush reads at one slot on 32 banks
#define WD_TSS (WD_TST + 1)
__shared__ __attribute__((aligned(16))) uint32_t wd_tst[64 * WD_TSS];

enum : uint32_t { WR_RUN = 0, WR_SYNC, WR_EOB, WR_ERR, WR_CAP, WR_END, WR_NOSYNC, WR_CHUNK, WR_OFF };

template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t wd_dpp_add(uint32_t x) {
    return x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ uint32_t wd_scan(uint32_t x) {   // inclusive wave scan (DPP)
    x = wd_dpp_add<0x111, 0xf>(x);
    x = wd_dpp_add<0x112, 0xf>(x);
    x = wd_dpp_add<0x114, 0xf>(x);
    x = wd_dpp_add<0x118, 0xf>(x);
    x = wd_dpp_add<0x142, 0xa>(x);
    x = wd_dpp_add<0x143, 0xc>(x);
    return x;
}
__device__ __forceinline__ uint32_t wd_uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint32_t wd_at(uint32_t x, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l); }

// table symbol of the code with 15-bit MSB-first prefix rc (low bits zero past the code's
// length), and that length: literals 0-255, 256 end of block, 257-285 lengths, distance
// symbols 0-29, WD_INV for codes past the tree's last code and the invalid symbols
__device__ __forceinline__ uint32_t wd_code(const HTree& T, const uint8_t* syms, bool lit, uint32_t rc, uint32_t& len) {
    if (rc >= T.lim[15]) { len = 15; return WD_INV; }
    const uint32_t v = tsel(T, rc);
    const int32_t idx = pk_rank(v, rc);
    len = 15u - (v & 15u);
    if (lit) {
        if (idx >= 288) return WD_INV;
        const uint32_t b = syms[idx];
        if (idx < (int32_t)((v >> 5) & 511u)) return b;
        return b >= 30 ? WD_INV : 256u + b;              // symbols 286, 287 (fixed tree): invalid
    }
    if (idx >= 30) return WD_INV;
    return syms[IL_DSYM + idx];
}
// A decoded code as the symbol loop uses it: code length (bits 0-3), extra bits (4-7), kind
// (8-9: 0 literal, 1 length, 2 distance, 3 end of block (value 0) or invalid code (value 1)) and
// value (16-31: the literal, or the base length / distance the extra bits are added to)
__device__ __forceinline__ uint32_t wd_entry(uint32_t sym, uint32_t len, bool lit) {
    uint32_t x, kind, val;
    if (lit) {
        if (sym < 256u) { kind = 0u; val = sym; x = 0u; }
        else if (sym == 256u) { kind = 3u; val = 0u; x = 0u; }
        else if (sym <= 285u) { kind = 1u; val = len_base(sym - 256u, x); }
        else { kind = 3u; val = 1u; x = 0u; }
    } else if (sym < 30u) { kind = 2u; val = dist_base(sym, x); }
    else { kind = 3u; val = 1u; x = 0u; }
    return len | (x << 4) | (kind << 8) | (val << 16);
}
// Two-level table of wd_entry words: a root entry is the code's (direct), or 0x8000 | k | off << 16
// (codes longer than R bits under this prefix: a subtable of 2^k entries at off, k = the longest
// code's length - R).  Returns false if the subtables do not fit (the block then runs the slow step).
template <int R>
__device__ __forceinline__ bool wd_table(const HTree& T, const uint8_t* syms, bool lit, uint32_t* tab, uint32_t cap) {
    const uint32_t lane = threadIdx.x & 63u;
    constexpr uint32_t NR = 1u << R, PER = NR / 64;
    uint32_t need = 0;
    uint32_t ks[PER];
#pragma unroll
    for (uint32_t m = 0; m < PER; ++m) {
        const uint32_t i = lane + 64u * m;
        const uint32_t rc = __builtin_bitreverse32(i) >> 17;
        uint32_t len, k = 0;
        uint32_t sym = wd_code(T, syms, lit, rc, len);
        if (rc < T.lim[15] && len > R) {
            uint32_t lm;
            (void)wd_code(T, syms, lit, rc | ((1u << (15 - R)) - 1u), lm);
            k = lm - R;
            need += 1u << k;
        } else if (rc >= T.lim[15]) {
            len = 1;                                      // every code under this prefix is invalid
            sym = WD_INV;
        }
        ks[m] = k;
        if (k == 0) tab[i] = wd_entry(sym, len, lit);
    }
    const uint32_t incl = wd_scan(need);
    const uint32_t total = wd_at(incl, 63);
    if (NR + total > cap) return false;
    uint32_t off = NR + incl - need;
#pragma unroll
    for (uint32_t m = 0; m < PER; ++m) {
        const uint32_t k = ks[m];
        if (k == 0) continue;
        const uint32_t i = lane + 64u * m;
        tab[i] = 0x8000u | k | (off << 16);
        for (uint32_t j = 0; j < (1u << k); ++j) {
            uint32_t len;
            const uint32_t x = i | (j << R);
            const uint32_t sym = wd_code(T, syms, lit, __builtin_bitreverse32(x) >> 17, len);
            tab[off + j] = wd_entry(sym, len, lit);
        }
        off += 1u << k;
    }
    return true;
}
// both tables from the trees in wd_tree and the symbol bytes in wd_region (whole wave)
__device__ __noinline__ bool wd_build() {
    HTree LL, DD;
#pragma unroll
    for (int k = 0; k < 16; ++k) { LL.lim[k] = wd_LL.lim[k]; DD.lim[k] = wd_DD.lim[k]; }
#pragma unroll
    for (int k = 0; k < 17; ++k) { LL.pk[k] = wd_LL.pk[k]; DD.pk[k] = wd_DD.pk[k]; }
    const bool a = wd_table<WD_LLR>(LL, wd_region, true, wd_ll, WD_LLT);
    const bool b = wd_table<WD_DR>(DD, wd_region, false, wd_dt, WD_DT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    return a && b;
}


struct WdRes {
    uint32_t st, stop, ntk, synco;
};

// One speculative iteration of the current block from S->bitpos (all of the wave; see the
// head comment).  Commits the chained lanes' tokens and the stream position to S (lane 0).
// Returns 0: go on; 1: the block ended, or the last input bits need the cold path; 2: the
// slow step must take this block from S->bitpos (an invalid code, or the output room);
// 3: no token room left this round.  cmax: chunk bits (halved on CAP stops).
__device__ __noinline__ int wd_iteration(DSave* S, const uint8_t* inp, uint64_t ilen, uint64_t cap,
                                         uint32_t* tb, uint32_t tcap, uint32_t* pv, uint64_t B0, uint32_t ntok0, uint64_t pos0,
                                         uint32_t& cmax, unsigned long long* dbg) {
    const uint32_t lane = threadIdx.x & 63u;
#ifdef SDZ_TIMING
    // development: dbg[18] loop cycles, [19] join cycles, [20] iterations, [21] CAP stops of J,
    // [22] symbol steps of all lanes, [23] tokens committed, [24] chained lanes, [25] lanes used,
    // [26] ERR / [27] NOSYNC / [28] EOB stops of J, [30] chunk bits (sum)
    const unsigned long long tw0 = dbg ? clock64() : 0;
    uint32_t nsym = 0;
#endif
    const uint64_t tbits = ilen * 8;
    const uint64_t lim64 = tbits - 64 - B0;
    const uint32_t lim = (uint32_t)(lim64 > (1ull << 30) ? (1ull << 30) : lim64);
    // chunks of C bits covering [0, lim) when 64 of them can (lanes past the block's end decode
    // nothing of use; CMAX x 64 bits is about one block of 16 Ki symbols of text)
    uint32_t C = (lim + 63u) / 64u;
    C = C < WD_CMIN ? WD_CMIN : C > cmax ? cmax : C;
    uint32_t n = (lim + C - 1u) / C;
    n = n < 1u ? 1u : n > 64u ? 64u : n;
    const uint32_t space = tcap > ntok0 + 8u ? tcap - ntok0 - 8u : 0u;   // ring room for the chained tokens
    if (space < 64u) return 3;
    if (space / n < 64u) n = space / 64u;
    uint32_t tcapl = space / n;
    tcapl = (tcapl > WD_CAP ? WD_CAP : tcapl) & ~7u;

    const bool on = lane < n;
    const bool lastl = lane == n - 1u;
    const uint32_t bj = lane * C;
    const uint32_t bn = lastl ? n * C : (lane + 1u) * C;
    uint32_t* bm = wd_bm + lane * WD_BMS;
    uint32_t* bmn = wd_bm + ((lane + 1u) & 63u) * WD_BMS;
    uint32_t* tst = wd_tst + lane * WD_TSS;
    uint32_t* tdum = tst + WD_TST;
    GLB uint32_t* prov = (GLB uint32_t*)(pv + lane * tcapl);
#pragma unroll
    for (int k = 0; k < WD_BMW; ++k) bm[k] = 0u;

    Hot H;
    H.ring = wd_ring + lane * 18u;
    uint32_t Kc = 0;
    if (on) {
        br_init(H, inp, B0 + bj, tbits, H.ring);
        H.vend = (g_uint4*)(((uintptr_t)(inp + ilen) + 15) & ~(uintptr_t)15);
        Kc = (uint32_t)(H.base_bit - B0) + (uint32_t)H.avail0;   // rel = Kc - avail + bo
    } else {
        H.ns = 0; H.vp = H.vend = nullptr; H.wpos = H.rpos = 0; H.avail = 0; H.bo = 0;
    }
    uint32_t st = on ? WR_RUN : WR_OFF;
    uint32_t prog = on ? 0u : 0x80000000u;                // offset recorded so far | stopped
    uint32_t ntk = 0, nfl = 0, litw = 0, nlit = 0, stop = 0, synco = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_wave_barrier();

    auto push = [&](uint32_t t) { tst[ntk & (WD_TST - 1)] = t; ntk++; };
#ifndef SDZ_TIMING
    uint32_t nsym = 0;
#endif
    // one code from table `tbase` (root bits rb) at peek pw: the root word, or its subtable's
    // (a wave-uniform branch, taken when some lane's code is longer than the root)
    auto look = [&](uint32_t tbase, uint32_t rb, uint32_t pw, uint32_t act) -> uint32_t {
        uint32_t e = wd_tab[tbase + (pw & ((1u << rb) - 1u))];
        if (__ballot(act & (e >> 15) & 1u))
            if (e & 0x8000u) e = wd_tab[tbase + (e >> 16) + ((pw >> rb) & ((1u << (e & 15u)) - 1u))];
        return e;
    };

    // One symbol per step, the same instructions on every lane: the literal/length code, then a
    // distance code decoded for every lane (some lane of 64 almost always has a match) and used by
    // the lanes that have one; kind, extra bits and base value come with the table words.  Flags
    // are 0/1 integers combined with & and | (short-circuit && and || compile to exec-mask
    // branches).  Stops at a symbol start (chunk end, sync, input end, token room) are checked
    // only in 4-step groups where some lane may reach one (CAREFUL); end of block and invalid
    // codes in every step.
    auto step = [&](auto carefulc, uint32_t spv, uint32_t sstop) {
        constexpr bool CAREFUL = decltype(carefulc)::value;
        const uint32_t run = st == WR_RUN;
        const uint32_t pw = br_refill_peek(H);            // (a refill never moves the position)
        const uint32_t p = Kc - (uint32_t)H.avail + H.bo;
        const uint32_t off = p - bj;
        uint32_t dec = run;
        if constexpr (CAREFUL) {
            const uint32_t past = run & (p >= bn);
            const uint32_t o = p - bn;
            const uint32_t inw = past & (uint32_t)!lastl & (o < WD_W);
            const uint32_t chk = inw & (o <= spv);
            const uint32_t bw = bmn[chk ? (o >> 5) : 0u];
            const uint32_t syn = chk & ((bw >> (o & 31u)) & 1u);
            const uint32_t waitS = inw & (o > spv) & (sstop ^ 1u);
            const uint32_t nosync = past & (uint32_t)!lastl & (syn ^ 1u) & ((o >= WD_W) | ((o > spv) & sstop));
            const uint32_t why = !run ? (uint32_t)WR_RUN : p >= lim ? (uint32_t)WR_END : ntk + 3u > tcapl ? (uint32_t)WR_CAP
                               : !past ? (uint32_t)WR_RUN : lastl ? (uint32_t)WR_CHUNK : syn ? (uint32_t)WR_SYNC
                               : nosync ? (uint32_t)WR_NOSYNC : (uint32_t)WR_RUN;
            const uint32_t halt = run & (why != WR_RUN);
            dec = run & (why == WR_RUN) & (waitS ^ 1u);
            st = halt ? why : st;
            stop = halt ? p : stop;
            synco = halt ? o : synco;
            prog |= halt << 31;
        }
        // record our symbol starts in the first WD_W bits (an OR of 0 elsewhere)
        const uint32_t head = (lane != 0u) & (off < WD_W);
        const uint32_t rec = dec & head;
        __hip_atomic_fetch_or(bm + (rec ? off >> 5 : 0u), rec << (off & 31u), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_WORKGROUP);
        prog = run ? (off | (prog & 0x80000000u)) : prog;
        nsym += dec;
        // the literal/length code
        const uint32_t e = look(0u, WD_LLR, pw, dec);
        const uint32_t len = e & 15u, xb = (e >> 4) & 15u, kind = (e >> 8) & 3u;
        const uint32_t val = (e >> 16) + __builtin_amdgcn_ubfe(pw, len, xb);
        const uint32_t isLit = kind == 0u, isLen = kind == 1u, isSp = kind == 3u;
        H.bo += (dec & (isSp ^ 1u)) ? len + xb : 0u;
        // the distance code (every lane; used by the lanes at a length code)
        const uint32_t pw2 = br_refill_peek(H);
        const uint32_t d = look(WD_LLT, WD_DR, pw2, dec & isLen);
        const uint32_t dlen = d & 15u, dxb = (d >> 4) & 15u;
        const uint32_t dist = (d >> 16) + __builtin_amdgcn_ubfe(pw2, dlen, dxb);
        const uint32_t derr = isLen & (((d >> 8) & 3u) != 2u);
        const uint32_t isM = isLen & (derr ^ 1u);
        H.bo += (dec & isM) ? dlen + dxb : 0u;
        // tokens: literals packed up to 3 (one per token in the recorded bits), a match after its
        // pending literals
        const uint32_t litw2 = litw | (val << (8u * nlit));
        const uint32_t nlit2 = nlit + 1u;
        const uint32_t emitL = isLit & ((nlit2 >= 3u) | head);
        const uint32_t emitP = isM & (nlit != 0u);          // a match's pending literals first
        const uint32_t tokL = ((isLit ? nlit : nlit - 1u) << 24) | (isLit ? litw2 : litw);
        const uint32_t tokM = 0x80000000u | ((val - 3u) << 16) | (dist - 1u);
        const uint32_t e1 = dec & (emitL | emitP), e2 = dec & isM;
        *(e1 ? tst + (ntk & (WD_TST - 1u)) : tdum) = tokL;
        *(e2 ? tst + ((ntk + e1) & (WD_TST - 1u)) : tdum) = tokM;
        ntk += e1 + e2;
        const uint32_t keepL = isLit & (emitL ^ 1u);      // literal still pending
        const uint32_t litwN = keepL ? litw2 : (isLit | isM) ? 0u : litw;
        const uint32_t nlitN = keepL ? nlit2 : (isLit | isM) ? 0u : nlit;
        litw = dec ? litwN : litw;
        nlit = dec ? nlitN : nlit;
        // end of block (value 0) or an invalid code (value 1, or a bad distance code)
        const uint32_t sp_ = dec & (isSp | derr);
        const uint32_t eob = isSp & (val == 0u);
        st = sp_ ? (eob ? (uint32_t)WR_EOB : (uint32_t)WR_ERR) : st;
        stop = sp_ ? (eob ? p + len : p) : stop;
        prog |= sp_ << 31;
    };

    for (;;) {
        if (st == WR_RUN) ring_step_wd(H);
        // staged tokens -> the lane's provisional slot, 8 at a time (at most 8 per 4 steps)
        {
            const bool f = ntk - nfl >= 8u;
            if (__ballot(f)) {
                if (f) {
                    const uint32_t* s1 = tst + (nfl & (WD_TST - 1));
                    uint32_t v[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) v[k] = s1[k];
                    GLB uint4* d = (GLB uint4*)(prov + nfl);
                    d[0] = make_uint4(v[0], v[1], v[2], v[3]);
                    d[1] = make_uint4(v[4], v[5], v[6], v[7]);
                    nfl += 8u;
                }
            }
        }
        // a lane may reach a stop in the next 4 steps (28 bits at most per step)?
        const uint32_t pn = Kc - (uint32_t)H.avail + H.bo;
        const bool nearE = st == WR_RUN && (pn + 4u * 48u >= bn || pn + 4u * 48u >= lim || ntk + 12u > tcapl);
        if (__ballot(nearE)) {
            // the successor's progress (stale by up to 4 steps: safe), for lanes past their chunk
            // or reaching it in these steps; "offset 0, running" when not fetched
            uint32_t sp = 0u;
            if (__ballot(st == WR_RUN && !lastl && pn + 4u * 48u >= bn)) sp = __shfl_down(prog, 1);
            const uint32_t spv = sp & 0x7fffffffu;
            const uint32_t sstop = sp >> 31;
#pragma unroll
            for (int rep = 0; rep < 4; ++rep) step(std::true_type{}, spv, sstop);
        } else {
#pragma unroll
            for (int rep = 0; rep < 4; ++rep) step(std::false_type{}, 0u, 0u);
        }
        if (!__ballot(st == WR_RUN)) break;
    }
#ifdef SDZ_TIMING
    const unsigned long long tw1 = dbg ? clock64() : 0;
#endif
    // pending literals, then the rest of the stage
    if (nlit) { push(((nlit - 1u) << 24) | litw); nlit = 0; }
    for (uint32_t q = nfl; q < ntk; ++q) prov[q] = tst[q & (WD_TST - 1)];

    // the successor's start index: its recorded starts before the sync offset
    uint32_t k = 0;
    {
        const bool sy = st == WR_SYNC;
        const uint32_t wmax = sy ? synco >> 5 : 0u;
        for (uint32_t w = 0; __ballot(sy && w <= wmax); ++w) {
            if (sy && w <= wmax) {
                uint32_t x = bmn[w];
                if (w == wmax) x &= (1u << (synco & 31u)) - 1u;
                k += __popc(x);
            }
        }
    }
    const uint32_t s0 = __shfl_up(k, 1);
    const uint32_t s = lane ? s0 : 0u;
    const uint64_t M = __ballot(st == WR_SYNC);
    const uint32_t J = (uint32_t)__builtin_ctzll(~M);     // first lane not chained to its successor
    const bool inc = lane <= J;
    const uint32_t c = inc && ntk >= s ? ntk - s : 0u;
    const uint32_t incl = wd_scan(c);
    const uint32_t total = wd_at(incl, 63);
    const uint32_t excl = incl - c;
    const uint32_t stJ = wd_at(st, J), stopJ = wd_at(stop, J);
#ifdef SDZ_TIMING
    if (dbg) {
        uint32_t ns = nsym;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) ns += __shfl_xor(ns, o);
        const uint64_t nsy = __ballot(st == WR_NOSYNC);
        if (lane == 0) {
            atomicAdd(&dbg[18], tw1 - tw0); atomicAdd(&dbg[20], 1ull); atomicAdd(&dbg[21], stJ == WR_CAP ? 1ull : 0ull);
            atomicAdd(&dbg[22], (unsigned long long)ns); atomicAdd(&dbg[23], (unsigned long long)total);
            atomicAdd(&dbg[24], (unsigned long long)(J + 1)); atomicAdd(&dbg[25], (unsigned long long)n);
            atomicAdd(&dbg[26], stJ == WR_ERR ? 1ull : 0ull); atomicAdd(&dbg[27], nsy ? 1ull : 0ull);
            atomicAdd(&dbg[28], stJ == WR_EOB ? 1ull : 0ull); atomicAdd(&dbg[30], (unsigned long long)C);
            atomicAdd(&dbg[19], clock64() - tw1);
        }
    }
#endif
    // compaction: chunk by chunk, the whole wave copies each chained lane's tokens (from its
    // successor's start index on) into the ring -- coalesced, 4 chunks' loads in flight at a time
    // (the provisional slots are a buffer of their own, so no copy overwrites another's source).
    // Loads and stores past a chunk's count go to the lane's dummy slot: no per-token branch.
    uint32_t bytes = 0;
#ifdef SDZ_TIMING
    const unsigned long long tc0 = dbg ? clock64() : 0;   // dbg[12]: compaction cycles
#endif
    {
        GLB uint32_t* dst0 = (GLB uint32_t*)(tb + ntok0);
        GLB uint32_t* dum = (GLB uint32_t*)(pv + 64u * WD_CAP + lane);
        for (uint32_t j0 = 0; j0 <= J; j0 += 4u) {
            uint32_t v[4][WD_CAP / 64];
            uint32_t cj[4], dj[4];
#pragma unroll
            for (uint32_t jj = 0; jj < 4u; ++jj) {
                const uint32_t j = j0 + jj < 64u ? j0 + jj : 63u;
                cj[jj] = j0 + jj <= J ? wd_at(c, j) : 0u;
                dj[jj] = wd_at(excl, j);
                const GLB uint32_t* src = (const GLB uint32_t*)(pv + j * tcapl + wd_at(s, j));
#pragma unroll
                for (uint32_t k = 0; k < WD_CAP / 64; ++k) {
                    const uint32_t q = lane + 64u * k;
                    v[jj][k] = *(q < cj[jj] ? src + q : (const GLB uint32_t*)dum);
                }
            }
#pragma unroll
            for (uint32_t jj = 0; jj < 4u; ++jj)
#pragma unroll
                for (uint32_t k = 0; k < WD_CAP / 64; ++k) {
                    const uint32_t q = lane + 64u * k;
                    const bool in = q < cj[jj];
                    const uint32_t t = v[jj][k];
                    *(in ? dst0 + dj[jj] + q : dum) = t;
                    bytes += !in ? 0u : (int32_t)t < 0 ? ((t >> 16) & 255u) + 3u : ((t >> 24) & 3u) + 1u;
                }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) bytes += __shfl_xor(bytes, o);
#ifdef SDZ_TIMING
    if (dbg && lane == 0) atomicAdd(&dbg[12], clock64() - tc0);
#endif
    if (stJ == WR_CAP && J == 0 && cmax > WD_CMIN) cmax >>= 1;
    if (pos0 + bytes > cap) return 2;                     // the slow step reports the overflow exactly
    if (lane == 0) {
        S->ntok = ntok0 + total;
        S->pos = pos0 + bytes;
        S->bitpos = B0 + stopJ;
        S->litw = 0;
        S->nlit = 0;
        if (stJ == WR_EOB) S->mode = S->last ? LM_TRAILER : LM_TYPE;
    }
    __threadfence_block();
    return stJ == WR_EOB || stJ == WR_END ? 1 : stJ == WR_ERR ? 2 : 0;
}

// The wave decoder's block-level work -- container header, block headers and trees, stored blocks,
// the trailer, the last input bits, and the exact slow step for blocks the wave declined (an
// invalid code, the output room, tables past the LDS budget) -- runs in k_inflate_wcold, one LANE
// per stream as in k_inflate_decode (cold_run), so that 64 streams' serial header work shares a
// wave.  k_inflate_wdec (one WAVE per stream) then decodes the block's symbols; the host
// alternates the two until no stream needs block-level work in this round.
// first: the round's first launch (round 0: starts the streams; later rounds: resumes the streams
// whose token ring filled).  A.flags: 2 = not live this round (finished earlier), else 0 until
// k_inflate_wdec records the round's end.  lane: after kWdLaneAfter alternations (a stream of many
// small blocks costs one launch pair per block) the lane decoder's whole loop (cold_run and
// hot_epoch, as in k_inflate_decode) finishes the stream's round here.
__global__ __launch_bounds__(IL_THREADS, 1) void k_inflate_wcold(InflateArgs A, uint32_t round, uint32_t first,
                                                                  uint32_t lane) {
#ifdef IL_PROF                                           // development: phase clocks of stream 0, printf
    uint64_t tq[8] = {};
#define WC_T(k) do { if (gid == 0) tq[k] = wall_clock64(); } while (0)
#else
#define WC_T(k) do { } while (0)
#endif
    uint8_t* region = lane_region();
    uint32_t* ts = lane_stage();
    const uint32_t gid = blockIdx.x * IL_STREAMS + lane_slot();
    WC_T(0);
    // the counters k_inflate_wdec fills next (no memset launch between the pair; this kernel
    // does not read them)
    if (blockIdx.x == 0 && threadIdx.x == 0) { A.active[0] = 0; A.active[1] = 0; }
    if (gid >= A.n || (threadIdx.x & 63u) >= IL_WAVE_LANES) return;
    const uint32_t sid = gid;
    DSave* S = (DSave*)A.dsave + sid;
    uint32_t* tb = A.tokens + (uint64_t)sid * A.round_tokens;
    const uint32_t tcap = A.round_tokens;
    uint8_t* lens = A.scratch + (uint64_t)sid * kInflateScratchPerStream;
    const uint8_t* inp = A.in + A.in_off[sid];
    const uint64_t ilen = A.in_len[sid];
    const uint64_t cap = A.out_cap[sid];
    const int32_t did = dict_id_of(A.dict_adler, A.dict_adler_dev);
    const SegStop G = { 0, nullptr, 0 };
    uint32_t init = 0;
    int force_slow = 0;
    if (first) {
        if (round == 0 && (A.out_off[sid] & 7)) {
            S->mode = LM_DONE; S->status = SDZ_BAD_RECORD; S->zmsg = 0; S->bitpos = 0; S->pos = 0;
            S->container = SDZ_CONTAINER_RAW; S->stored_ck = 0; S->stored_size = 0; S->mtime = 0;
            S->name_off = 0; S->name_len = 0; S->dict_used = 0; S->ntok = 0; S->litw = 0;
            S->nlit = 0; S->full = 0; S->stall = 0;
            A.ntok[sid] = 0; A.flags[sid] = 2;
            return;
        }
        if (round > 0 && S->mode == LM_DONE) { A.ntok[sid] = 0; A.flags[sid] = 2; return; }
        A.flags[sid] = 0;
        if (round == 0) init = 1;
        else { S->ntok = 0; S->full = 0; }               // a new round: the token ring from 0
    } else {
        if (A.flags[sid] == 2 || S->mode == LM_DONE || S->full) return;
        force_slow = S->mode == LM_CODES ? 1 : 0;        // the wave declined the rest of this block
    }
    WC_T(1);
    if (!init) {
        copy_dw((uint32_t*)region, (const uint32_t*)S->region, IL_REGION / 4);
        const uint32_t nt = S->ntok, b = nt & ~(IL_TSTAGE - 1u);   // the open 32-token line
        copy_dw(ts, tb + b, nt - b);
    }
    WC_T(2);
    if (lane && !init) epochs<0>(A, S, inp, ilen, cap, tb, tcap, lens, true, G);
    else cold_run<0>(S, inp, ilen, cap, tb, tcap, lens, A.format, A.dict != nullptr, did, init, G, force_slow);
    WC_T(3);
    Core H;                                              // flush the token stage
    H.tb = tb; H.ts = ts; H.ntok = S->ntok; H.litw = S->litw; H.nlit = S->nlit; H.tcap = tcap;
#ifdef IL_HOT_CHECK
    H.chk_lo = H.chk_hi = nullptr; H.chk_id = sid;
#endif
    tok_finish(H);
    S->ntok = H.ntok; S->litw = 0; S->nlit = 0;
    if (S->mode == LM_CODES)
        copy_dw((uint32_t*)S->region, (const uint32_t*)region, IL_REGION / 4);
    WC_T(4);
#ifdef IL_PROF
    if (gid == 0)
        printf("WC_PROF round %u first %u init %u mode %d | entry %lu region+stage %lu cold %lu flush+save %lu [x10ns]\n",
               round, first, init, (int)S->mode, tq[1] - tq[0], tq[2] - tq[1], tq[3] - tq[2], tq[4] - tq[3]);
#endif
}

// One WAVE per stream: the current block's symbols by speculative iterations, until the block
// ends, the input's last bits, or anything the wave declines (k_inflate_wcold takes those).
// Records the stream's round state for k_inflate_resolve; counts the streams that need block-level
// work (A.active[1]) and those whose token ring filled (A.active[0], another round).
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WD_WPE, WD_WPE))) void k_inflate_wdec(InflateArgs A, uint32_t round) {
    const uint32_t sid = blockIdx.x, lane = threadIdx.x;
    if (sid >= A.n) return;
    if (wd_uni(lane == 0 ? A.flags[sid] : 0u) == 2u) return;   // not live this round
    DSave* S = (DSave*)A.dsave + sid;
    uint32_t* tb = A.tokens + (uint64_t)sid * A.round_tokens;
    const uint32_t tcap = A.round_tokens;
    const uint8_t* inp = A.in + A.in_off[sid];
    const uint64_t ilen = A.in_len[sid];
    const uint64_t cap = A.out_cap[sid];
    const uint64_t tbits = ilen * 8;
#ifdef SDZ_TIMING
    // development: the first 64 streams' waves (dbg[14] total cycles, [15] launches, [17] table
    // builds' cycles, [29] iteration cycles, [31] table builds)
    unsigned long long* wdbg = A.dbg && sid < 64 ? A.dbg : nullptr;
    const unsigned long long tk0 = wdbg ? clock64() : 0;
#else
    unsigned long long* wdbg = nullptr;
#endif
    const uint32_t mode0 = wd_uni(lane == 0 ? (uint32_t)S->mode : 0u);
    const uint32_t full0 = wd_uni(lane == 0 ? (uint32_t)S->full : 0u);
    if (mode0 == LM_CODES && !full0) {
        for (uint32_t k = lane; k < IL_REGION / 4; k += 64) ((uint32_t*)wd_region)[k] = ((const uint32_t*)S->region)[k];
        if (lane == 0) { wd_LL = S->LL; wd_DD = S->DD; }
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        bool built = false;
        uint32_t cmax = WD_CMAX;
        for (;;) {
            // the stream's state as lane 0 left it (lane 0 reads its own stores; broadcast)
            if (wd_uni(lane == 0 ? (uint32_t)S->mode : 0u) != LM_CODES) break;   // the block ended
            const uint64_t bp = lane == 0 ? S->bitpos : 0;
            const uint64_t B0 = ((uint64_t)wd_uni((uint32_t)(bp >> 32)) << 32) | wd_uni((uint32_t)bp);
            const uint32_t ntok = wd_uni(lane == 0 ? S->ntok : 0u);
            const uint64_t ps = lane == 0 ? S->pos : 0;
            const uint64_t pos = ((uint64_t)wd_uni((uint32_t)(ps >> 32)) << 32) | wd_uni((uint32_t)ps);
            if (tbits < B0 + 64 + WD_MINSPEC || tcap < ntok + 80u) break;   // the slow step's
            if (!built) {
#ifdef SDZ_TIMING
                const unsigned long long tb0 = wdbg ? clock64() : 0;
#endif
                const bool okb = wd_build();
#ifdef SDZ_TIMING
                if (wdbg && lane == 0) { atomicAdd(&wdbg[17], clock64() - tb0); atomicAdd(&wdbg[31], 1ull); }
#endif
                if (!okb) break;
                built = true;
            }
#ifdef SDZ_TIMING
            const unsigned long long tb0 = wdbg ? clock64() : 0;
#endif
            const int r = wd_iteration(S, inp, ilen, cap, tb, tcap, A.wdprov + (uint64_t)sid * kWdProvTokens, B0, ntok,
                                       pos, cmax, wdbg);
#ifdef SDZ_TIMING
            if (wdbg && lane == 0) atomicAdd(&wdbg[29], clock64() - tb0);
#endif
            if (r >= 2) break;                           // the slow step takes the block from here
        }
    }
#ifdef SDZ_TIMING
    if (wdbg && lane == 0) { atomicAdd(&wdbg[14], clock64() - tk0); atomicAdd(&wdbg[15], 1ull); }
#endif
    if (lane == 0) {
        const uint32_t m = (uint32_t)S->mode, f = (uint32_t)S->full;
        A.ntok[sid] = S->ntok;
        A.flags[sid] = m == LM_DONE ? 1u : 0u;
        if (m != LM_DONE && !f) atomicAdd(A.active + 1, 1u);   // block-level work next
        if (m != LM_DONE && f) atomicAdd(A.active, 1u);        // another round
    }
}

void launch_seg_decode(const InflateArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_inflate_decode, dim3((a.n + IL_STREAMS - 1) / IL_STREAMS), dim3(IL_THREADS), 0, s, a, 0u);
}

void launch_inflate_resolve(const InflateArgs& a, uint32_t round, dim3 grid, hipStream_t s);
uint32_t resolve_block_threads();
uint32_t resolve_streams_per_block();
void launch_inflate_finalize(const InflateArgs& a, hipStream_t s);

// the state arrays are indexed as DSave* / RSave* arrays: the strides are the struct sizes
uint64_t inflate_dsave_bytes() { return sizeof(DSave); }
int inflate_wdec_mode() {
    const char* e = getenv("SDZ_WDEC");
    return e && *e ? (atoi(e) != 0 ? 1 : 0) : -1;
}
bool inflate_wave_policy(uint32_t n, const uint64_t* host_len, const uint64_t* dev_len, void* stream) {
    const int m = inflate_wdec_mode();
    if (m >= 0) return m == 1;
    if (n == 0 || n > kWdAutoStreams) return false;
    std::vector<uint64_t> len;
    if (!host_len) {
        len.resize(n);
        if (hipMemcpyAsync(len.data(), dev_len, n * sizeof(uint64_t), hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
            hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
            return false;
        host_len = len.data();
    }
    uint64_t mx = 0, tot = 0;
    for (uint32_t i = 0; i < n; ++i) { mx = host_len[i] > mx ? host_len[i] : mx; tot += host_len[i]; }
    return mx >= kWdAutoMinBytes && mx <= kWdAutoBytes && tot <= kWdAutoRatio * mx;
}
uint64_t inflate_rsave_bytes() { return sizeof(RSave); }

// SDZ_DEBUG_SYNC=1 (development): wait after every launch of the round driver and report the first
// kernel whose run ends in an error, by name (a fault is otherwise seen at the next API call)
static bool dbg_sync_on() {
    static const bool on = getenv("SDZ_DEBUG_SYNC") != nullptr;
    return on;
}
static int dbg_sync(hipStream_t s, const char* what, uint32_t round, uint32_t it) {
    if (!dbg_sync_on()) return 0;
    const hipError_t e = hipStreamSynchronize(s);
    if (e == hipSuccess) return 0;
    fprintf(stderr, "sdz debug sync: %s (round %u, step %u): %s\n", what, round, it, hipGetErrorString(e));
    return -1;
}
#define DBG_SYNC(s, what, round, it) do { if (dbg_sync((s), (what), (round), (it))) { rc = -1; break; } } while (0)

// host driver: rounds of (decode, resolve) until no stream needs another round.
// kernel_ms (optional, 3 entries) accumulates decode / resolve / finalize times.
#ifndef WD_PAIRS
#define WD_PAIRS 2                        // wave decoder: launch pairs queued per count read-back
#endif
int run_inflate_rounds(const InflateArgs& a, hipStream_t s, uint32_t* host_active, float* kernel_ms,
                       int (*hook)(void*), void* hook_ctx) {
    if (a.n == 0) return 0;
    uint32_t spb = resolve_streams_per_block();
    dim3 g1((a.n + IL_STREAMS - 1) / IL_STREAMS), g2((a.n + spb - 1) / spb);
    hipEvent_t ev[4] = { nullptr, nullptr, nullptr, nullptr };
    if (kernel_ms) {
        for (auto& e : ev) (void)hipEventCreate(&e);
        kernel_ms[0] = kernel_ms[1] = kernel_ms[2] = 0.f;
    }
    int rc = 0;
    // the wave decoder (k_inflate_wdec) for one-shot batches; the lane decoder keeps the
    // incremental mode (and the block-parallel split of long streams, off with the wave decoder)
    const bool use_wd = a.wave && a.wdprov && !a.streaming && !a.segmode && !a.split_plan;
    uint32_t lane_after = kWdLaneAfter;                  // SDZ_WD_LANE_AFTER: development / tests
    if (const char* e = getenv("SDZ_WD_LANE_AFTER")) lane_after = (uint32_t)strtoul(e, nullptr, 10);
    // one round and no wave decoder: nothing reads the active counter (a launch less per call)
    const bool count_active = !(a.one_round && !a.split_plan && !use_wd);
    for (uint32_t round = 0;; ++round) {
        if (count_active && hipMemsetAsync(a.active, 0, sizeof(uint32_t), s) != hipSuccess) { rc = -1; break; }
        if (kernel_ms) (void)hipEventRecord(ev[0], s);
        if (use_wd) {
            // block-level work (a lane per stream) and the blocks' symbols (a wave per stream),
            // alternately, until no stream of this round needs block-level work
            // pairs are queued WD_PAIRS at a time between read-backs of the count (a pair past
            // the end finds nothing to do: ~10 us, against a ~25 us host round trip per read)
            for (uint32_t it = 0;;) {
                for (uint32_t b = 0; b < WD_PAIRS; ++b, ++it) {
                    // (round 0 starts over on the lane decoder after lane_after pairs: no pair of that
                    // round runs with the lane flag, whose work the restart would throw away)
                    if (round == 0 && it >= lane_after) break;
                    hipLaunchKernelGGL(k_inflate_wcold, g1, dim3(IL_THREADS), 0, s, a, round, it == 0 ? 1u : 0u,
                                       it >= lane_after ? 1u : 0u);
                    DBG_SYNC(s, "k_inflate_wcold", round, it);
                    hipLaunchKernelGGL(k_inflate_wdec, dim3(a.n), dim3(64), 0, s, a, round);
                    DBG_SYNC(s, "k_inflate_wdec", round, it);
                }
                if (hipMemcpyAsync(host_active, a.active + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
                    hipStreamSynchronize(s) != hipSuccess) { rc = -1; break; }
                if (*host_active == 0) break;
                // a stream of many small blocks costs a launch pair per block here: the first
                // round starts over on the lane decoder with the block-parallel split (nothing
                // is resolved yet); later rounds hand the rest to the lane decoder in
                // k_inflate_wcold
                if (round == 0 && it >= lane_after) { rc = kWdRestart; break; }
            }
            if (rc) break;
        } else {
            hipLaunchKernelGGL(k_inflate_decode, g1, dim3(IL_THREADS), 0, s, a, round);
            DBG_SYNC(s, "k_inflate_decode", round, 0);
        }
        if (round == 0 && hook) {
            if (int hr = hook(hook_ctx)) { rc = hr; break; }
        }
        if (a.split_plan) {                              // the split streams (k_split.hip)
            if (round == 0) {
                // segments decoded on the side stream meanwhile: chain them, decode the
                // streams whose chain broke, serially from their start
                const SplitPlan& P = *a.split_plan;
                if (hipStreamWaitEvent(s, (hipEvent_t)P.ready, 0) != hipSuccess) { rc = -1; break; }
                if (dbg_sync_on()) {                              // the side stream's finder and segments
                    const hipError_t e = hipEventSynchronize((hipEvent_t)P.ready);
                    if (e != hipSuccess) {
                        fprintf(stderr, "sdz debug sync: side stream (split finder, segment decode): %s\n",
                                hipGetErrorString(e));
                        rc = -1;
                        break;
                    }
                }
                launch_seg_chain(a, P.sp, P.nsplit, P.seg, P.cand, P.segD, P.chain, P.chain_tok, a.split_state, s);
                DBG_SYNC(s, "k_seg_chain", round, 0);
                InflateArgs f = a;
                f.fallback_pass = 1;
                hipLaunchKernelGGL(k_inflate_decode, g1, dim3(IL_THREADS), 0, s, f, 0u);
                DBG_SYNC(s, "k_inflate_decode (fallback pass)", round, 0);
            }
            launch_seg_feed(a, round, s);
            DBG_SYNC(s, "k_seg_feed", round, 0);
        }
        if (kernel_ms) (void)hipEventRecord(ev[1], s);
        launch_inflate_resolve(a, round, g2, s);
        DBG_SYNC(s, "k_inflate_resolve", round, 0);
        if (kernel_ms) (void)hipEventRecord(ev[2], s);
        if (a.one_round && !a.split_plan) break;         // (times read after finalize)
        if (hipMemcpyAsync(host_active, a.active, sizeof(uint32_t), hipMemcpyDeviceToHost, s) != hipSuccess) { rc = -1; break; }
        if (hipStreamSynchronize(s) != hipSuccess) { rc = -1; break; }
        if (kernel_ms) {
            float t0 = 0.f, t1 = 0.f;
            (void)hipEventElapsedTime(&t0, ev[0], ev[1]);
            (void)hipEventElapsedTime(&t1, ev[1], ev[2]);
            kernel_ms[0] += t0;
            kernel_ms[1] += t1;
        }
        if (*host_active == 0) break;
    }
    if (rc == 0) {
        if (kernel_ms) (void)hipEventRecord(ev[2], s);
        if (!a.no_gzip) launch_inflate_finalize(a, s);   // (only gzip streams need it)
        if (kernel_ms) {
            (void)hipEventRecord(ev[3], s);
            (void)hipEventSynchronize(ev[3]);
            if (a.one_round && !a.split_plan) {
                float t0 = 0.f, t1 = 0.f;
                (void)hipEventElapsedTime(&t0, ev[0], ev[1]);
                (void)hipEventElapsedTime(&t1, ev[1], ev[2]);
                kernel_ms[0] = t0;
                kernel_ms[1] = t1;
            }
            float t2 = 0.f;
            (void)hipEventElapsedTime(&t2, ev[2], ev[3]);
            kernel_ms[2] = t2;
        }
        if (hipGetLastError() != hipSuccess) rc = -1;
    } else if (rc == kWdRestart && kernel_ms) {
        // the wave attempt's time (the call starts over on the lane decoder) counts as decode
        float t0 = 0.f;
        (void)hipEventRecord(ev[1], s);
        (void)hipEventSynchronize(ev[1]);
        (void)hipEventElapsedTime(&t0, ev[0], ev[1]);
        kernel_ms[0] = t0;
    }
    if (kernel_ms) for (auto& e : ev) (void)hipEventDestroy(e);
    return rc;
}

}  // namespace sdz
