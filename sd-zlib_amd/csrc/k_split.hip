// k_split.hip -- block-parallel decode of long streams.
//
// One lane decodes one stream, so a batch of mixed sizes (BASELINE C4: 4 KiB - 16 MiB) waits
// for its longest stream: a 12 MB stream decodes serially for seconds.  A DEFLATE block is
// Huffman-decodable on its own once its start bit is known (its tables are in its header;
// only the LZ77 window spans blocks, and that is resolved later, in stream order).  So:
//
//  1. k_split_find: every bit position of a long stream is tested for a dynamic-block header
//     (BTYPE 2, HLIT/HDIST <= 29, a complete code-length code, code lengths that decode
//     without overrun into a complete literal/length code with an end-of-block code and a
//     complete distance code).  Positions that pass are CANDIDATE block starts.
//  2. k_split_sort: each stream's candidates in bit order.
//  3. k_inflate_decode in segment mode (k_inflate.hip): one lane per SEGMENT -- the stream's
//     start, and each candidate -- decodes blocks until it reaches a block boundary that is a
//     candidate, or the end of the last block.
//  4. k_seg_chain: from the stream's start, each segment hands over to the segment that
//     starts where it ended.  The start is a true block start, and a segment from a true
//     start decodes exactly what the serial decoder would, up to a true block boundary: by
//     induction the chain is the serial decode.  Candidates that are not block starts are
//     never reached.  A chain that breaks (an error, a full token buffer, a trailer that
//     needs more input) sends the stream to the serial path, which reports it exactly.
//  5. k_seg_feed, each round: the stream's tokens, in chain order, go to the resolve phase
//     (k_resolve.hip) like the serial decoder's would.
#include "inflate_state.h"
#include "split.h"

namespace sdz {

__constant__ uint8_t c_split_border[19] = { 16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15 };

// little-endian u32 at byte q of an input of `len` bytes (q may be unaligned; bytes past the
// end read as 0, so no lane reads past its stream's last byte)
__device__ __forceinline__ uint32_t sp_u32(const uint8_t* p, uint64_t q, uint64_t len) {
    if (q + 4 <= len) {
        const uint8_t* r = p + q;
        return (uint32_t)r[0] | ((uint32_t)r[1] << 8) | ((uint32_t)r[2] << 16) | ((uint32_t)r[3] << 24);
    }
    uint32_t v = 0;
    for (uint32_t j = 0; j < 4; ++j) if (q + j < len) v |= (uint32_t)p[q + j] << (8 * j);
    return v;
}
__device__ __forceinline__ uint32_t sp_u32a(const uint8_t* p, uint64_t q, uint64_t len) {   // q % 4 == 0
    if (q + 4 <= len && (((uintptr_t)(p + q)) & 3) == 0) return *(const uint32_t*)(p + q);
    return sp_u32(p, q, len);
}

// Pass 1 (k_split_filter): one lane tests 32 consecutive bit positions.  Bit-sliced over the
// 32 positions (one mask bit each): BTYPE = 2, HLIT <= 29, HDIST <= 29 and room for a header
// (about 22 % pass); then, per remaining position, the Kraft sum of the code-length code's
// first HCLEN + 4 lengths (their order does not matter for the sum) from a 4096-entry LDS
// table of 4-length partial sums, 5 lookups.  (Bit-sliced Kraft tests mod 4 ahead of it, the
// sums from 32-bit words with 6 lookups, and a table-free v_perm/v_sad sum were all slower:
// the loop is VALU-bound, 9.0 ms on C4 at 1/8.)  About 0.1 % of positions pass (measured on zlib
// output); they go, (position << 20 | split index), to the block's own survivor region.
// Each block walks a contiguous range of lanes, so the split stream of a lane is found by
// stepping forward, not by a search per lane.
__global__ __launch_bounds__(256) void k_split_filter(const uint8_t* in, const uint64_t* in_off, const SplitInfo* sp,
                                                      uint32_t nsplit, uint64_t total_lanes, uint64_t lanes_per_block,
                                                      uint64_t* surv, uint32_t* nsurv, uint32_t bcap) {
    __shared__ uint32_t cnt;
    __shared__ uint8_t klut[4096];                        // 4 lengths (3 bits each) -> sum of 128 >> len (len > 0)
    const uint64_t L0 = (uint64_t)blockIdx.x * lanes_per_block;
    if (L0 >= total_lanes) return;
    for (uint32_t x = threadIdx.x; x < 4096; x += 256) {
        uint32_t k = 0;
        for (int j = 0; j < 4; ++j) k += (128u >> ((x >> (3 * j)) & 7u)) & 127u;
        klut[x] = (uint8_t)(k < 255 ? k : 255);
    }
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    surv += (uint64_t)blockIdx.x * bcap;                  // this block's own region: no global atomics
    const uint64_t L1 = L0 + lanes_per_block < total_lanes ? L0 + lanes_per_block : total_lanes;
    uint32_t lo = 0, hi = nsplit;                         // the split stream holding lane L0
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sp[mid].lane0 <= L0) lo = mid; else hi = mid;
    }
    // the lane's split stream, cached: a lane steps to the next stream only at its boundary,
    // and the next lane group's 16 bytes are loaded while this one is tested
    uint32_t sk = lo;
    uint64_t slane0 = sp[sk].lane0, snbits = sp[sk].nbits;
    uint64_t snxt = sk + 1 < nsplit ? sp[sk + 1].lane0 : ~0ull;
    const uint8_t* sbase = in + in_off[sp[sk].sid];
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;             // the words of the next lane group
    uint64_t cp0 = 0, cnb = 0;
    uint32_t ck = 0;
    auto fetch = [&](uint64_t g) {
        while (g >= snxt) {
            ++sk;
            slane0 = snxt;
            snbits = sp[sk].nbits;
            sbase = in + in_off[sp[sk].sid];
            snxt = sk + 1 < nsplit ? sp[sk + 1].lane0 : ~0ull;
        }
        cp0 = 32 * (g - slane0); cnb = snbits; ck = sk;
        const uint64_t q = cp0 >> 3, nbytes = snbits >> 3;
        c0 = sp_u32a(sbase, q, nbytes); c1 = sp_u32a(sbase, q + 4, nbytes);
        c2 = sp_u32a(sbase, q + 8, nbytes); c3 = sp_u32a(sbase, q + 12, nbytes);
    };
    if (L0 + threadIdx.x < L1) fetch(L0 + threadIdx.x);
    for (uint64_t g = L0 + threadIdx.x; g < L1; g += 256) {
        const uint32_t w0 = c0, w1 = c1, w2 = c2, w3 = c3;
        const uint64_t p0 = cp0, nbits = cnb;
        const uint32_t k = ck;
        if (g + 256 < L1) fetch(g + 256);                 // (issued before this group's tests)
        const uint64_t W = (uint64_t)w0 | ((uint64_t)w1 << 32);
#define SPB(d) ((uint32_t)(W >> (d)))
        uint32_t M = ~SPB(1) & SPB(2)                                   // BTYPE = 2 (bits 1, 2 = 0, 1)
                   & ~(SPB(4) & SPB(5) & SPB(6) & SPB(7))               // HLIT (bits 3-7) < 30
                   & ~(SPB(9) & SPB(10) & SPB(11) & SPB(12));           // HDIST (bits 8-12) < 30
#undef SPB
        const uint64_t room = nbits >= p0 + 74 ? nbits - p0 - 74 + 1 : 0;   // header of 17 + 57 bits fits
        M &= room >= 32 ? 0xffffffffu : (uint32_t)((1ull << room) - 1);
        uint64_t out[4];
        uint32_t no = 0;
        while (M) {
            const uint32_t i = (uint32_t)__builtin_ctz(M);
            M &= M - 1;
            const uint32_t a = __builtin_amdgcn_alignbit(w1, w0, i);    // bits i .. i+31
            const uint32_t b = __builtin_amdgcn_alignbit(w2, w1, i);    // bits i+32 .. i+63
            const uint32_t c = __builtin_amdgcn_alignbit(w3, w2, i);    // bits i+64 .. i+95
            const uint32_t hclen = (a >> 13) & 15u;
            uint64_t X = ((((uint64_t)b << 32) | a) >> 17) | ((uint64_t)c << 47);   // the 19 lengths' bits
            X &= (1ull << (3 * hclen + 12)) - 1;                          // the HCLEN + 4 sent
            const uint32_t kraft = (uint32_t)klut[X & 4095u] + klut[(X >> 12) & 4095u] + klut[(X >> 24) & 4095u] +
                                   klut[(X >> 36) & 4095u] + klut[(X >> 48) & 4095u];
            if (kraft == 128u && no < 4) out[no++] = ((p0 + i) << 20) | k;
        }
        // append this lane's survivors (at most 4 of 32 positions: more is not a real stream)
        const uint64_t bm = __ballot(no != 0);
        if (bm) {
            uint32_t tot = no;                             // wave prefix of the counts
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = __shfl_up(tot, o);
                if ((threadIdx.x & 63u) >= (uint32_t)o) tot += v;
            }
            const uint32_t pre = tot - no;
            const uint32_t wsum = __shfl(tot, 63);
            uint32_t base = 0;
            if ((threadIdx.x & 63u) == 63u) base = atomicAdd(&cnt, wsum);
            base = __shfl(base, 63);
            for (uint32_t j = 0; j < no; ++j)
                if (base + pre + j < bcap) surv[base + pre + j] = out[j];
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) nsurv[blockIdx.x] = cnt < bcap ? cnt : bcap;
}

// bit reader over one input for k_split_deep: 64-bit buffer, refilled a word at a time
struct SpBits {
    const uint8_t* p;
    uint64_t len, next;                                   // next byte to load
    uint64_t buf;
    uint32_t nb;                                          // valid bits in buf
    __device__ __forceinline__ void init(const uint8_t* p_, uint64_t len_, uint64_t pos) {
        p = p_; len = len_;
        const uint64_t q = pos >> 3;
        buf = ((uint64_t)sp_u32(p, q, len) | ((uint64_t)sp_u32(p, q + 4, len) << 32)) >> (pos & 7);
        nb = 64 - (uint32_t)(pos & 7);
        next = q + 8;
    }
    __device__ __forceinline__ void fill() {              // nb >= 32 after
        if (nb < 32) { buf |= (uint64_t)sp_u32(p, next, len) << nb; next += 4; nb += 32; }
    }
    __device__ __forceinline__ uint32_t peek(uint32_t n) const { return (uint32_t)buf & ((1u << n) - 1u); }
    __device__ __forceinline__ void drop(uint32_t n) { buf >>= n; nb -= n; }
};

// Pass 2 (k_split_deep): survivors' code lengths decoded (infblocks.ts:354-551 /
// inftree.ts:313-379 on a strict reading: every code complete) with the code-length code in a
// 128-entry LDS table per lane, and running Kraft sums of the literal/length and distance
// lengths, so a random bit string is rejected as soon as one is over-subscribed.  Survivors
// that pass are candidates.  A survivor takes 45 code-length symbols on average but up to
// ~300 (zlib output), so lanes are persistent: one wave works through one filter block's
// survivor region, and whenever 16 of its lanes are idle they take the next 16 survivors
// together -- the wave's steps stay busy instead of waiting for its slowest survivor.
// k_split_deep's bit reader: the survivor's first 64 bytes are staged in the lane's LDS slot
// when it starts (one batch of loads for the lanes starting together), so a refill is an LDS
// read; only a survivor that runs past them (~10 %) reads global memory again.
struct SpBitsL {
    const uint8_t* p;
    uint32_t* W;                                          // the lane's 16 staged dwords
    uint64_t len, q0;                                     // stream bytes; first staged byte
    uint64_t buf;
    uint32_t nb, next;                                    // valid bits in buf; next dword to load
    __device__ __forceinline__ void init(const uint8_t* p_, uint32_t* W_, uint64_t len_, uint64_t pos) {
        p = p_; W = W_; len = len_;
        q0 = (pos >> 3) & ~3ull;
        const uint8_t* r = p + q0;
        if (q0 + 64 <= len && (((uintptr_t)r) & 15) == 0) {
            const uint4* r4 = (const uint4*)r;
            const uint4 a = r4[0], b = r4[1], c = r4[2], d = r4[3];
            W[0] = a.x; W[1] = a.y; W[2] = a.z; W[3] = a.w; W[4] = b.x; W[5] = b.y; W[6] = b.z; W[7] = b.w;
            W[8] = c.x; W[9] = c.y; W[10] = c.z; W[11] = c.w; W[12] = d.x; W[13] = d.y; W[14] = d.z; W[15] = d.w;
        } else {
            for (uint32_t j = 0; j < 16; ++j) W[j] = sp_u32(p, q0 + 4 * j, len);
        }
        const uint32_t sh = (uint32_t)(pos - 8 * q0);     // 0 .. 31
        buf = ((uint64_t)W[0] | ((uint64_t)W[1] << 32)) >> sh;
        nb = 64 - sh;
        next = 2;
    }
    __device__ __forceinline__ void fill() {              // nb >= 32 after
        if (nb < 32) {
            const uint32_t d = next < 16 ? W[next] : sp_u32(p, q0 + 4 * (uint64_t)next, len);
            buf |= (uint64_t)d << nb;
            ++next;
            nb += 32;
        }
    }
    __device__ __forceinline__ uint32_t peek(uint32_t n) const { return (uint32_t)buf & ((1u << n) - 1u); }
    __device__ __forceinline__ void drop(uint32_t n) { buf >>= n; nb -= n; }
};

// The code-length code is decoded table-free (a LUT per lane cost more to fill than the
// ~45 symbols it serves: a fill loop's trip count differs per lane): 6 left-justified limits
// give the code length of the next 7 bits read MSB-first, then rank = base[len] + code, and
// the rank's symbol comes from the lane's 19 sorted symbols in LDS.
struct DeepLane {
    SpBitsL R;
    uint64_t pos, nbits;
    uint64_t base;                                        // per length 1..7: rank - code + 128, 8 bits each
    uint32_t lim1, lim2, lim3, lim4, lim5, lim6;          // (first code + count) << (7 - len)
    uint32_t k;                                           // split index
    int n, prev, hlit, total;
    uint32_t kl, kd;                                      // Kraft sums in units of 2^-15
    bool eob;
};

__device__ __forceinline__ void deep_start(DeepLane& L, uint8_t* T, uint32_t* W, const uint8_t* in,
                                           const uint64_t* in_off, const SplitInfo* sp, uint64_t e) {
    L.k = (uint32_t)(e & 0xfffffu);
    L.pos = e >> 20;
    const SplitInfo& S = sp[L.k];
    L.nbits = S.nbits;
    L.R.init(in + in_off[S.sid], W, L.nbits >> 3, L.pos);
    const uint32_t h = L.R.peek(17);
    L.R.drop(17);
    L.R.fill();
    const int hclen = (int)(h >> 13) + 4;
    L.hlit = (int)((h >> 3) & 31u) + 257;
    L.total = L.hlit + (int)((h >> 8) & 31u) + 1;
    L.pos += 17 + 3 * (uint64_t)hclen;
    uint64_t cl = 0;                                      // the 19 lengths, 3 bits each, symbol order
    uint64_t bl = 0;                                      // lengths 1..7: their counts, 8 bits each
    for (int i = 0; i < 19; ++i) {                        // (uniform trip count; fields past HCLEN + 4 are 0)
        const uint32_t l = i < hclen ? L.R.peek(3) : 0u;
        if (i < hclen) L.R.drop(3);
        if (i == 9) L.R.fill();
        cl |= (uint64_t)l << (3 * c_split_border[i]);
        bl += l ? 1ull << (8 * l) : 0ull;
    }
    // canonical codes (inftree.ts: shorter first, then symbol order)
    uint64_t nx = 0;                                      // next rank of each length, 8 bits each
    uint32_t code = 0, off = 0, lim[7];
    L.base = 0;
#pragma unroll
    for (int l = 1; l < 8; ++l) {
        const uint32_t c = (uint32_t)(bl >> (8 * l)) & 255u;
        code = (code + ((uint32_t)(bl >> (8 * (l - 1))) & 255u)) << 1;   // first code of length l
        lim[l - 1] = (code + c) << (7 - l);
        L.base |= (uint64_t)((off - code + 128u) & 255u) << (8 * l);
        nx |= (uint64_t)off << (8 * l);
        off += c;
    }
    L.lim1 = lim[0]; L.lim2 = lim[1]; L.lim3 = lim[2]; L.lim4 = lim[3]; L.lim5 = lim[4]; L.lim6 = lim[5];
    for (int sym = 0; sym < 19; ++sym) {                  // the symbols in rank order
        const uint32_t l = (uint32_t)(cl >> (3 * sym)) & 7u;
        const uint32_t r = (uint32_t)(nx >> (8 * l)) & 255u;
        if (l) T[r] = (uint8_t)sym;
        nx += l ? 1ull << (8 * l) : 0ull;
    }
    L.n = 0; L.prev = 0; L.kl = 0; L.kd = 0; L.eob = false;
}

// one code-length symbol; 0: go on, 1: rejected, 2: complete and valid (a candidate)
__device__ __forceinline__ int deep_step(DeepLane& L, const uint8_t* T) {
    if (L.pos + 14 > L.nbits) return 1;
    L.R.fill();
    const uint32_t w = L.R.peek(14);
    const uint32_t v = __builtin_bitreverse32(w) >> 25;  // the next 7 bits, first one most significant
    const uint32_t l = 1u + (v >= L.lim1) + (v >= L.lim2) + (v >= L.lim3) + (v >= L.lim4) + (v >= L.lim5) +
                       (v >= L.lim6);
    const uint32_t rank = (uint32_t)((L.base >> (8 * l)) & 255u) - 128u + (v >> (7 - l));
    const int sym = (int)T[rank];
    int rep = 1, val = sym, used = (int)l;
    if (sym >= 16) {
        const int eb = sym == 16 ? 2 : sym == 17 ? 3 : 7;
        rep = (sym == 18 ? 11 : 3) + (int)((w >> l) & ((1u << eb) - 1u));
        used += eb;
        if (sym == 16 && L.n == 0) return 1;
        val = sym == 16 ? L.prev : 0;
        if (L.n + rep > L.total) return 1;
    }
    L.R.drop((uint32_t)used);
    L.pos += (uint64_t)used;
    if (val) {
        const uint32_t u = 32768u >> val;
        const int nl = L.n < L.hlit ? (L.hlit - L.n < rep ? L.hlit - L.n : rep) : 0;   // of them literal/length
        L.kl += (uint32_t)nl * u;
        L.kd += (uint32_t)(rep - nl) * u;
        L.eob = L.eob || (L.n <= 256 && 256 < L.n + nl);
        if (L.kl > 32768u || L.kd > 32768u) return 1;
    }
    L.n += rep;
    L.prev = val;
    if (L.n < L.total) return 0;
    return L.eob && L.kl == 32768u && L.kd == 32768u ? 2 : 1;
}

__global__ __launch_bounds__(256) void k_split_deep(const uint8_t* in, const uint64_t* in_off, SplitInfo* sp,
                                                    const uint64_t* surv, const uint32_t* nsurv, uint32_t bcap,
                                                    uint64_t* cand) {
    // per lane, at odd dword strides (5 and 17: lanes' slots start in different banks)
    __shared__ uint32_t syms[256 * 5];                    // the code-length code's symbols by rank (bytes)
    __shared__ uint32_t win[256 * 17];                    // staged input, 64 B
    uint8_t* T = (uint8_t*)(syms + threadIdx.x * 5);
    uint32_t* W = win + threadIdx.x * 17;
    const uint32_t wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    for (uint32_t r = wid; r < SPLIT_FILTER_BLOCKS; r += nw) {
        const uint32_t cnt = nsurv[r];
        const uint64_t* S = surv + (uint64_t)r * bcap;
        uint32_t next = 0;                                // next survivor to hand out (wave-uniform)
        bool act = false;
        uint64_t e = 0;
        DeepLane L;
        for (;;) {
            const uint64_t idle = __ballot(!act);
            const uint32_t nidle = (uint32_t)__popcll(idle);
            if (next < cnt && nidle >= 16) {
                if (!act) {
                    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                    if (next + rank < cnt) {
                        e = S[next + rank];
                        deep_start(L, T, W, in, in_off, sp, e);
                        act = true;
                    }
                }
                next += nidle;
            }
            if (!__ballot(act)) {
                if (next >= cnt) break;
                continue;
            }
            if (act) {
                const int st = deep_step(L, T);
                if (st) {
                    act = false;
                    if (st == 2) {
                        const uint32_t j = atomicAdd(&sp[L.k].ncand, 1u);
                        if (j < SP_CAND_MAX) cand[(uint64_t)L.k * SP_CAND_MAX + j] = e >> 20;
                    }
                }
            }
        }
    }
}

// bitonic sort of each stream's candidates in LDS (one workgroup per split stream)
__global__ __launch_bounds__(256) void k_split_sort(SplitInfo* sp, uint64_t* cand) {
    __shared__ uint64_t v[SP_CAND_MAX];
    SplitInfo& S = sp[blockIdx.x];
    const uint32_t n = S.ncand < SP_CAND_MAX ? S.ncand : SP_CAND_MAX;
    uint64_t* c = cand + (uint64_t)blockIdx.x * SP_CAND_MAX;
    uint32_t m = 1;
    while (m < n) m <<= 1;
    for (uint32_t k = threadIdx.x; k < m; k += 256) v[k] = k < n ? c[k] : ~0ull;
    __syncthreads();
    for (uint32_t size = 2; size <= m; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (uint32_t k = threadIdx.x; k < m; k += 256) {
                const uint32_t j = k ^ stride;
                if (j > k) {
                    const bool up = (k & size) == 0;
                    const uint64_t x = v[k], y = v[j];
                    if ((x > y) == up) { v[k] = y; v[j] = x; }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t k = threadIdx.x; k < n; k += 256) c[k] = v[k];
}

// the candidates of the streams that split (ncand <= SP_CAND_MAX), packed in stream order for
// the host's segment plan: one block scans the counts, then one block per stream copies
__global__ __launch_bounds__(1024) void k_split_pack_scan(SplitInfo* sp, uint32_t nsplit, uint32_t* total) {
    __shared__ uint32_t part[1024];
    uint32_t base = 0;
    for (uint32_t k0 = 0; k0 < nsplit; k0 += 1024) {
        const uint32_t k = k0 + threadIdx.x;
        const uint32_t c = k < nsplit && sp[k].ncand <= SP_CAND_MAX ? sp[k].ncand : 0u;
        part[threadIdx.x] = c;
        __syncthreads();
        for (uint32_t o = 1; o < 1024; o <<= 1) {         // inclusive scan
            const uint32_t v = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
            __syncthreads();
            part[threadIdx.x] += v;
            __syncthreads();
        }
        if (k < nsplit) sp[k].cand0 = base + part[threadIdx.x] - c;
        base += part[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = base;
}
__global__ __launch_bounds__(256) void k_split_pack(const SplitInfo* sp, const uint64_t* cand, uint64_t* packed) {
    const SplitInfo& S = sp[blockIdx.x];
    if (S.ncand > SP_CAND_MAX) return;
    const uint64_t* c = cand + (uint64_t)blockIdx.x * SP_CAND_MAX;
    for (uint32_t k = threadIdx.x; k < S.ncand; k += 256) packed[S.cand0 + k] = c[k];
}

__device__ __forceinline__ int64_t sp_find(const uint64_t* c, uint32_t n, uint64_t bit) {   // index of bit, or -1
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (c[mid] < bit) lo = mid + 1; else hi = mid;
    }
    return lo < n && c[lo] == bit ? (int64_t)lo : -1;
}

// one thread per split stream: walk its segments from the start; write the stream's decode
// state (the trailer parsed here) and its chain, or hand the stream to the serial path
__global__ void k_seg_chain(InflateArgs A, SplitInfo* sp, uint32_t nsplit, const SegInfo* seg, const uint64_t* cand,
                            const DSave* segD, uint32_t* chain, uint64_t* chain_tok, uint32_t* split_state) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nsplit) return;
    SplitInfo& S = sp[k];
    const uint32_t sid = S.sid;
    const uint64_t* c = cand + (uint64_t)k * SP_CAND_MAX;
    const uint32_t nc = S.ncand < SP_CAND_MAX ? S.ncand : SP_CAND_MAX;
    uint32_t* ch = chain + S.chain0;
    uint64_t* ct = chain_tok + S.chain0;
    uint32_t s = S.seg0, len = 0;
    uint64_t ntok = 0, out = 0;
    bool ok = S.ncand <= SP_CAND_MAX;
    const DSave* D = segD + s;
    while (ok) {
        D = segD + s;
        if (D->status != SDZ_OK || D->full || len > nc) { ok = false; break; }
        ch[len] = s;
        ct[len] = ntok;
        ++len;
        ntok += D->ntok;
        out += D->pos;
        if (D->stall == SEG_FINAL) break;
        if (D->stall != SEG_HANDOVER) { ok = false; break; }
        const int64_t j = sp_find(c, nc, D->bitpos);
        if (j < 0) { ok = false; break; }
        const uint32_t nx = S.seg0 + 1 + (uint32_t)j - S.skip0;   // segment of candidate j
        if (nx <= s || nx >= S.seg0 + S.nseg || seg[nx].bit != D->bitpos) { ok = false; break; }
        s = nx;
    }
    const DSave* H = segD + S.seg0;                        // the stream's start: container header
    DSave* O = (DSave*)A.dsave + sid;
    const uint64_t cap = A.out_cap[sid];
    const uint64_t nbits = A.in_len[sid] * 8;
    int status = SDZ_OK;
    int32_t ck = 0, size = 0;
    uint64_t end = D->bitpos;
    if (ok) {
        // the trailer (inflate.ts:423-463): WASH to a byte, then 4 (zlib) or 8 (gzip) bytes
        end = (end + 7) & ~7ull;
        const uint8_t* p = A.in + A.in_off[sid];
        const int tb = H->container == SDZ_CONTAINER_ZLIB ? 4 : H->container == SDZ_CONTAINER_GZIP ? 8 : 0;
        if (end + 8 * (uint64_t)tb > nbits || out > cap) ok = false;
        else if (tb == 4) {
            const uint8_t* q = p + (end >> 3);
            ck = (int32_t)(((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3]);
        } else if (tb == 8) {
            const uint8_t* q = p + (end >> 3);
            ck = (int32_t)((uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24));
            size = (int32_t)((uint32_t)q[4] | ((uint32_t)q[5] << 8) | ((uint32_t)q[6] << 16) | ((uint32_t)q[7] << 24));
        }
        end += 8 * (uint64_t)tb;
        status = end < nbits ? SDZ_TRAILING : SDZ_OK;
    }
    if (A.out_off[sid] & 7) ok = false;                  // (the serial path reports it)
    S.chain_len = ok ? len : 0;
    S.ntok = ok ? ntok : 0;
    split_state[sid] = ok ? SPS_FED : SPS_FALLBACK;
    if (!ok) return;
    O->mode = LM_DONE; O->status = status; O->zmsg = 0; O->stall = 0; O->full = 0;
    O->bitpos = end; O->pos = out;
    O->container = H->container; O->mtime = H->mtime; O->name_off = H->name_off; O->name_len = H->name_len;
    O->dict_used = H->dict_used; O->stored_ck = ck; O->stored_size = size;
    O->ntok = 0; O->litw = 0; O->nlit = 0;
}

// each round: the next round_tokens tokens of every chained stream, from its segments'
// buffers in chain order, into the stream's token ring (one workgroup per split stream)
__global__ __launch_bounds__(256) void k_seg_feed(InflateArgs A, const SplitInfo* sp, const SegInfo* seg,
                                                  const uint32_t* chain, const uint64_t* chain_tok,
                                                  const uint32_t* segtok, const uint32_t* split_state,
                                                  uint32_t round) {
    const SplitInfo& S = sp[blockIdx.x];
    const uint32_t sid = S.sid;
    if (split_state[sid] != SPS_FED) return;            // serial path
    const uint64_t T = A.round_tokens, t0 = (uint64_t)round * T;
    if (t0 > S.ntok || (t0 == S.ntok && round > 0)) {    // finished in an earlier round
        if (threadIdx.x == 0) { A.ntok[sid] = 0; A.flags[sid] = 2; }
        return;
    }
    const uint64_t t1 = t0 + T < S.ntok ? t0 + T : S.ntok;
    const uint32_t* ch = chain + S.chain0;
    const uint64_t* ct = chain_tok + S.chain0;
    uint32_t* dst = A.tokens + (uint64_t)sid * T;
    uint32_t lo = 0, hi = S.chain_len;                   // the chain entry holding stream token t0
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ct[mid] <= t0) lo = mid; else hi = mid;
    }
    // entry by entry, the whole block copies the entry's part of [t0, t1)
    for (uint32_t c = lo; c < S.chain_len && ct[c] < t1; ++c) {
        const uint64_t a = ct[c] > t0 ? ct[c] : t0;
        const uint64_t b = c + 1 < S.chain_len && ct[c + 1] < t1 ? ct[c + 1] : t1;
        const uint32_t* src = segtok + seg[ch[c]].tok + (a - ct[c]);
        uint32_t* d = dst + (a - t0);
        for (uint64_t t = threadIdx.x; t < b - a; t += 256) d[t] = src[t];
    }
    if (threadIdx.x == 0) {
        const bool last = t1 == S.ntok;
        A.ntok[sid] = (uint32_t)(t1 - t0);
        A.flags[sid] = last ? 1u : 0u;
        if (!last) atomicAdd(A.active, 1u);
    }
}

void launch_split_pack(SplitInfo* sp, uint32_t nsplit, const uint64_t* cand, uint64_t* packed, uint32_t* total,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_split_pack_scan, dim3(1), dim3(1024), 0, s, sp, nsplit, total);
    hipLaunchKernelGGL(k_split_pack, dim3(nsplit), dim3(256), 0, s, sp, cand, packed);
}
void launch_split_find(const uint8_t* in, const uint64_t* in_off, SplitInfo* sp, uint32_t nsplit, uint64_t* cand,
                       uint64_t total_lanes, uint64_t* surv, uint32_t* nsurv, uint32_t cap, hipStream_t s) {
    // persistent: each block a contiguous lane range and its own survivor region (cap / 8192
    // entries; nsurv: SPLIT_FILTER_BLOCKS counts, zeroed by the caller)
    const uint64_t blocks = SPLIT_FILTER_BLOCKS;
    const uint64_t per = ((total_lanes + blocks - 1) / blocks + 255) & ~255ull;
    const uint32_t bcap = cap / SPLIT_FILTER_BLOCKS;
    hipLaunchKernelGGL(k_split_filter, dim3((uint32_t)((total_lanes + per - 1) / per)), dim3(256), 0, s, in, in_off,
                       sp, nsplit, total_lanes, per, surv, nsurv, bcap);
    hipLaunchKernelGGL(k_split_deep, dim3(SPLIT_FILTER_BLOCKS / 4), dim3(256), 0, s, in, in_off, sp, surv, nsurv,
                       bcap, cand);                       // one wave per survivor region
    hipLaunchKernelGGL(k_split_sort, dim3(nsplit), dim3(256), 0, s, sp, cand);
}
void launch_seg_chain(const InflateArgs& a, SplitInfo* sp, uint32_t nsplit, const SegInfo* seg, const uint64_t* cand,
                      const void* segD, uint32_t* chain, uint64_t* chain_tok, uint32_t* split_state, hipStream_t s) {
    hipLaunchKernelGGL(k_seg_chain, dim3((nsplit + 63) / 64), dim3(64), 0, s, a, sp, nsplit, seg, cand,
                       (const DSave*)segD, chain, chain_tok, split_state);
}
void launch_seg_feed(const InflateArgs& a, uint32_t round, hipStream_t s) {
    const SplitPlan& P = *a.split_plan;
    hipLaunchKernelGGL(k_seg_feed, dim3(P.nsplit), dim3(256), 0, s, a, P.sp, P.seg, P.chain, P.chain_tok,
                       P.segtok, a.split_state, round);
}

}  // namespace sdz
