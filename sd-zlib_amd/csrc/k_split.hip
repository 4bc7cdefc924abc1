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

// n <= 25 bits at bit position `pos` of p (byte loads: any alignment, reads <= 4 bytes on)
__device__ __forceinline__ uint32_t sp_bits(const uint8_t* p, uint64_t pos, int n) {
    const uint8_t* q = p + (pos >> 3);
    const uint32_t v = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
    return (v >> (pos & 7)) & ((1u << n) - 1u);
}

// The deep test from the code-length code on (infblocks.ts:354-551 / inftree.ts:313-379 on a
// strict reading: every code complete).  cl: the 19 code-length code lengths.  Literal/
// length and distance lengths are summed into Kraft counters as they are decoded, so a
// random bit string is usually rejected after a few lengths.
__device__ __noinline__ bool sp_deep(const uint8_t* p, uint64_t nbits, uint64_t pos, int hlit, int hdist,
                                     uint64_t cl) {
    int cnt[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) cnt[k] = 0;
    for (int s = 0; s < 19; ++s) cnt[(cl >> (3 * s)) & 7]++;
    // canonical code-length code: first code and first index per length
    int first[8], base[8];
    uint8_t syms[19];
    {
        int code = 0, k = 0;
        for (int l = 1; l < 8; ++l) {
            first[l] = code;
            base[l] = k;
            for (int s = 0; s < 19; ++s)
                if ((int)((cl >> (3 * s)) & 7) == l) syms[k++] = (uint8_t)s;
            code = (code + cnt[l]) << 1;
        }
    }
    const int total = hlit + hdist;
    int n = 0, prev = 0;
    uint32_t kl = 0, kd = 0;                              // Kraft sums in units of 2^-15
    bool eob = false;
    while (n < total) {
        if (pos + 7 + 7 > nbits) return false;
        const uint32_t w = sp_bits(p, pos, 14);
        int code = 0, sym = -1, l = 1;
        for (; l < 8; ++l) {
            code = (code << 1) | (int)((w >> (l - 1)) & 1u);
            if (cnt[l] && code - first[l] < cnt[l]) { sym = syms[base[l] + code - first[l]]; break; }
        }
        if (sym < 0) return false;
        pos += (uint64_t)l;
        int rep = 1, val = sym;
        if (sym >= 16) {
            const int eb = sym == 16 ? 2 : sym == 17 ? 3 : 7;
            const int r = (int)((w >> l) & ((1u << eb) - 1u));
            pos += (uint64_t)eb;
            rep = (sym == 16 ? 3 : sym == 17 ? 3 : 11) + r;
            if (sym == 16 && n == 0) return false;
            val = sym == 16 ? prev : 0;
            if (n + rep > total) return false;
        }
        if (val) {
            const uint32_t u = 32768u >> val;
            for (int r = 0; r < rep; ++r, ++n) {
                if (n < hlit) { kl += u; if (n == 256) eob = true; }
                else kd += u;
            }
            if (kl > 32768u || kd > 32768u) return false;
        } else {
            n += rep;
        }
        prev = val;
    }
    return eob && kl == 32768u && kd == 32768u;
}

// One lane tests 32 consecutive bit positions: the block-type bits of all 32 at once from a
// 64-bit window, then the header fields and the code-length code's Kraft sum (from a
// 160-bit window in registers) for the survivors, then the deep test for the rare rest.
__global__ __launch_bounds__(256) void k_split_find(const uint8_t* in, const uint64_t* in_off, SplitInfo* sp,
                                                    uint32_t nsplit, uint64_t* cand, uint64_t total_lanes) {
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= total_lanes) return;
    uint32_t lo = 0, hi = nsplit;                         // the stream whose lane range holds g
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sp[mid].lane0 <= g) lo = mid; else hi = mid;
    }
    SplitInfo& S = sp[lo];
    const uint64_t p0 = 32 * (g - S.lane0);
    const uint64_t nbits = S.nbits;
    if (p0 >= nbits) return;
    const uint8_t* p = in + in_off[S.sid];
    uint32_t w[5];
    const uint32_t* p32 = (const uint32_t*)(p + (p0 >> 3));   // p0 is a multiple of 32: 4-byte aligned
#pragma unroll
    for (int k = 0; k < 5; ++k) w[k] = p32[k];                // 64 B of slack past every input
    const uint64_t W = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    uint32_t M = (uint32_t)((~W >> 1) & (W >> 2));            // BTYPE = 2 (bits 1, 2 = 0, 1)
    while (M) {
        const int i = __builtin_ctz(M);
        M &= M - 1;
        const uint64_t pos = p0 + (uint64_t)i;
        if (pos + 17 + 57 > nbits) continue;
        auto win = [&](int b) -> uint32_t {                  // 32 bits from bit b of the window
            const int k = b >> 5, s = b & 31;
            const uint32_t a = k == 0 ? w[0] : k == 1 ? w[1] : k == 2 ? w[2] : w[3];
            const uint32_t c = k == 0 ? w[1] : k == 1 ? w[2] : k == 2 ? w[3] : w[4];
            return s ? (a >> s) | (c << (32 - s)) : a;
        };
        const uint32_t h = win(i) & 0x1ffffu;
        const int hlit = (int)((h >> 3) & 31u), hdist = (int)((h >> 8) & 31u), hclen = (int)(h >> 13) + 4;
        if (hlit > 29 || hdist > 29) continue;
        const uint32_t a = win(i + 17), b = win(i + 17 + 32);
        const uint64_t bits = (uint64_t)a | ((uint64_t)b << 32);  // the code-length code lengths
        uint64_t cl = 0;
        uint32_t kraft = 0;
        for (int k = 0; k < hclen; ++k) {
            const uint32_t len = (uint32_t)(bits >> (3 * k)) & 7u;
            cl |= (uint64_t)len << (3 * c_split_border[k]);
            kraft += len ? 128u >> len : 0u;
        }
        if (kraft != 128u) continue;                      // complete code-length code
        if (!sp_deep(p, nbits, pos + 17 + 3 * (uint64_t)hclen, hlit + 257, hdist + 1, cl)) continue;
        const uint32_t k = atomicAdd(&S.ncand, 1u);
        if (k < SP_CAND_MAX) cand[(uint64_t)lo * SP_CAND_MAX + k] = pos;
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
    S.chain_len = ok ? len : 0;
    S.ntok = ok ? ntok : 0;
    split_state[sid] = ok ? 1u : 0u;
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
    if (!split_state[sid]) return;                       // serial path
    const uint64_t T = A.round_tokens, t0 = (uint64_t)round * T;
    if (t0 > S.ntok || (t0 == S.ntok && round > 0)) {    // finished in an earlier round
        if (threadIdx.x == 0) { A.ntok[sid] = 0; A.flags[sid] = 2; }
        return;
    }
    const uint64_t t1 = t0 + T < S.ntok ? t0 + T : S.ntok;
    const uint32_t* ch = chain + S.chain0;
    const uint64_t* ct = chain_tok + S.chain0;
    uint32_t* dst = A.tokens + (uint64_t)sid * T;
    for (uint64_t t = t0 + threadIdx.x; t < t1; t += 256) {
        uint32_t lo = 0, hi = S.chain_len;               // the chain entry holding stream token t
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (ct[mid] <= t) lo = mid; else hi = mid;
        }
        dst[t - t0] = segtok[seg[ch[lo]].tok + (t - ct[lo])];
    }
    if (threadIdx.x == 0) {
        const bool last = t1 == S.ntok;
        A.ntok[sid] = (uint32_t)(t1 - t0);
        A.flags[sid] = last ? 1u : 0u;
        if (!last) atomicAdd(A.active, 1u);
    }
}

void launch_split_find(const uint8_t* in, const uint64_t* in_off, SplitInfo* sp, uint32_t nsplit, uint64_t* cand,
                       uint64_t total_lanes, hipStream_t s) {
    hipLaunchKernelGGL(k_split_find, dim3((uint32_t)((total_lanes + 255) / 256)), dim3(256), 0, s, in, in_off, sp,
                       nsplit, cand, total_lanes);
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
