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

// Pass 1 (k_split_filter): one lane tests 32 consecutive bit positions -- the block-type bits
// of all 32 at once from a 64-bit window, then HLIT/HDIST and the Kraft sum of the code-length
// code (its order does not matter for the sum) from registers.  About 0.1 % of positions pass
// (measured on zlib output); they are appended, (position << 20 | split index), to a list.
// Each block walks a contiguous range of lanes, so the split stream of a lane is found by
// stepping forward, not by a search per lane.
__global__ __launch_bounds__(256) void k_split_filter(const uint8_t* in, const uint64_t* in_off, const SplitInfo* sp,
                                                      uint32_t nsplit, uint64_t total_lanes, uint64_t lanes_per_block,
                                                      uint64_t* surv, uint32_t* nsurv, uint32_t cap) {
    const uint64_t L0 = (uint64_t)blockIdx.x * lanes_per_block;
    if (L0 >= total_lanes) return;
    const uint64_t L1 = L0 + lanes_per_block < total_lanes ? L0 + lanes_per_block : total_lanes;
    uint32_t lo = 0, hi = nsplit;                         // the split stream holding lane L0
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sp[mid].lane0 <= L0) lo = mid; else hi = mid;
    }
    uint32_t k = lo;
    for (uint64_t g = L0 + threadIdx.x; g < L1; g += 256) {
        while (k + 1 < nsplit && sp[k + 1].lane0 <= g) ++k;
        const SplitInfo& S = sp[k];
        const uint64_t p0 = 32 * (g - S.lane0);
        const uint64_t nbits = S.nbits;
        const uint32_t* p32 = (const uint32_t*)(in + in_off[S.sid] + (p0 >> 3));   // 4-byte aligned
        uint32_t w0 = p32[0], w1 = p32[1], w2 = p32[2], w3 = p32[3];   // 64 B of slack past every input
        const uint64_t W = (uint64_t)w0 | ((uint64_t)w1 << 32);
        uint32_t M = (uint32_t)((~W >> 1) & (W >> 2));        // BTYPE = 2 (bits 1, 2 = 0, 1)
        uint64_t out[4];
        uint32_t no = 0;
        while (M) {
            const uint32_t i = (uint32_t)__builtin_ctz(M);
            M &= M - 1;
            const uint32_t a = __builtin_amdgcn_alignbit(w1, w0, i);    // bits i .. i+31
            const uint32_t b = __builtin_amdgcn_alignbit(w2, w1, i);    // bits i+32 .. i+63
            const uint32_t c = __builtin_amdgcn_alignbit(w3, w2, i);    // bits i+64 .. i+95
            const uint32_t hlit = (a >> 3) & 31u, hdist = (a >> 8) & 31u, hclen = (a >> 13) & 15u;
            const uint64_t q = (((uint64_t)b << 32) | a) >> 17;          // fields 0..14 of the code-length code
            const uint32_t r = (uint32_t)((((uint64_t)c << 32) | b) >> 30);   // fields 15..18
            uint32_t kraft = 0;
#pragma unroll
            for (int f = 0; f < 19; ++f) {
                const uint32_t len = f < 15 ? (uint32_t)(q >> (3 * f)) & 7u : (r >> (3 * (f - 15))) & 7u;
                kraft += (f < (int)hclen + 4 && len) ? 128u >> len : 0u;
            }
            const bool pass = hlit <= 29 && hdist <= 29 && kraft == 128u && p0 + i + 17 + 57 <= nbits;
            if (pass && no < 4) out[no++] = ((p0 + i) << 20) | k;
        }
        // append this lane's survivors (at most 4 of 32 positions: more is not a real stream)
        const uint64_t bm = __ballot(no != 0);
        if (bm) {
            uint32_t tot = no;                             // wave prefix of the counts
            uint32_t pre = 0;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = __shfl_up(tot, o);
                if ((threadIdx.x & 63u) >= (uint32_t)o) tot += v;
            }
            pre = tot - no;
            const uint32_t wsum = __shfl(tot, 63);
            uint32_t base = 0;
            if ((threadIdx.x & 63u) == 63u) base = atomicAdd(nsurv, wsum);
            base = __shfl(base, 63);
            for (uint32_t j = 0; j < no; ++j)
                if (base + pre + j < cap) surv[base + pre + j] = out[j];
        }
    }
}

// Pass 2 (k_split_deep): one lane per survivor decodes the code lengths (infblocks.ts:354-551 /
// inftree.ts:313-379 on a strict reading: every code complete) with the code-length code in a
// 128-entry LDS table, and keeps Kraft sums of the literal/length and distance lengths as it
// goes, so a random bit string is rejected after a few lengths.  Survivors are candidates.
__global__ __launch_bounds__(256) void k_split_deep(const uint8_t* in, const uint64_t* in_off, SplitInfo* sp,
                                                    const uint64_t* surv, const uint32_t* nsurv, uint32_t cap,
                                                    uint64_t* cand) {
    __shared__ uint8_t lut[256][128];                     // 7 stream bits -> symbol << 3 | code length
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    const uint32_t ns = *nsurv < cap ? *nsurv : cap;
    if (t >= ns) return;
    const uint64_t e = surv[t];
    const uint32_t k = (uint32_t)(e & 0xfffffu);
    uint64_t pos = e >> 20;
    SplitInfo& S = sp[k];
    const uint8_t* p = in + in_off[S.sid];
    const uint64_t nbits = S.nbits;
    const uint64_t h = sp_bits(p, pos, 17);
    const int hlit = (int)((h >> 3) & 31u) + 257, hdist = (int)((h >> 8) & 31u) + 1, hclen = (int)(h >> 13) + 4;
    pos += 17;
    uint64_t cl = 0;                                      // the 19 lengths, 3 bits each, symbol order
    for (int i = 0; i < hclen; ++i) { cl |= (uint64_t)sp_bits(p, pos, 3) << (3 * c_split_border[i]); pos += 3; }
    uint8_t* T = lut[threadIdx.x];
    {
        int code = 0;
        for (int l = 1; l < 8; ++l) {                     // canonical codes, MSB first in the stream
            for (int sym = 0; sym < 19; ++sym) {
                if ((int)((cl >> (3 * sym)) & 7u) != l) continue;
                uint32_t rev = 0;
                for (int j = 0; j < l; ++j) rev |= (uint32_t)((code >> (l - 1 - j)) & 1) << j;
                for (uint32_t x = rev; x < 128u; x += 1u << l) T[x] = (uint8_t)(sym << 3 | l);
                ++code;
            }
            code <<= 1;
        }
    }
    const int total = hlit + hdist;
    int n = 0, prev = 0;
    uint32_t kl = 0, kd = 0;                              // Kraft sums in units of 2^-15
    bool eob = false;
    while (n < total) {
        if (pos + 14 > nbits) return;
        const uint32_t w = sp_bits(p, pos, 14);
        const uint32_t v = T[w & 127u];
        const int sym = (int)(v >> 3), l = (int)(v & 7u);
        pos += (uint64_t)l;
        int rep = 1, val = sym;
        if (sym >= 16) {
            const int eb = sym == 16 ? 2 : sym == 17 ? 3 : 7;
            rep = (sym == 18 ? 11 : 3) + (int)((w >> l) & ((1u << eb) - 1u));
            pos += (uint64_t)eb;
            if (sym == 16 && n == 0) return;
            val = sym == 16 ? prev : 0;
            if (n + rep > total) return;
        }
        if (val) {
            const uint32_t u = 32768u >> val;
            const int nl = n < hlit ? (hlit - n < rep ? hlit - n : rep) : 0;   // of them literal/length
            kl += (uint32_t)nl * u;
            kd += (uint32_t)(rep - nl) * u;
            eob = eob || (n <= 256 && 256 < n + nl);
            if (kl > 32768u || kd > 32768u) return;
        }
        n += rep;
        prev = val;
    }
    if (!(eob && kl == 32768u && kd == 32768u)) return;
    const uint32_t j = atomicAdd(&S.ncand, 1u);
    if (j < SP_CAND_MAX) cand[(uint64_t)k * SP_CAND_MAX + j] = e >> 20;
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

void launch_split_find(const uint8_t* in, const uint64_t* in_off, SplitInfo* sp, uint32_t nsplit, uint64_t* cand,
                       uint64_t total_lanes, uint64_t* surv, uint32_t* nsurv, uint32_t cap, hipStream_t s) {
    const uint64_t blocks = 8192;                         // persistent: each block a contiguous lane range
    const uint64_t per = ((total_lanes + blocks - 1) / blocks + 255) & ~255ull;
    hipLaunchKernelGGL(k_split_filter, dim3((uint32_t)((total_lanes + per - 1) / per)), dim3(256), 0, s, in, in_off,
                       sp, nsplit, total_lanes, per, surv, nsurv, cap);
    hipLaunchKernelGGL(k_split_deep, dim3((cap + 255) / 256), dim3(256), 0, s, in, in_off, sp, surv, nsurv, cap, cand);
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
