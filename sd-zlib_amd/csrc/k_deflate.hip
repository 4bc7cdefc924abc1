// k_deflate.hip -- batched, bit-exact DEFLATE encoder for gfx950 (MI355X).
//
// Replaces the serial compressor of @stardazed/zlib:
//   Deflate (fill_window, longest_match, deflate_fast/slow, _tr_tally,
//            _tr_flush_block, compress_block, send_bits)   src/deflate.ts:102-1327
//   Tree (build_tree, gen_bitlen, gen_codes)                src/deftree.ts:40-267
//   config_table                                            src/defconfig.ts:33-44
//   Deflater container header/trailer                       src/sd-deflate.ts:98-253
//
// v1 design: one lane per stream, the reference's exact state machine, with the
// per-stream state (64 KiB window, 32 K-entry head/prev chains, the 64 KiB
// pending_buf with its d_buf@8192 / l_buf@49152 overlay, trees) in an HBM
// scratch slab, scalars in registers.  Bit-exactness needs the reference's
// quirks verbatim: TRUNCATE_BLOCK, 4-byte clz compare from +2,
// stale window bytes past the input, the pending_buf overlay, (freq, depth)
// heap ties.  The output is produced with the reference's block decisions and
// flushed straight into the stream's output slot.
#include "sdz_internal.h"

namespace sdz {

#define DF_THREADS 64
#define GLB __attribute__((address_space(1)))   // global memory (no flat ops)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define W_SIZE 32768
#define W_MASK (W_SIZE - 1)
#define WINDOW_SIZE (2 * W_SIZE)
#define HASH_SIZE 32768
#define HASH_MASK (HASH_SIZE - 1)
#define HASH_SHIFT 5
#define LIT_BUFSIZE 16384
#define PENDING_SIZE (4 * LIT_BUFSIZE)
#define D_BUF (LIT_BUFSIZE / 2)
#define L_BUF (3 * LIT_BUFSIZE)
#define MIN_MATCH 3
#define MAX_MATCH 258
#define MIN_LOOKAHEAD (MAX_MATCH + MIN_MATCH + 1)
#define MAX_DIST (W_SIZE - MIN_LOOKAHEAD)
#define L_CODES 286
#define D_CODES 30
#define BL_CODES 19
#define HEAP_SIZE (2 * L_CODES + 1)
#define END_BLOCK 256

// the scalar state of a Deflater between appends (sdz_deflate_append_batch_device)
struct DfScal {
    int32_t status;                 // 0 INIT (nothing appended), 1 BUSY, 2 FINISH (deflate.ts DeflateState)
    int32_t checksum;               // running adler32 / crc32 of the input (sd-deflate.ts:185-190)
    uint32_t orig;                  // input bytes so far, mod 2^32 (sd-deflate.ts:191)
    int32_t pending, ins_h, block_start, match_length, match_available, strstart, match_start, lookahead,
        prev_length, last_lit, matches, opt_len, static_len, bi_valid;
    uint32_t bi_buf;
};

struct DSlab {                      // per-stream HBM state
    uint8_t window[WINDOW_SIZE];
    uint8_t pending[PENDING_SIZE];
    uint16_t prev[W_SIZE];
    uint16_t head[HASH_SIZE];
    uint16_t ltree[HEAP_SIZE * 2];
    uint16_t dtree[(2 * D_CODES + 1) * 2];
    uint16_t bltree[(2 * BL_CODES + 1) * 2];
    uint16_t depth[2 * L_CODES + 1];
    uint16_t heap[2 * L_CODES + 1];
    uint16_t bl_count[16];
    uint16_t next_code[16];
    DfScal sc;                      // incremental Deflater only
};

#define SLAB_BYTES ((sizeof(DSlab) + 255) & ~(uint64_t)255)

// record path (inputs up to kDeflateRecMax): per stream a FStream header in its
// slab, and per block a slot (FBlock + code table + header words) in the block area; records,
// links and symbols in the record buffers (positions from rp0[k]).
#define PM_TAIL (MAX_MATCH + MIN_MATCH + 1)       // last positions: searched by k_dfl_tail
#define FB_TAB_BYTES 2048                           // per block: codes + header words
#define FB_HDR_OFF 1280                             // header words within a block's table
#define FB_HDR_WORDS 176
#define FB_SLOT (64 + FB_TAB_BYTES)                 // FBlock, then the table
struct FBlock {
    uint32_t sym0, nsym;            // the block's symbols in the stream's symbol buffer
    int32_t block_start, strstart;  // reference (window) coordinates at the flush
    int64_t off;                    // original position of window index 0 at the flush
    uint32_t eof;
    uint32_t type;                  // k_dfl_trees: 0 stored, 1 static, 2 dynamic
    uint32_t hbits;                 // header bits (3 block-type bits + dynamic tree description)
    uint32_t dbits;                 // symbol bits incl. END_BLOCK (static / dynamic)
    uint32_t stored_len;
    uint32_t carry;                 // k_dfl_encode: bi_valid at the block's start
    uint64_t bstart;                // k_dfl_encode: the block's first bit in the output slot
};
struct FStream {
    uint32_t nblk;
    uint32_t flag;                  // nonzero: the stream is redone by the serial kernel
    uint32_t pad[2];
};
static_assert(sizeof(FBlock) <= 64, "FBlock fits its slot head");
static_assert(FB_HDR_OFF >= (L_CODES + D_CODES) * 4 && FB_HDR_OFF + FB_HDR_WORDS * 4 <= FB_TAB_BYTES, "table layout");

uint64_t deflate_state_bytes() { return SLAB_BYTES; }
uint64_t deflate_rec_blocks(uint64_t len) { return len / 8192 + 2; }   // a non-final block covers >= 8192 symbols

// tables shared by all streams (deftree.ts:25-38, 269-298, 319-337)
struct DTables {
    uint8_t dist_code[512];
    uint8_t length_code[256];
    uint16_t base_length[29];
    uint16_t base_dist[30];
    uint16_t static_ltree[288 * 2];
    uint16_t static_dtree[30 * 2];
    uint8_t extra_lbits[29], extra_dbits[30], extra_blbits[19];
};
__device__ DTables g_dt;                                     // built once per device (dt_ready)
__constant__ uint8_t c_extra_lbits[29] = { 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0 };
__constant__ uint8_t c_extra_dbits[30] = { 0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13 };
__constant__ uint8_t c_extra_blbits[19] = { 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7 };
__constant__ uint8_t c_bl_order[19] = { 16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15 };
// defconfig.ts:33-44 {good, lazy, nice, chain, fast?}
__constant__ int c_config[10][5] = {
    { 0, 0, 0, 0, 0 }, { 4, 4, 8, 4, 1 }, { 4, 5, 16, 8, 1 }, { 4, 6, 32, 32, 1 },
    { 4, 4, 16, 16, 0 }, { 8, 16, 32, 32, 0 }, { 8, 16, 128, 128, 0 }, { 8, 32, 128, 256, 0 },
    { 32, 128, 258, 1024, 0 }, { 32, 258, 258, 4096, 0 } };

__device__ __forceinline__ uint32_t bitrev_n(uint32_t code, int len) {
    return __builtin_bitreverse32(code) >> (32 - len);
}

// build the shared tables in LDS (zlib trees.h derivation, deftree.ts literals)
__global__ void k_deflate_tables() {
    DTables& T = g_dt;
    {
        for (int i = 0; i < 29; ++i) T.extra_lbits[i] = c_extra_lbits[i];
        for (int i = 0; i < 30; ++i) T.extra_dbits[i] = c_extra_dbits[i];
        for (int i = 0; i < 19; ++i) T.extra_blbits[i] = c_extra_blbits[i];
        int length = 0, code, n, dist;
        for (code = 0; code < 28; code++) {
            T.base_length[code] = (uint16_t)length;
            for (n = 0; n < (1 << c_extra_lbits[code]); n++) T.length_code[length++] = (uint8_t)code;
        }
        T.length_code[length - 1] = (uint8_t)code;
        T.base_length[28] = 0;
        dist = 0;
        for (code = 0; code < 16; code++) {
            T.base_dist[code] = (uint16_t)dist;
            for (n = 0; n < (1 << c_extra_dbits[code]); n++) T.dist_code[dist++] = (uint8_t)code;
        }
        T.dist_code[256] = 0; T.dist_code[257] = 0;
        dist >>= 7;
        for (; code < 30; code++) {
            T.base_dist[code] = (uint16_t)(dist << 7);
            for (n = 0; n < (1 << (c_extra_dbits[code] - 7)); n++) T.dist_code[256 + dist++] = (uint8_t)code;
        }
        int nc[16] = { 0 }, cnt[16] = { 0 };
        for (n = 0; n < 288; n++) {
            int l = n < 144 ? 8 : n < 256 ? 9 : n < 280 ? 7 : 8;
            T.static_ltree[n * 2 + 1] = (uint16_t)l;
            cnt[l]++;
        }
        int c = 0;
        for (int b = 1; b < 16; b++) { c = (c + cnt[b - 1]) << 1; nc[b] = c; }
        for (n = 0; n < 288; n++) {
            int l = T.static_ltree[n * 2 + 1];
            T.static_ltree[n * 2] = (uint16_t)bitrev_n((uint32_t)nc[l]++, l);
        }
        for (n = 0; n < 30; n++) { T.static_dtree[n * 2 + 1] = 5; T.static_dtree[n * 2] = (uint16_t)bitrev_n((uint32_t)n, 5); }
    }
}

// the tables depend on nothing: built on a device's first compress call, and waited for there
// (a later call may run on another stream)
static bool g_dt_ready[64];
static void dt_ready(hipStream_t s) {
    int d = 0;
    if (hipGetDevice(&d) == hipSuccess && d >= 0 && d < 64 && g_dt_ready[d]) return;
    hipLaunchKernelGGL(k_deflate_tables, dim3(1), dim3(1), 0, s);
    if (hipStreamSynchronize(s) == hipSuccess && d >= 0 && d < 64) g_dt_ready[d] = true;
}

// scalar state of one stream (deflate.ts:102-194), registers
struct DS {
    GLB DSlab* S;
    const GLB DTables* T;
    const GLB uint8_t* in;
    uint64_t in_len, in_pos;
    GLB uint8_t* out;
    uint64_t out_cap, out_len;
    int pending;
    int ins_h, block_start, match_length, match_available, strstart, match_start, lookahead, prev_length;
    int level, good_match, nice_match, max_chain, max_lazy;
    int last_lit, matches;
    int opt_len, static_len;
    uint32_t bi_buf;
    int bi_valid;
    int heap_len, heap_max;
    int l_max_code, d_max_code, bl_max_code;
    int err;                        // 1 = pending_buf overflow (reference undefined), 2 = out overflow
#ifdef SDZ_TIMING
    bool timed;
    unsigned long long tlast, tacc[8];
#endif
};
#ifdef SDZ_TIMING                   // development aid: cycles per phase, lane 0 of a few waves
#define DF_STAMP(s, k) do { if ((s).timed) { const unsigned long long t_ = clock64(); (s).tacc[k] += t_ - (s).tlast; (s).tlast = t_; } } while (0)
#else
#define DF_STAMP(s, k) do {} while (0)
#endif

// ------------------------------------------------------------------ bit writer (deflate.ts:347-374)

__device__ __forceinline__ void pput(DS& s, int idx, uint32_t v) {
    if ((unsigned)idx < PENDING_SIZE) s.S->pending[idx] = (uint8_t)v; else s.err |= 1;
}
__device__ __forceinline__ void put_short(DS& s, uint32_t w) {
    pput(s, s.pending++, w & 0xff);
    pput(s, s.pending++, (w >> 8) & 0xff);
}
__device__ __forceinline__ void send_bits(DS& s, uint32_t value, int length) {
    if (s.bi_valid > 16 - length) {
        s.bi_buf |= (value << s.bi_valid) & 0xffff;
        pput(s, s.pending, s.bi_buf);
        pput(s, s.pending + 1, s.bi_buf >> 8);
        s.pending += 2;
        s.bi_buf = value >> (16 - s.bi_valid);
        s.bi_valid += length - 16;
    } else {
        s.bi_buf |= (value << s.bi_valid) & 0xffff;
        s.bi_valid += length;
    }
}
__device__ __forceinline__ void send_code(DS& s, int c, const GLB uint16_t* tree) {
    send_bits(s, tree[c * 2], tree[c * 2 + 1]);
}

// ------------------------------------------------------------------ trees (deftree.ts)

// The tree builders are templated on a context C (heap / depth / bl_count / next_code /
// bltree arrays + heap_len, heap_max, opt_len, static_len) so the serial path (HBM slab)
// and the record path's tree kernel (LDS) run the same code.
template <class TP, class DP>
__device__ __forceinline__ bool smaller(TP tree, int n, int m, DP depth) {
    int tn = tree[n * 2], tm = tree[m * 2];
    return tn < tm || (tn == tm && depth[n] <= depth[m]);
}

template <class C, class TP>
__device__ void pqdownheap(C& s, TP tree, int k) {                            // deflate.ts:241-263
    auto* heap = s.heap;
    auto* depth = s.depth;
    int v = heap[k];
    int j = k << 1;
    while (j <= s.heap_len) {
        if (j < s.heap_len && smaller(tree, heap[j + 1], heap[j], depth)) j++;
        if (smaller(tree, v, heap[j], depth)) break;
        heap[k] = heap[j];
        k = j;
        j <<= 1;
    }
    heap[k] = (uint16_t)v;
}

// deftree.ts:60-132 gen_bitlen
template <class C, class TP>
__device__ void gen_bitlen(C& s, TP tree, int max_code, const GLB uint16_t* stree,
                           const GLB uint8_t* extra, int base, int max_length) {
    auto* heap = s.heap;
    auto* bl_count = s.bl_count;
    int h, n, m, bits, xbits, f, overflow = 0;
    for (bits = 0; bits <= 15; bits++) bl_count[bits] = 0;
    tree[heap[s.heap_max] * 2 + 1] = 0;
    for (h = s.heap_max + 1; h < HEAP_SIZE; h++) {
        n = heap[h];
        bits = tree[tree[n * 2 + 1] * 2 + 1] + 1;
        if (bits > max_length) { bits = max_length; overflow++; }
        tree[n * 2 + 1] = (uint16_t)bits;
        if (n > max_code) continue;
        bl_count[bits]++;
        xbits = 0;
        if (n >= base) xbits = extra[n - base];
        f = tree[n * 2];
        s.opt_len += f * (bits + xbits);
        if (stree) s.static_len += f * (stree[n * 2 + 1] + xbits);
    }
    if (overflow == 0) return;
    do {
        bits = max_length - 1;
        while (bl_count[bits] == 0) bits--;
        bl_count[bits]--;
        bl_count[bits + 1] += 2;
        bl_count[max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    for (bits = max_length; bits != 0; bits--) {
        n = bl_count[bits];
        while (n != 0) {
            m = heap[--h];
            if (m > max_code) continue;
            if (tree[m * 2 + 1] != bits) {
                s.opt_len += (bits - tree[m * 2 + 1]) * tree[m * 2];
                tree[m * 2 + 1] = (uint16_t)bits;
            }
            n--;
        }
    }
}

// deftree.ts:155-182 gen_codes
template <class C, class TP>
__device__ void gen_codes(C& s, TP tree, int max_code) {
    auto* next_code = s.next_code;
    auto* bl_count = s.bl_count;
    int code = 0;
    for (int bits = 1; bits <= 15; bits++) {
        code = (code + bl_count[bits - 1]) << 1;
        next_code[bits] = (uint16_t)code;
    }
    for (int n = 0; n <= max_code; n++) {
        int len = tree[n * 2 + 1];
        if (len == 0) continue;
        tree[n * 2] = (uint16_t)bitrev_n(next_code[len]++, len);
    }
}

// deftree.ts:190-267 build_tree; returns max_code
template <class C, class TP>
__device__ int build_tree(C& s, TP tree, const GLB uint16_t* stree, const GLB uint8_t* extra,
                          int base, int elems, int max_length) {
    auto* heap = s.heap;
    auto* depth = s.depth;
    int n, m, max_code = -1, node;
    s.heap_len = 0;
    s.heap_max = HEAP_SIZE;
    for (n = 0; n < elems; n++) {
        if (tree[n * 2] != 0) { heap[++s.heap_len] = (uint16_t)(max_code = n); depth[n] = 0; }
        else tree[n * 2 + 1] = 0;
    }
    while (s.heap_len < 2) {
        node = max_code < 2 ? ++max_code : 0;
        heap[++s.heap_len] = (uint16_t)node;
        tree[node * 2] = 1;
        depth[node] = 0;
        s.opt_len--;
        if (stree) s.static_len -= stree[node * 2 + 1];
    }
    for (n = s.heap_len / 2; n >= 1; n--) pqdownheap(s, tree, n);
    node = elems;
    do {
        n = heap[1];
        heap[1] = heap[s.heap_len--];
        pqdownheap(s, tree, 1);
        m = heap[1];
        heap[--s.heap_max] = (uint16_t)n;
        heap[--s.heap_max] = (uint16_t)m;
        tree[node * 2] = (uint16_t)(tree[n * 2] + tree[m * 2]);
        depth[node] = (uint16_t)((depth[n] > depth[m] ? depth[n] : depth[m]) + 1);
        tree[n * 2 + 1] = tree[m * 2 + 1] = (uint16_t)node;
        heap[1] = (uint16_t)(node++);
        pqdownheap(s, tree, 1);
    } while (s.heap_len >= 2);
    heap[--s.heap_max] = heap[1];
    gen_bitlen(s, tree, max_code, stree, extra, base, max_length);
    gen_codes(s, tree, max_code);
    return max_code;
}

// deflate.ts:267-312 scan_tree
template <class C, class TP>
__device__ void scan_tree(C& s, TP tree, int max_code) {
    auto* bl = s.bltree;
    int prevlen = -1, curlen, nextlen = tree[1], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    tree[(max_code + 1) * 2 + 1] = 0xffff;
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = tree[(n + 1) * 2 + 1];
        if (++count < max_count && curlen == nextlen) continue;
        else if (count < min_count) bl[curlen * 2] = (uint16_t)(bl[curlen * 2] + count);
        else if (curlen != 0) { if (curlen != prevlen) bl[curlen * 2]++; bl[16 * 2]++; }
        else if (count <= 10) bl[17 * 2]++;
        else bl[18 * 2]++;
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

// deflate.ts:378-429 send_tree, through the context's bit writer
template <class C, class TP>
__device__ void send_tree(C& s, TP tree, int max_code) {
    auto* bl = s.bltree;
    int prevlen = -1, curlen, nextlen = tree[1], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = tree[(n + 1) * 2 + 1];
        if (++count < max_count && curlen == nextlen) continue;
        else if (count < min_count) { do { s.bits(bl[curlen * 2], bl[curlen * 2 + 1]); } while (--count != 0); }
        else if (curlen != 0) {
            if (curlen != prevlen) { s.bits(bl[curlen * 2], bl[curlen * 2 + 1]); count--; }
            s.bits(bl[16 * 2], bl[16 * 2 + 1]);
            s.bits((uint32_t)(count - 3), 2);
        } else if (count <= 10) { s.bits(bl[17 * 2], bl[17 * 2 + 1]); s.bits((uint32_t)(count - 3), 3); }
        else { s.bits(bl[18 * 2], bl[18 * 2 + 1]); s.bits((uint32_t)(count - 11), 7); }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

// tree context of the serial path: the slab's arrays, the stream's scalars, its bit writer
struct GTreeCtx {
    DS& ds;
    GLB uint16_t *heap, *depth, *bl_count, *next_code, *bltree;
    int heap_len, heap_max, opt_len, static_len;
    __device__ void bits(uint32_t v, int len) { send_bits(ds, v, len); }
};

__device__ __forceinline__ int d_code(const GLB DTables* T, int dist) {
    return dist < 256 ? T->dist_code[dist] : T->dist_code[256 + (dist >> 7)];
}

// deflate.ts:222-234
__device__ void init_block(DS& s) {
    for (int i = 0; i < L_CODES; i++) s.S->ltree[i * 2] = 0;
    for (int i = 0; i < D_CODES; i++) s.S->dtree[i * 2] = 0;
    for (int i = 0; i < BL_CODES; i++) s.S->bltree[i * 2] = 0;
    s.S->ltree[END_BLOCK * 2] = 1;
    s.opt_len = s.static_len = 0;
    s.last_lit = s.matches = 0;
}

// deflate.ts:488-524 _tr_tally (TRUNCATE_BLOCK heuristic kept)
__device__ __forceinline__ bool tr_tally(DS& s, int dist, int lc) {
    auto* pb = s.S->pending;
    pb[D_BUF + s.last_lit * 2] = (uint8_t)(dist >> 8);
    pb[D_BUF + s.last_lit * 2 + 1] = (uint8_t)dist;
    pb[L_BUF + s.last_lit] = (uint8_t)lc;
    s.last_lit++;
    if (dist == 0) {
        s.S->ltree[lc * 2]++;
    } else {
        s.matches++;
        dist--;
        s.S->ltree[(s.T->length_code[lc] + 257) * 2]++;
        s.S->dtree[d_code(s.T, dist) * 2]++;
    }
    if ((s.last_lit & 0x1fff) == 0 && s.level > 2) {
        uint32_t out_length = (uint32_t)s.last_lit * 8;
        int in_length = s.strstart - s.block_start;
        for (int dc = 0; dc < D_CODES; dc++) out_length += (uint32_t)s.S->dtree[dc * 2] * (5 + c_extra_dbits[dc]);
        out_length >>= 3;
        if (s.matches < s.last_lit / 2 && (int)out_length < in_length / 2) return true;
    }
    return s.last_lit == LIT_BUFSIZE - 1;
}

// deflate.ts:527-571 compress_block: reads d_buf/l_buf out of the pending_buf it writes
__device__ void compress_block(DS& s, const GLB uint16_t* ltree, const GLB uint16_t* dtree) {
    auto* pb = s.S->pending;
    int lx = 0;
    if (s.last_lit != 0) {
        do {
            int dist = (pb[D_BUF + lx * 2] << 8) | pb[D_BUF + lx * 2 + 1];
            int lc = pb[L_BUF + lx];
            lx++;
            if (dist == 0) {
                send_code(s, lc, ltree);
            } else {
                int code = s.T->length_code[lc];
                send_code(s, code + 257, ltree);
                int extra = c_extra_lbits[code];
                if (extra != 0) send_bits(s, (uint32_t)(lc - s.T->base_length[code]), extra);
                dist--;
                code = d_code(s.T, dist);
                send_code(s, code, dtree);
                extra = c_extra_dbits[code];
                if (extra != 0) send_bits(s, (uint32_t)(dist - s.T->base_dist[code]), extra);
            }
        } while (lx < s.last_lit);
    }
    send_code(s, END_BLOCK, ltree);
}

// deflate.ts:574-583
__device__ void bi_windup(DS& s) {
    if (s.bi_valid > 8) put_short(s, s.bi_buf);
    else if (s.bi_valid > 0) pput(s, s.pending++, s.bi_buf);
    s.bi_buf = 0;
    s.bi_valid = 0;
}

// zstream.ts:76-94 into the stream's output slot
__device__ void flush_pending(DS& s) {
    int len = s.pending;
    if (len == 0) return;
    if (s.out_len + (uint64_t)len > s.out_cap) { s.err |= 2; s.pending = 0; return; }
    if (len > PENDING_SIZE) { s.err |= 1; len = PENDING_SIZE; }
    auto* pb = s.S->pending;
    for (int i = 0; i < len; i++) s.out[s.out_len + i] = pb[i];
    s.out_len += (uint64_t)s.pending;
    s.pending = 0;
}

// deflate.ts:614-674 _tr_flush_block (+ flush_block_only 676-680)
__device__ __noinline__ void flush_block(DS& s, bool eof) {
    DF_STAMP(s, 1);
    int buf = s.block_start >= 0 ? s.block_start : -1;
    int stored_len = s.strstart - s.block_start;
    GTreeCtx c{s, s.S->heap, s.S->depth, s.S->bl_count, s.S->next_code, s.S->bltree,
               s.heap_len, s.heap_max, s.opt_len, s.static_len};
    s.l_max_code = build_tree(c, s.S->ltree, s.T->static_ltree, s.T->extra_lbits, 257, L_CODES, 15);
    s.d_max_code = build_tree(c, s.S->dtree, s.T->static_dtree, s.T->extra_dbits, 0, D_CODES, 15);
    // build_bl_tree (deflate.ts:316-339)
    scan_tree(c, s.S->ltree, s.l_max_code);
    scan_tree(c, s.S->dtree, s.d_max_code);
    build_tree(c, s.S->bltree, (const GLB uint16_t*)nullptr, s.T->extra_blbits, 0, BL_CODES, 7);
    s.heap_len = c.heap_len; s.heap_max = c.heap_max; s.opt_len = c.opt_len; s.static_len = c.static_len;
    int max_blindex;
    for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
        if (s.S->bltree[c_bl_order[max_blindex] * 2 + 1] != 0) break;
    s.opt_len += 3 * (max_blindex + 1) + 5 + 5 + 4;
    uint32_t opt_lenb = (uint32_t)(s.opt_len + 3 + 7) >> 3;
    uint32_t static_lenb = (uint32_t)(s.static_len + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    DF_STAMP(s, 2);
    if ((uint32_t)(stored_len + 4) <= opt_lenb && buf != -1) {
        send_bits(s, eof ? 1u : 0u, 3);                     // _tr_stored_block
        bi_windup(s);
        put_short(s, (uint32_t)stored_len);
        put_short(s, ~(uint32_t)stored_len);
        if (s.pending + stored_len > PENDING_SIZE) s.err |= 1;
        else {
            for (int i = 0; i < stored_len; i++) s.S->pending[s.pending + i] = s.S->window[buf + i];
            s.pending += stored_len;
        }
    } else if (static_lenb == opt_lenb) {
        send_bits(s, 2u + (eof ? 1u : 0u), 3);
        compress_block(s, s.T->static_ltree, s.T->static_dtree);
    } else {
        send_bits(s, 4u + (eof ? 1u : 0u), 3);
        int lcodes = s.l_max_code + 1, dcodes = s.d_max_code + 1, blcodes = max_blindex + 1;
        send_bits(s, (uint32_t)(lcodes - 257), 5);
        send_bits(s, (uint32_t)(dcodes - 1), 5);
        send_bits(s, (uint32_t)(blcodes - 4), 4);
        for (int rank = 0; rank < blcodes; rank++) send_bits(s, s.S->bltree[c_bl_order[rank] * 2 + 1], 3);
        GTreeCtx c{s, s.S->heap, s.S->depth, s.S->bl_count, s.S->next_code, s.S->bltree, 0, 0, 0, 0};
        send_tree(c, s.S->ltree, lcodes - 1);
        send_tree(c, s.S->dtree, dcodes - 1);
        compress_block(s, s.S->ltree, s.S->dtree);
    }
    DF_STAMP(s, 3);
    init_block(s);
    if (eof) bi_windup(s);
    s.block_start = s.strstart;
    flush_pending(s);
    DF_STAMP(s, 4);
}

// deflate.ts:690-766 fill_window (the whole input is available: one-shot append)
__device__ __forceinline__ void fill_window(DS& s) {
    do {
        int more = WINDOW_SIZE - s.lookahead - s.strstart;
        if (more == 0 && s.strstart == 0 && s.lookahead == 0) more = W_SIZE;
        else if (more == -1) more--;
        else if (s.strstart >= W_SIZE + W_SIZE - MIN_LOOKAHEAD) {
            GLB u32x4* w4 = (GLB u32x4*)s.S->window;
            for (int i = 0; i < W_SIZE / 16; i++) w4[i] = w4[i + W_SIZE / 16];
            s.match_start -= W_SIZE;
            s.strstart -= W_SIZE;
            s.block_start -= W_SIZE;
            for (int p = 0; p < HASH_SIZE; p++) { int m = s.S->head[p]; s.S->head[p] = (uint16_t)(m >= W_SIZE ? m - W_SIZE : 0); }
            for (int p = 0; p < W_SIZE; p++) { int m = s.S->prev[p]; s.S->prev[p] = (uint16_t)(m >= W_SIZE ? m - W_SIZE : 0); }
            more += W_SIZE;
        }
        uint64_t avail = s.in_len - s.in_pos;
        if (avail == 0) return;
        int n = avail > (uint64_t)more ? more : (int)avail;
        auto* dst = s.S->window + s.strstart + s.lookahead;
        for (int i = 0; i < n; i++) dst[i] = s.in[s.in_pos + i];
        s.in_pos += (uint64_t)n;
        s.lookahead += n;
        if (s.lookahead >= MIN_MATCH) {
            s.ins_h = s.S->window[s.strstart];
            s.ins_h = ((s.ins_h << HASH_SHIFT) ^ s.S->window[s.strstart + 1]) & HASH_MASK;
        }
    } while (s.lookahead < MIN_LOOKAHEAD && s.in_pos < s.in_len);
}

__device__ __forceinline__ uint32_t ld_u32(const GLB uint8_t* p) { uint32_t v; __builtin_memcpy(&v, p, 4); return v; }
__device__ __forceinline__ uint32_t ld_u16(const GLB uint8_t* p) { uint16_t v; __builtin_memcpy(&v, p, 2); return v; }

// deflate.ts:827-946 longest_match
__device__ __forceinline__ int longest_match(DS& s, int cur_match) {
    auto* win = s.S->window;
    auto* prev = s.S->prev;
    int chain_length = s.max_chain;
    int scan = s.strstart;
    int best_len = s.prev_length;
    int limit = s.strstart > MAX_DIST ? s.strstart - MAX_DIST : 0;
    int nice = s.nice_match;
    int strend = s.strstart + MAX_MATCH;
    int scan_end1 = win[scan + best_len - 1];
    int scan_end = win[scan + best_len];
    if (s.prev_length >= s.good_match) chain_length >>= 2;
    if (nice > s.lookahead) nice = s.lookahead;
    // scan bytes kept in registers; each candidate is loaded with unaligned dword reads and
    // its next chain link is fetched together with them (one dependent round trip per candidate)
    const uint32_t s0 = ld_u32(win + scan);                    // bytes scan .. scan+3
    int next = prev[cur_match & W_MASK];
    do {
        const int match = cur_match;
        const uint32_t m0 = ld_u32(win + match);
        const uint32_t be = ld_u16(win + match + best_len - 1);  // bytes best_len-1, best_len
        cur_match = next;
        next = prev[cur_match & W_MASK];                        // prefetch the link after this one
        if (be != ((uint32_t)scan_end1 | ((uint32_t)scan_end << 8)) || ((m0 ^ s0) & 0xffffu) != 0) continue;
        // compare 4 bytes at a time from offset 2 (deflate.ts:899-921): first differing byte
        int sp = scan + 2, mp = match + 2;
        do {
            const uint32_t x = ld_u32(win + sp) ^ ld_u32(win + mp);
            if (x) { const int mb = __builtin_ctz(x) >> 3; sp += mb; mp += mb; break; }
            sp += 4; mp += 4;
        } while (sp < strend);
        if (sp > strend) sp = strend;
        int len = MAX_MATCH - (strend - sp);
        if (len > best_len) {
            s.match_start = match;
            best_len = len;
            if (len >= nice) break;
            scan_end1 = win[scan + best_len - 1];
            scan_end = win[scan + best_len];
        }
    } while (cur_match > limit && --chain_length != 0);
    return best_len <= s.lookahead ? best_len : s.lookahead;
}

__device__ __forceinline__ int insert_string(DS& s) {
    s.ins_h = ((s.ins_h << HASH_SHIFT) ^ s.S->window[s.strstart + (MIN_MATCH - 1)]) & HASH_MASK;
    int hh = s.S->head[s.ins_h];
    s.S->prev[s.strstart & W_MASK] = (uint16_t)hh;
    s.S->head[s.ins_h] = (uint16_t)s.strstart;
    return hh;
}

// deflate.ts:953-1049 (levels 1-3).  One-shot (STREAM false): the whole input, to FINISH.
// STREAM: an append's chunk; without `finish` the loop stops where the reference's
// deflate(NO_FLUSH) returns NeedMore (lookahead < MIN_LOOKAHEAD after fill_window, deflate.ts
// 968-975), returning false.
template <bool STREAM>
__device__ __forceinline__ bool deflate_fast(DS& s, bool finish = true) {
    int hash_head = 0;
    for (;;) {
        if (s.lookahead < MIN_LOOKAHEAD) {
            fill_window(s);
            if (STREAM && s.lookahead < MIN_LOOKAHEAD && !finish) return false;
            if (s.lookahead == 0) break;
        }
        if (s.lookahead >= MIN_MATCH) hash_head = insert_string(s);
        if (hash_head != 0 && ((s.strstart - hash_head) & 0xffff) <= MAX_DIST)
            s.match_length = longest_match(s, hash_head);
        bool bflush;
        if (s.match_length >= MIN_MATCH) {
            bflush = tr_tally(s, s.strstart - s.match_start, s.match_length - MIN_MATCH);
            s.lookahead -= s.match_length;
            if (s.match_length <= s.max_lazy && s.lookahead >= MIN_MATCH) {
                s.match_length--;
                do { s.strstart++; hash_head = insert_string(s); } while (--s.match_length != 0);
                s.strstart++;
            } else {
                s.strstart += s.match_length;
                s.match_length = 0;
                s.ins_h = s.S->window[s.strstart];
                s.ins_h = ((s.ins_h << HASH_SHIFT) ^ s.S->window[s.strstart + 1]) & HASH_MASK;
            }
        } else {
            bflush = tr_tally(s, 0, s.S->window[s.strstart]);
            s.lookahead--;
            s.strstart++;
        }
        if (bflush) flush_block(s, false);
    }
    flush_block(s, true);
    return true;
}

// deflate.ts:1054-1182 (levels 4-9); STREAM and finish as deflate_fast
template <bool STREAM>
__device__ __forceinline__ bool deflate_slow(DS& s, bool finish = true) {
    int hash_head = 0;
    for (;;) {
        if (s.lookahead < MIN_LOOKAHEAD) {
            fill_window(s);
            if (STREAM && s.lookahead < MIN_LOOKAHEAD && !finish) return false;
            if (s.lookahead == 0) break;
        }
        if (s.lookahead >= MIN_MATCH) hash_head = insert_string(s);
        s.prev_length = s.match_length;
        int prev_match = s.match_start;
        s.match_length = MIN_MATCH - 1;
        if (hash_head != 0 && s.prev_length < s.max_lazy && ((s.strstart - hash_head) & 0xffff) <= MAX_DIST) {
            s.match_length = longest_match(s, hash_head);
            if (s.match_length <= 5 && s.match_length == MIN_MATCH && s.strstart - s.match_start > 4096)
                s.match_length = MIN_MATCH - 1;
        }
        if (s.prev_length >= MIN_MATCH && s.match_length <= s.prev_length) {
            int max_insert = s.strstart + s.lookahead - MIN_MATCH;
            bool bflush = tr_tally(s, s.strstart - 1 - prev_match, s.prev_length - MIN_MATCH);
            s.lookahead -= s.prev_length - 1;
            s.prev_length -= 2;
            do {
                if (++s.strstart <= max_insert) hash_head = insert_string(s);
            } while (--s.prev_length != 0);
            s.match_available = 0;
            s.match_length = MIN_MATCH - 1;
            s.strstart++;
            if (bflush) flush_block(s, false);
        } else if (s.match_available) {
            bool bflush = tr_tally(s, 0, s.S->window[s.strstart - 1]);
            if (bflush) flush_block(s, false);
            s.strstart++;
            s.lookahead--;
        } else {
            s.match_available = 1;
            s.strstart++;
            s.lookahead--;
        }
    }
    if (s.match_available) {
        tr_tally(s, 0, s.S->window[s.strstart - 1]);
        s.match_available = 0;
    }
    flush_block(s, true);
    return true;
}

// deflate.ts:1184-1216 deflateSetDictionary: the dictionary's last <= MAX_DIST bytes become
// the window's start, with their strings in the hash chains (shorter than MIN_MATCH: nothing)
__device__ void set_dictionary(DS& s, const GLB uint8_t* dict, uint32_t dict_len) {
    int length = (int)dict_len;
    if (length < MIN_MATCH) return;
    uint32_t index = 0;
    if (length > MAX_DIST) {
        length = MAX_DIST;
        index = dict_len - (uint32_t)length;
    }
    for (int i = 0; i < length; i++) s.S->window[i] = dict[index + i];
    s.strstart = length;
    s.block_start = length;
    s.ins_h = s.S->window[0];
    s.ins_h = ((s.ins_h << HASH_SHIFT) ^ s.S->window[1]) & HASH_MASK;
    for (int n = 0; n <= length - MIN_MATCH; n++) {
        s.ins_h = ((s.ins_h << HASH_SHIFT) ^ s.S->window[n + (MIN_MATCH - 1)]) & HASH_MASK;
        s.S->prev[n & W_MASK] = s.S->head[s.ins_h];
        s.S->head[s.ins_h] = (uint16_t)n;
    }
}

// adler32.ts:34-105 / crc32.ts:48-106 over the input (Deflater.append, sd-deflate.ts:185-190)
__device__ int32_t input_checksum(const GLB uint8_t* p, uint64_t n, bool gzip, const uint32_t* crct) {
    if (gzip) {
        uint32_t c = 0xffffffffu;
        for (uint64_t i = 0; i < n; i++) c = crct[(c ^ p[i]) & 255] ^ (c >> 8);
        return (int32_t)~c;
    }
    uint64_t a = 1, s2 = 0, len = n, off = 0;
    while (len >= 5552) {
        len -= 5552;
        for (int i = 0; i < 5552; i++) { a += p[off++]; s2 += a; }
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

__global__ __launch_bounds__(DF_THREADS) void k_deflate(DeflateArgs A) {
    __shared__ uint32_t crct[256];
    for (int n = threadIdx.x; n < 256; n += DF_THREADS) {
        uint32_t c = (uint32_t)n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
        crct[n] = c;
    }
    __syncthreads();
    uint32_t sid = blockIdx.x * DF_THREADS + threadIdx.x;
    if (sid >= A.n) return;

    DS s;
#ifdef SDZ_TIMING
    s.timed = A.dbg && (sid & 63) == 0 && sid < 64 * 16;
    for (int k = 0; k < 8; ++k) s.tacc[k] = 0;
    s.tlast = clock64();
#endif
    s.S = (GLB DSlab*)(A.state + (uint64_t)sid * SLAB_BYTES);
    s.T = (const GLB DTables*)&g_dt;
    s.in = (const GLB uint8_t*)(A.in + A.in_off[sid]);
    s.in_len = A.in_len[sid];
    s.in_pos = 0;
    s.out = (GLB uint8_t*)(A.out + A.out_off[sid]);
    s.out_cap = A.out_cap[sid];
    s.out_len = 0;
    s.err = 0;
    // after the record path (A.fast) only the streams it handed back run here
    if (A.fast && !((const GLB FStream*)s.S->window)->flag) return;
    sdz_deflate_record R;
    R.status = SDZ_OK; R.checksum = 0; R.out_len = 0; R.reserved = 0;
    if (s.in_len == 0) {                        // sd-deflate.ts:180-182 + 232-234
        R.status = SDZ_DATA_ERROR;
        A.rec[sid] = R;
        return;
    }
    // Deflate constructor (deflate.ts:196-220) + window zero fill (deflate.ts:119)
    {
        const u32x4 z = {0u, 0u, 0u, 0u};
        GLB u32x4* w4 = (GLB u32x4*)s.S->window;
        for (int i = 0; i < WINDOW_SIZE / 16; i++) w4[i] = z;
        GLB u32x4* h4 = (GLB u32x4*)s.S->head;
        for (int i = 0; i < HASH_SIZE * 2 / 16; i++) h4[i] = z;
        GLB u32x4* p4 = (GLB u32x4*)s.S->prev;
        for (int i = 0; i < W_SIZE * 2 / 16; i++) p4[i] = z;
    }
    {
        for (int i = 0; i < HEAP_SIZE * 2; i++) s.S->ltree[i] = 0;
        for (int i = 0; i < (2 * D_CODES + 1) * 2; i++) s.S->dtree[i] = 0;
        for (int i = 0; i < (2 * BL_CODES + 1) * 2; i++) s.S->bltree[i] = 0;
    }
    s.level = A.level;
    s.good_match = c_config[A.level][0];
    s.max_lazy = c_config[A.level][1];
    s.nice_match = c_config[A.level][2];
    s.max_chain = c_config[A.level][3];
    s.pending = 0;
    s.ins_h = 0; s.block_start = 0; s.match_length = MIN_MATCH - 1; s.match_available = 0;
    s.strstart = 0; s.match_start = 0; s.lookahead = 0; s.prev_length = MIN_MATCH - 1;
    s.bi_buf = 0; s.bi_valid = 0;
    s.heap_len = 0; s.heap_max = HEAP_SIZE;
    s.l_max_code = s.d_max_code = s.bl_max_code = 0;
    init_block(s);
    if (A.dict) set_dictionary(s, (const GLB uint8_t*)A.dict, A.dict_len);   // sd-deflate.ts:80-90

    bool gzip = A.format == SDZ_DEFLATE_GZIP;
    DF_STAMP(s, 5);
    int32_t cks = input_checksum(s.in, s.in_len, gzip, crct);
    DF_STAMP(s, 0);
    // container header (sd-deflate.ts:98-152): written straight to the output slot
    // zlib: 78 01, or 78 20 + DICTID when the dictionary's adler32 is nonzero (sd-deflate.ts:98-115)
    const bool dictid = A.format == SDZ_DEFLATE_ZLIB && A.dict && dict_id_of(A.dict_adler, A.dict_adler_dev) != 0;
    uint64_t hdr = A.format == SDZ_DEFLATE_ZLIB ? (dictid ? 6 : 2) : gzip ? 10 + (A.fname_len ? A.fname_len + 1 : 0) : 0;
    if (hdr > s.out_cap) { R.status = SDZ_OUT_OVERFLOW; A.rec[sid] = R; return; }
    if (dictid) {
        const uint32_t d = (uint32_t)dict_id_of(A.dict_adler, A.dict_adler_dev);
        s.out[0] = 0x78; s.out[1] = 0x20;
        s.out[2] = (uint8_t)(d >> 24); s.out[3] = (uint8_t)(d >> 16); s.out[4] = (uint8_t)(d >> 8); s.out[5] = (uint8_t)d;
    } else if (A.format == SDZ_DEFLATE_ZLIB) { s.out[0] = 0x78; s.out[1] = 0x01; }
    else if (gzip) {
        s.out[0] = 0x1f; s.out[1] = 0x8b; s.out[2] = 8; s.out[3] = A.fname_len ? 8 : 0;
        s.out[4] = (uint8_t)A.mtime; s.out[5] = (uint8_t)(A.mtime >> 8);
        s.out[6] = (uint8_t)(A.mtime >> 16); s.out[7] = (uint8_t)(A.mtime >> 24);
        s.out[8] = 0; s.out[9] = 0xff;
        for (uint32_t i = 0; i < A.fname_len; i++) s.out[10 + i] = A.fname[i];
        if (A.fname_len) s.out[10 + A.fname_len] = 0;
    }
    s.out_len = hdr;

    if (c_config[A.level][4]) deflate_fast<false>(s);
    else deflate_slow<false>(s);

    // trailer (sd-deflate.ts:154-165)
    uint64_t tl = A.format == SDZ_DEFLATE_ZLIB ? 4 : gzip ? 8 : 0;
    if (s.out_len + tl > s.out_cap) s.err |= 2;
    else if (A.format == SDZ_DEFLATE_ZLIB) {
        uint32_t c = (uint32_t)cks;
        s.out[s.out_len] = (uint8_t)(c >> 24); s.out[s.out_len + 1] = (uint8_t)(c >> 16);
        s.out[s.out_len + 2] = (uint8_t)(c >> 8); s.out[s.out_len + 3] = (uint8_t)c;
        s.out_len += 4;
    } else if (gzip) {
        uint32_t c = (uint32_t)cks, z = (uint32_t)s.in_len;
        for (int k = 0; k < 4; k++) s.out[s.out_len + k] = (uint8_t)(c >> (8 * k));
        for (int k = 0; k < 4; k++) s.out[s.out_len + 4 + k] = (uint8_t)(z >> (8 * k));
        s.out_len += 8;
    }
    R.status = (s.err & 2) ? SDZ_OUT_OVERFLOW : (s.err & 1) ? SDZ_DATA_ERROR : SDZ_OK;
    DF_STAMP(s, 5);
#ifdef SDZ_TIMING
    if (s.timed) for (int k = 0; k < 8; ++k) atomicAdd(&A.dbg[k], s.tacc[k]);
#endif
    R.checksum = cks;
    R.out_len = s.out_len;
    A.rec[sid] = R;
}

// ------------------------------------------------------------------ incremental Deflater

// adler32(chunk, seed) / crc32(chunk, seed) (adler32.ts:34-105 with the NMAX grid from the
// chunk's start, crc32.ts:48-106): the running checksum of Deflater.append
__device__ int32_t chunk_checksum(const GLB uint8_t* p, uint64_t n, bool gzip, const uint32_t* crct, int32_t seed) {
    if (gzip) {
        uint32_t c = ~(uint32_t)seed;
        for (uint64_t i = 0; i < n; i++) c = crct[(c ^ p[i]) & 255] ^ (c >> 8);
        return (int32_t)~c;
    }
    uint64_t a = (uint32_t)seed & 0xffffu, s2 = ((uint32_t)seed >> 16) & 0xffffu, len = n, off = 0;
    while (len >= 5552) {
        len -= 5552;
        for (int i = 0; i < 5552; i++) { a += p[off++]; s2 += a; }
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

__global__ void k_deflate_reset(uint8_t* state, uint32_t n) {
    const uint32_t sid = blockIdx.x * blockDim.x + threadIdx.x;
    if (sid < n) ((GLB DSlab*)(state + (uint64_t)sid * SLAB_BYTES))->sc.status = 0;
}

// One Deflater.append(chunk) (finish = 0) or finish() (finish = 1) per stream, the stream's
// whole state in its slab between calls (sd-deflate.ts:173-253 over deflate.ts:1218-1327 with
// NO_FLUSH / FINISH).  The output of a call is what the reference's append()/finish() returns,
// concatenated: the header on the first non-empty append, the blocks flushed during the call
// (flush_block_only -> flush_pending), and the trailer at finish.  A record's out_len is this
// call's output; its checksum the running one.  finish() before any append and an append after
// finish() report SDZ_DATA_ERROR (the reference throws, sd-deflate.ts:232-234, 211-214).
__global__ __launch_bounds__(DF_THREADS) void k_deflate_stream(DeflateArgs A, uint32_t finish) {
    __shared__ uint32_t crct[256];
    for (int n = threadIdx.x; n < 256; n += DF_THREADS) {
        uint32_t c = (uint32_t)n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
        crct[n] = c;
    }
    __syncthreads();
    const uint32_t sid = blockIdx.x * DF_THREADS + threadIdx.x;
    if (sid >= A.n) return;
    DS s;
#ifdef SDZ_TIMING
    s.timed = false;
#endif
    s.S = (GLB DSlab*)(A.state + (uint64_t)sid * SLAB_BYTES);
    s.T = (const GLB DTables*)&g_dt;
    s.in = (const GLB uint8_t*)(A.in + A.in_off[sid]);
    s.in_len = A.in_len[sid];
    s.in_pos = 0;
    s.out = (GLB uint8_t*)(A.out + A.out_off[sid]);
    s.out_cap = A.out_cap[sid];
    s.out_len = 0;
    s.err = 0;
    GLB DfScal& C = s.S->sc;
    const bool gzip = A.format == SDZ_DEFLATE_GZIP;
    sdz_deflate_record R;
    R.status = SDZ_OK; R.out_len = 0; R.reserved = 0;
    const int32_t st = C.status;
    R.checksum = st ? C.checksum : 0;
    if ((finish && st == 0) || (!finish && st == 2 && s.in_len)) {
        R.status = SDZ_DATA_ERROR;
        A.rec[sid] = R;
        return;
    }
    if (!finish && s.in_len == 0) { A.rec[sid] = R; return; }   // sd-deflate.ts:180-182: nothing
    s.level = A.level;
    s.good_match = c_config[A.level][0];
    s.max_lazy = c_config[A.level][1];
    s.nice_match = c_config[A.level][2];
    s.max_chain = c_config[A.level][3];
    s.heap_len = 0; s.heap_max = HEAP_SIZE;
    s.l_max_code = s.d_max_code = s.bl_max_code = 0;
    if (st == 0) {
        // Deflate constructor (deflate.ts:196-220) + deflateSetDictionary, as k_deflate
        const u32x4 z = {0u, 0u, 0u, 0u};
        GLB u32x4* w4 = (GLB u32x4*)s.S->window;
        for (int i = 0; i < WINDOW_SIZE / 16; i++) w4[i] = z;
        GLB u32x4* h4 = (GLB u32x4*)s.S->head;
        for (int i = 0; i < HASH_SIZE * 2 / 16; i++) h4[i] = z;
        GLB u32x4* p4 = (GLB u32x4*)s.S->prev;
        for (int i = 0; i < W_SIZE * 2 / 16; i++) p4[i] = z;
        for (int i = 0; i < HEAP_SIZE * 2; i++) s.S->ltree[i] = 0;
        for (int i = 0; i < (2 * D_CODES + 1) * 2; i++) s.S->dtree[i] = 0;
        for (int i = 0; i < (2 * BL_CODES + 1) * 2; i++) s.S->bltree[i] = 0;
        s.pending = 0;
        s.ins_h = 0; s.block_start = 0; s.match_length = MIN_MATCH - 1; s.match_available = 0;
        s.strstart = 0; s.match_start = 0; s.lookahead = 0; s.prev_length = MIN_MATCH - 1;
        s.bi_buf = 0; s.bi_valid = 0;
        init_block(s);
        if (A.dict) set_dictionary(s, (const GLB uint8_t*)A.dict, A.dict_len);
        C.checksum = gzip ? 0 : 1;
        C.orig = 0;
        // container header (sd-deflate.ts:98-152), on the first append
        const bool dictid = A.format == SDZ_DEFLATE_ZLIB && A.dict && dict_id_of(A.dict_adler, A.dict_adler_dev) != 0;
        const uint64_t hdr = A.format == SDZ_DEFLATE_ZLIB ? (dictid ? 6 : 2)
                           : gzip ? 10 + (A.fname_len ? A.fname_len + 1 : 0) : 0;
        if (hdr > s.out_cap) { R.status = SDZ_OUT_OVERFLOW; A.rec[sid] = R; return; }
        if (dictid) {
            const uint32_t d = (uint32_t)dict_id_of(A.dict_adler, A.dict_adler_dev);
            s.out[0] = 0x78; s.out[1] = 0x20;
            s.out[2] = (uint8_t)(d >> 24); s.out[3] = (uint8_t)(d >> 16); s.out[4] = (uint8_t)(d >> 8); s.out[5] = (uint8_t)d;
        } else if (A.format == SDZ_DEFLATE_ZLIB) { s.out[0] = 0x78; s.out[1] = 0x01; }
        else if (gzip) {
            s.out[0] = 0x1f; s.out[1] = 0x8b; s.out[2] = 8; s.out[3] = A.fname_len ? 8 : 0;
            s.out[4] = (uint8_t)A.mtime; s.out[5] = (uint8_t)(A.mtime >> 8);
            s.out[6] = (uint8_t)(A.mtime >> 16); s.out[7] = (uint8_t)(A.mtime >> 24);
            s.out[8] = 0; s.out[9] = 0xff;
            for (uint32_t i = 0; i < A.fname_len; i++) s.out[10 + i] = A.fname[i];
            if (A.fname_len) s.out[10 + A.fname_len] = 0;
        }
        s.out_len = hdr;
    } else {
        s.pending = C.pending; s.ins_h = C.ins_h; s.block_start = C.block_start; s.match_length = C.match_length;
        s.match_available = C.match_available; s.strstart = C.strstart; s.match_start = C.match_start;
        s.lookahead = C.lookahead; s.prev_length = C.prev_length; s.last_lit = C.last_lit; s.matches = C.matches;
        s.opt_len = C.opt_len; s.static_len = C.static_len; s.bi_buf = C.bi_buf; s.bi_valid = C.bi_valid;
    }
    if (s.in_len) {
        C.checksum = chunk_checksum(s.in, s.in_len, gzip, crct, C.checksum);
        C.orig += (uint32_t)s.in_len;
    }
    // deflate.ts:1290: a call runs the compressor when there is input, lookahead, or a first
    // FINISH; a repeated finish() only adds the trailer again (as the reference does)
    if (st != 2) {
        if (c_config[A.level][4]) deflate_fast<true>(s, finish != 0);
        else deflate_slow<true>(s, finish != 0);
    }
    if (finish) {
        const uint64_t tl = A.format == SDZ_DEFLATE_ZLIB ? 4 : gzip ? 8 : 0;
        const uint32_t c = (uint32_t)C.checksum, z = C.orig;
        if (s.out_len + tl > s.out_cap) s.err |= 2;
        else if (A.format == SDZ_DEFLATE_ZLIB) {
            s.out[s.out_len] = (uint8_t)(c >> 24); s.out[s.out_len + 1] = (uint8_t)(c >> 16);
            s.out[s.out_len + 2] = (uint8_t)(c >> 8); s.out[s.out_len + 3] = (uint8_t)c;
            s.out_len += 4;
        } else if (gzip) {
            for (int k = 0; k < 4; k++) s.out[s.out_len + k] = (uint8_t)(c >> (8 * k));
            for (int k = 0; k < 4; k++) s.out[s.out_len + 4 + k] = (uint8_t)(z >> (8 * k));
            s.out_len += 8;
        }
    }
    C.status = finish ? 2 : 1;
    C.pending = s.pending; C.ins_h = s.ins_h; C.block_start = s.block_start; C.match_length = s.match_length;
    C.match_available = s.match_available; C.strstart = s.strstart; C.match_start = s.match_start;
    C.lookahead = s.lookahead; C.prev_length = s.prev_length; C.last_lit = s.last_lit; C.matches = s.matches;
    C.opt_len = s.opt_len; C.static_len = s.static_len; C.bi_buf = s.bi_buf; C.bi_valid = s.bi_valid;
    R.status = (s.err & 2) ? SDZ_OUT_OVERFLOW : (s.err & 1) ? SDZ_DATA_ERROR : SDZ_OK;
    R.checksum = C.checksum;
    R.out_len = s.out_len;
    A.rec[sid] = R;
}

void launch_deflate_reset(uint8_t* state, uint32_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_deflate_reset, dim3((n + 255) / 256), dim3(256), 0, s, state, n);
}
void launch_deflate_stream(const DeflateArgs& a, uint32_t finish, hipStream_t s) {
    if (!a.n) return;
    dt_ready(s);
    hipLaunchKernelGGL(k_deflate_stream, dim3((a.n + DF_THREADS - 1) / DF_THREADS), dim3(DF_THREADS), 0, s, a, finish);
}

// ------------------------------------------------------------------ record path kernels

// k_dfl_chain: one wave per chain unit walks its positions in order, 1024 at a time: each lane
// hashes 16 consecutive positions from registers (the next chunk's bytes are already in
// flight) into LDS, then 16 rounds of 64 positions swap themselves into the LDS head table.
// Same-address lanes of one ds_wrxchg are served in lane order (tools/ubench/
// lds_xchg_order.hip), so a lane receives the position of the previous lane with the same
// hash, or the head: exactly insert_string's sequence (deflate_slow inserts every position
// with lookahead >= MIN_MATCH, deflate.ts:1079-1085, 1124-1131).
// Units: unit 0 of a stream covers positions [0, 64 Ki); unit j >= 1 covers
// [64 Ki + (j - 1) 32 Ki, + 32 Ki) after hashing the 32 Ki before it (history: heads only), so
// every unit's positions fit 16 bits relative to its history start h0 (0 = none: position h0
// itself is never within MAX_DIST of a unit position, and position 0 is never matched, as
// the reference's hash_head == 0 test, deflate.ts:1092).  The link stored for position P is
// the distance to the previous same-hash position, 0 if none or farther than 32767 (beyond
// MAX_DIST: every walk stops there, as the reference's does at `limit`, deflate.ts:941).
#define CH_CHUNK 1024
#define CH_UNIT 32768
uint32_t deflate_chain_units(uint64_t len) {
    return len <= 65536 ? 1u : 1u + (uint32_t)((len - 65536 + CH_UNIT - 1) / CH_UNIT);
}
__device__ __forceinline__ void ch_load(const GLB uint8_t* in, uint32_t n, uint32_t at, uint32_t (&w)[5]) {
    if (at + 20 <= n) {
        for (int i = 0; i < 5; ++i) __builtin_memcpy(&w[i], (const uint8_t*)(in + at + 4 * i), 4);
    } else {
        for (int i = 0; i < 5; ++i) {
            uint32_t v = 0;
            for (int b = 0; b < 4; ++b) {
                const uint32_t q = at + 4 * i + b;
                v |= (q < n ? (uint32_t)in[q] : 0u) << (8 * b);
            }
            w[i] = v;
        }
    }
}
// Two units share one block and one head table: wave w keeps its heads in half w of each
// dword and swaps them in with ds_mskor_rtn_b32, a masked exchange that, like ds_wrxchg,
// serves same-address lanes in lane order.  That is two waves per CU where one unit's
// 128 KiB table allowed one.  Each wave only syncs with itself.
#define CH_WAVES 2
__device__ __forceinline__ uint32_t lds_mskor_rtn(uint32_t* p, uint32_t mask, uint32_t v) {
    uint32_t r;
    const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)p;
    asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(mask), "v"(v) : "memory");
    return r;
}
__global__ __launch_bounds__(64 * CH_WAVES) void k_dfl_chain(DeflateArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t head[HASH_SIZE];   // 128 KiB, a 16-bit half per wave
    __shared__ uint16_t hsw[CH_WAVES][CH_CHUNK];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t u = blockIdx.x * CH_WAVES + wv;
    for (uint32_t i = threadIdx.x; i < HASH_SIZE / 4; i += 64 * CH_WAVES) ((uint4*)head)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    if (u >= A.ncunit) return;
    const uint32_t k = A.cunit[u] >> kRecUnitShift, j = A.cunit[u] & ((1u << kRecUnitShift) - 1);
    const uint64_t in_len = A.in_len[k];
    const uint64_t rp = A.rp0[k];
    if (rp == ~0ull) return;
    const GLB uint8_t* in = (const GLB uint8_t*)(A.in + A.in_off[k]);
    GLB uint16_t* pv = (GLB uint16_t*)A.pv_buf + rp;
    uint16_t* hs = hsw[wv];
    const uint32_t sh = 16u * wv, msk = 0xffffu << sh;
    const uint32_t n = (uint32_t)in_len;
    const uint32_t a = j == 0 ? 0u : 65536u + (j - 1) * CH_UNIT;
    const uint32_t e = j == 0 ? (n < 65536u ? n : 65536u) : (n - a < CH_UNIT ? n : a + CH_UNIT);
    const uint32_t h0 = j == 0 ? 0u : a - 32768u;
    uint32_t w[5];
    ch_load(in, n, h0 + 16 * lane, w);
    for (uint32_t base = h0; base < e; base += CH_CHUNK) {
        uint32_t wn[5];
        if (base + CH_CHUNK < e) ch_load(in, n, base + CH_CHUNK + 16 * lane, wn);
        for (int q = 0; q < 16; q += 2) {                // hashes of positions base + 16 lane + q
            uint32_t h2 = 0;
            for (int r = 0; r < 2; ++r) {
                const int o = q + r;
                const uint32_t b0 = (w[o >> 2] >> (8 * (o & 3))) & 255u;
                const uint32_t b1 = (w[(o + 1) >> 2] >> (8 * ((o + 1) & 3))) & 255u;
                const uint32_t b2 = (w[(o + 2) >> 2] >> (8 * ((o + 2) & 3))) & 255u;
                h2 |= (((b0 << 10) ^ (b1 << 5) ^ b2) & HASH_MASK) << (16 * r);
            }
            *(uint32_t*)&hs[16 * lane + q] = h2;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // all hash reads, then the 16 exchanges back to back (one wave's LDS operations run in
        // order, so position order holds), then the stores: a few LDS round trips per chunk
        uint32_t hv[CH_CHUNK / 64], old[CH_CHUNK / 64];
#pragma unroll
        for (uint32_t t = 0; t < CH_CHUNK / 64; ++t) hv[t] = hs[64 * t + lane];
#pragma unroll
        for (uint32_t t = 0; t < CH_CHUNK / 64; ++t) {
            const uint32_t p = base + 64 * t + lane;
            old[t] = 0;
            // insert_string runs while lookahead >= 3
            if (p < e && p + 2 < n) old[t] = lds_mskor_rtn(&head[hv[t]], msk, (p - h0) << sh);
        }
#pragma unroll
        for (uint32_t t = 0; t < CH_CHUNK / 64; ++t) {
            const uint32_t p = base + 64 * t + lane;
            if (p >= a && p < e) {
                const uint32_t q = (old[t] >> sh) & 0xffffu;          // relative to h0; 0 = none
                const uint32_t d = q ? p - (q + h0) : 0u;
                pv[p] = (uint16_t)(d <= 32767u ? d : 0u);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int i = 0; i < 5; ++i) w[i] = wn[i];
    }
}

// k_dfl_match: what longest_match returns at every position (but the last PM_TAIL), for both
// chain lengths.  A workgroup takes PM_SEG positions of one stream with the 32 KiB before
// them staged in LDS: window bytes and chain links.  Each wave works through its share of
// positions with persistent lanes: a lane whose chain walk ends takes the next position,
// so the wave runs ~ (total candidates / 64) steps, not (longest chain x positions / 64).
// Record per position: bits 0-15 distance, 16-24 length (<= 2: no candidate beats
// MIN_MATCH - 1) -- chain max_chain in the low word, max_chain >> 2 in the high word.
// With seg_merge the host lists a stream's segment 0 for segments 0-2 (no history before them:
// the same 48 KiB of window and links is staged), first in the list -- workgroups go to the XCDs
// round-robin in list order, so the long ones are spread over all 8 and start first.
#define PM_SEG 16384
#define PM_THREADS 1024
#ifndef PM_CHUNK
#define PM_CHUNK 128                                    // positions a wave takes at a time
#endif
#ifndef PM_REFILL
#define PM_REFILL 12                                    // idle lanes that trigger a refill (8: 1 % slower)
#endif
#ifndef PM_LAZYW4
#define PM_LAZYW4 0                                     // measured slower: C3 543 -> 576 ms
#endif
#ifndef PM_MORE_IF
#define PM_MORE_IF 1                                    // long compares behind one uniform test
#endif
#ifndef PM_COUNT
#define PM_COUNT 0                                      // development: long-compare counters in A.dbg[16..19]
#endif
#ifndef PM_WBSKIP
#define PM_WBSKIP 0                                     // the byte-at-best filter only where best >= 4
#endif
#ifndef PM_W8
#define PM_W8 (!PM_LAZYW4 && !PM_WBSKIP)                // first compare over 8 bytes (default form only)
#endif
#ifndef PM_ISSUE
#define PM_ISSUE 1                                      // every read of a step issued before the first use
#endif
#ifndef PM_UNIFORM
#define PM_UNIFORM 1                                    // the wave's queue head in SGPRs (uniform loop exit)
#endif
#ifndef PM_SBREG
#define PM_SBREG 0                                      // the position's byte at best in a register (measured slower: C3 312.3 -> 323.2 ms)
#endif
#ifndef PM_SELFILL
#define PM_SELFILL 0                                    // refill without a divergent region (measured slower: C3 309.4 -> 312.7 ms)
#endif
#ifndef PM_WBLATE
#define PM_WBLATE 0                                     // the filter read after the 8-byte compare (measured slower: C3 344.5 -> 353.4 ms)
#endif
#define PM_WINB (W_SIZE + PM_SEG + PM_TAIL + MAX_MATCH + 16)   // staged window bytes (+ the last positions'
#define PM_PV (W_SIZE + PM_SEG + PM_TAIL)                         // staged links      ... in a last segment)
// Match records: one u32 per position p, at u32 index rp0 + p of the record buffer (8 bytes per
// position are allocated): the full-chain result -- distance in bits 0-14 (0: no match), length - 3
// in bits 15-22 --, bit 23 set when the quarter-chain result (deflate.ts:836-838, prev_length >=
// good_match) differs, and input byte p - 1 (the literal the parse emits from there) in bits
// 24-31.  A differing quarter result is the u32 at qoff + rp0 + p (same low 23 bits; qoff: the
// batch's positions, or a Deflater's record capacity).  The parse reads one word per step, and the
// quarter word only on the steps that use it and where it differs (4 bytes per position each way
// instead of 8).  The symbols later go to u32 rp0 + k, over records already read.
__device__ __forceinline__ uint32_t rc_res(uint32_t len, uint32_t dist) {    // a search's result (len >= 3)
    return dist | ((len - MIN_MATCH) << 15);
}
__device__ __forceinline__ uint32_t rc_len(uint32_t e) { return (e & 0x7fffu) ? ((e >> 15) & 255u) + MIN_MATCH : 0u; }
__device__ __forceinline__ uint32_t rc_word(uint32_t full, uint32_t quarter, uint32_t lb) {
    return full | (quarter != full ? 1u << 23 : 0u) | (lb << 24);
}
// (len << 16 | dist, 0: none -- the search functions' form) as a result word
__device__ __forceinline__ uint32_t rc_from16(uint32_t w) { return (w >> 16) >= MIN_MATCH ? rc_res(w >> 16, w & 0xffffu) : 0u; }
__device__ __forceinline__ uint32_t pm_w4(const uint8_t* w, uint32_t x) {   // 4 bytes at x, aligned reads
    const uint32_t* w32 = (const uint32_t*)w;
    return __builtin_amdgcn_alignbyte(w32[(x >> 2) + 1], w32[x >> 2], x & 3u);
}
// 8 bytes at x as two words (lo: bytes x..x+3, hi: x+4..x+7) from three aligned dword reads
__device__ __forceinline__ void pm_w8(const uint8_t* w, uint32_t x, uint32_t& lo, uint32_t& hi) {
    const uint32_t* w32 = (const uint32_t*)w + (x >> 2);
    const uint32_t d0 = w32[0], d1 = w32[1], d2 = w32[2];
    lo = __builtin_amdgcn_alignbyte(d1, d0, x & 3u);
    hi = __builtin_amdgcn_alignbyte(d2, d1, x & 3u);
}
uint32_t deflate_match_segs(uint64_t len, uint32_t seg) {
    const uint64_t tail = len > PM_TAIL ? len - PM_TAIL : 0;
    return (uint32_t)((tail + seg - 1) / seg);
}
__device__ uint32_t win_byte(const GLB uint8_t* in, int64_t n, int64_t off, int64_t i);
__device__ __forceinline__ int64_t slide_off(int64_t n, int64_t P);
// The last PM_TAIL positions of a stream search the window the reference has there (stale bytes
// past the input, tail_search below); a slide can fall among them, so they form one or two groups
// of one window offset each.  k_dfl_match searches the larger group [mlo, mhi) (offset offM) in
// its last segment's LDS window, with that group's bytes past the input staged after it;
// k_dfl_tail the other.
struct TailGroups {
    int64_t mlo, mhi, offM;
};
__device__ __forceinline__ TailGroups tail_groups(int64_t n, int64_t tail) {
    const int64_t offA = slide_off(n, tail), offB = slide_off(n, n - 1);
    int64_t ps = n;                                       // first position with offB
    if (offA != offB) {
        int64_t lo = tail + 1, hi = n - 1;                // slide_off grows with P
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (slide_off(n, mid) == offB) hi = mid; else lo = mid + 1;
        }
        ps = lo;
    }
    TailGroups t;
    if (n - ps >= ps - tail) { t.mlo = ps == n ? tail : ps; t.mhi = n; t.offM = offB; }
    else { t.mlo = tail; t.mhi = ps; t.offM = offA; }
    return t;
}
#ifndef PM_LDS0
#define PM_LDS0 1                                       // window bytes at LDS address 0
#endif
__global__ __launch_bounds__(PM_THREADS) void k_dfl_match(DeflateArgs A) {
#if PM_LDS0
    // one LDS object: the window at address 0 and the links right after it, so every window
    // address is the index itself and every link address folds its base into the instruction's
    // 16-bit offset (separate arrays put the larger link array first, the window at 96.5 KiB)
    __shared__ __attribute__((aligned(16))) struct { uint8_t win[(PM_WINB + 15) & ~15]; uint16_t pvl[PM_PV]; } pm_lds;
    uint8_t* const win = pm_lds.win;
    uint16_t* const pvl = pm_lds.pvl;
#else
    __shared__ __attribute__((aligned(16))) uint8_t win[(PM_WINB + 15) & ~15];
    __shared__ __attribute__((aligned(16))) uint16_t pvl[PM_PV];
#endif
    __shared__ int pm_next;                                 // first position not yet handed to a wave
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u, wv = tid >> 6;
    if (blockIdx.x >= A.nmseg) return;
    const uint32_t sid = A.mseg[blockIdx.x] >> kRecUnitShift, seg = A.mseg[blockIdx.x] & ((1u << kRecUnitShift) - 1);
    const uint64_t in_len = A.in_len[sid];
    const uint64_t rp = A.rp0[sid];
    if (rp == ~0ull) return;
    const int n = (int)in_len;
    const int tail = n > PM_TAIL ? n - PM_TAIL : 0;
    // (segments of pm_seg <= PM_SEG positions: few streams spread over more workgroups; the LDS
    // window is sized for PM_SEG, and every segment stages its own 32 KiB of history)
    const int pseg = A.pm_seg ? (int)A.pm_seg : PM_SEG;
    const int s0 = (int)seg * pseg, e0 = s0 + (A.seg_merge && seg == 0 ? 3 * pseg : pseg);
    // the stream's last segment also takes the last positions (A.tail_in_match): all of them are
    // handed out, the larger window-offset group [mlo, mhi) is searched, the rest are left to
    // k_dfl_tail (which runs after and overwrites their records)
    const bool tl = A.tail_in_match && e0 >= tail && tail < n;
    const int s1 = tl ? n : e0 < tail ? e0 : tail;
    if (s0 >= s1) return;
    const int ws = s0 > W_SIZE ? s0 - W_SIZE : 0;          // staged range [ws, we) (ws even)
    const int we = s1 + MAX_MATCH + 8 < n ? s1 + MAX_MATCH + 8 : n;
    const GLB uint8_t* in = (const GLB uint8_t*)(A.in + A.in_off[sid]);
    const GLB uint16_t* pv = (const GLB uint16_t*)A.pv_buf + rp;
    TailGroups tg = { n, n, 0 };
    if (tl) tg = tail_groups(n, tail);
    {
        const int nw = (we - ws) >> 2;                     // whole dwords (unaligned global reads)
        uint32_t* w32 = (uint32_t*)win;
        for (int i = (int)tid; i < nw; i += PM_THREADS) {
            uint32_t v;
            __builtin_memcpy(&v, (const uint8_t*)(in + ws + 4 * i), 4);
            w32[i] = v;
        }
        for (int i = 4 * nw + (int)tid; i < we - ws; i += PM_THREADS) win[i] = in[ws + i];
        // past the input: the bytes the larger group's window holds there (tail_search's wb)
        if (tl)
            for (int j = (int)tid; j < MAX_MATCH + 16; j += PM_THREADS)
                win[n - ws + j] = (uint8_t)win_byte(in, n, tg.offM, (int64_t)n + j - tg.offM);
        const int np = (s1 - ws) >> 1;                     // link pairs (ws even, rp a multiple of 64)
        uint32_t* p32 = (uint32_t*)pvl;
        // links (distances) are staged as the previous position relative to ws (0 for none,
        // or at or below ws: below every walk's limit, and never a searchable head), so the
        // walk indexes LDS with them directly
        for (int i = (int)tid; i < np; i += PM_THREADS) {
            const uint32_t v = *(const GLB uint32_t*)(pv + ws + 2 * i);
            const uint32_t lo = v & 0xffffu, hi = v >> 16;   // staged positions 2 i and 2 i + 1
            const uint32_t r0 = 2u * (uint32_t)i, r1 = r0 + 1u;
            p32[i] = (lo && lo < r0 ? r0 - lo : 0u) | ((hi && hi < r1 ? r1 - hi : 0u) << 16);
        }
        for (int i = 2 * np + (int)tid; i < s1 - ws; i += PM_THREADS) {
            const uint32_t v = pv[ws + i];
            pvl[i] = (uint16_t)(v && v < (uint32_t)i ? (uint32_t)i - v : 0u);
        }
        if (tid == 0) pm_next = s0 + (PM_THREADS / 64) * PM_CHUNK;
    }
    __syncthreads();
    GLB uint32_t* rec = (GLB uint32_t*)A.rec_buf + rp;
    GLB uint32_t* qrec = (GLB uint32_t*)A.rec_buf + A.qoff + rp;   // the differing quarter results
    const int max_chain = c_config[A.level][3], qchain = max_chain >> 2, nice0 = c_config[A.level][2];
    int nice = nice0;                                       // (a last position: at most its lookahead)
    // Positions in chunks of PM_CHUNK: each wave starts on its own chunk and takes the next
    // free one from an LDS counter when it has handed out its last position, so waves whose
    // positions have long chains do not hold up the workgroup.
    // (the wave's queue head and end held wave-uniform -- SGPRs -- so that the loop's exit is a
    // uniform branch: no per-lane exit masks and copies of the loop state at every step)
#if PM_UNIFORM
    const int c0 = s0 + (int)__builtin_amdgcn_readfirstlane(wv) * PM_CHUNK;
#else
    const int c0 = s0 + (int)wv * PM_CHUNK;
#endif
    int next = c0 < s1 ? c0 : s1;                           // wave-uniform queue head
    int q1 = c0 + PM_CHUNK < s1 ? c0 + PM_CHUNK : s1;
    // A lane walks while chain > 0 (chain counts the candidates left); a finished lane keeps
    // its results (pend) until the next refill stores them.  The quarter walk ends at the
    // step where chain == cq, i.e. after qchain candidates.
    bool pend = false;
    const int cq = max_chain - qchain + 1;
    // cur: this step's candidate; nxt: the link after it (read a step ahead, so the chain
    // link of a step does not wait on the previous one).  cur, nxt, bpos, qpos, limit and sp
    // (the position itself) are relative to ws; p is absolute.
    int p = s0, sp = 0, cur = 0, nxt = 0, best = 0, bpos = 0, qbest = 0, qpos = 0, chain = 0, limit = 0;
    uint32_t s4 = 0, s4b = 0, sbv = 0;
    (void)s4b;
    (void)sbv;
    unsigned long long n_live = 0, n_step = 0, n_fill = 0;   // SDZ_PHASE_TIMING counters (PM_COUNT builds)
    (void)n_live; (void)n_step; (void)n_fill;
#if PM_COUNT
    unsigned long long n_it = 0, n_itl = 0, n_lst = 0, n_upd = 0;   // long-compare iterations, their lanes, steps with one
#endif
    for (;;) {
        // Idle lanes store their records and take the next positions once PM_REFILL lanes
        // are idle (or all are): the refill and the record store then run once per several
        // steps rather than at nearly every step (some lane ends its walk at most steps).
        const uint64_t im = __ballot(chain <= 0);
        const int nidle = __popcll(im);
        if (nidle >= PM_REFILL || nidle == 64) {
            if (pend) {
                if (qbest < 0) { qbest = best; qpos = bpos; }
                const uint32_t full = best > MIN_MATCH - 1 ? rc_res((uint32_t)best, (uint32_t)(sp - bpos)) : 0u;
                const uint32_t quarter = qbest > MIN_MATCH - 1 ? rc_res((uint32_t)qbest, (uint32_t)(sp - qpos)) : 0u;
                rec[p] = rc_word(full, quarter, win[p > 0 ? sp - 1 : 0]);
                if (quarter != full) qrec[p] = quarter;
                pend = false;
            }
            if (next >= q1) {                               // chunk handed out: take another
                const int b = __builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(&pm_next, PM_CHUNK) : 0);
                if (b < s1) {
                    next = b;
                    q1 = b + PM_CHUNK < s1 ? b + PM_CHUNK : s1;
                }
            }
            if (next >= q1 && nidle == 64) break;
#if PM_COUNT
            ++n_fill;
#endif
            if (next < q1) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(im >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)im, 0u));
                const int pn = next + (int)rank;
                next += nidle;
#if PM_SELFILL && PM_W8 && !PM_LAZYW4 && !PM_SBREG
                // every lane reads (a lane that takes no position reads at its own position) and
                // the taken lanes' new state is selected in place: no divergent region, so the
                // walk state keeps its registers and the steps without a refill copy nothing
                const bool take = chain <= 0 && pn < q1;
                const int spn = take ? pn - ws : sp;
                const int h = pvl[spn];                         // hash_head
                const uint32_t w0 = pm_w4(win, (uint32_t)spn), w1 = pm_w4(win, (uint32_t)spn + 4u);
                const bool last = pn >= tail;                   // a last position (tl only): searched
                // if in the larger group and lookahead >= MIN_MATCH; window index 0 (position offM)
                // is NIL there; nice_match at most the lookahead
                const bool search = h != 0 && spn - h <= MAX_DIST &&   // deflate.ts:1092
                                    (!last || (pn <= n - MIN_MATCH && pn >= tg.mlo && pn < tg.mhi &&
                                               (int64_t)(h + ws) > tg.offM));
                const int nx = pvl[search ? h : spn];
                p = take ? pn : p;
                sp = spn;
                cur = take ? h : cur;
                best = take ? MIN_MATCH - 1 : best;
                bpos = take ? 0 : bpos;
                qbest = take ? -1 : qbest;
                limit = take ? (pn > MAX_DIST ? pn - MAX_DIST : 0) - ws : limit;   // >= 0
                s4 = take ? w0 : s4;
                s4b = take ? w1 : s4b;
                nice = take ? (last && n - pn < nice0 ? n - pn : nice0) : nice;
                chain = take ? (search ? max_chain : 0) : chain;
                pend = take ? !search : pend;                   // no search: record 0
                nxt = take ? nx : nxt;
#else
                if (chain <= 0 && pn < q1) {
                    p = pn;
                    sp = p - ws;
                    cur = pvl[sp];                              // hash_head
                    best = MIN_MATCH - 1; bpos = 0; qbest = -1;
#if PM_LAZYW4
                    sbv = win[sp + best];
#endif
                    limit = (p > MAX_DIST ? p - MAX_DIST : 0) - ws;   // >= 0
                    s4 = pm_w4(win, (uint32_t)sp);
#if PM_W8
                    s4b = pm_w4(win, (uint32_t)sp + 4u);
#endif
#if PM_SBREG
                    sbv = (s4 >> 16) & 255u;                    // the position's byte at best = 2
#endif

                    bool search = cur != 0 && sp - cur <= MAX_DIST;  // deflate.ts:1092
                    if (p >= tail) {                                  // a last position (tl only)
                        // searched if in the larger group and lookahead >= MIN_MATCH; window index
                        // 0 (position offM) is NIL there; nice_match at most the lookahead
                        search = search && p <= n - MIN_MATCH && p >= tg.mlo && p < tg.mhi &&
                                 (int64_t)(cur + ws) > tg.offM;
                        nice = n - p < nice0 ? n - p : nice0;
                    } else {
                        nice = nice0;
                    }
                    chain = search ? max_chain : 0;
                    pend = !search;                             // no search: record 0
                    nxt = pvl[search ? cur : sp];
                }
#endif
            }
        }
        // two candidates per walking lane and step: cur (c1) and nxt (c2).  Both pass the
        // reference's pre-check against the step's starting best: a candidate that beats the
        // best after c1 also beats that, so the check only filters (deflate.ts:866-882), and
        // a candidate that passes gets its exact length.  The links after c2 (c3, then c4)
        // are read in turn, so the next step starts with two candidates again.
        const bool live = chain > 0;
#if PM_COUNT
        if (A.dbg) { ++n_step; n_live += __popcll(__ballot(live)); }
#endif
        const bool go1 = nxt > limit && chain > 1;           // the walk continues after c1
        const bool l2 = live && go1;                          // c2 is walked (unless nice at c1)
        const uint32_t c1 = (uint32_t)(live ? cur : sp), c2 = (uint32_t)(l2 ? nxt : sp);
        const int c3 = pvl[c2];
#if PM_LAZYW4
        // the 4-byte head compare only for candidates that pass the byte at best: once best
        // has grown most candidates fail there, and the skipped loads are random window reads
        // (LDS bank conflicts).  The byte of the position at best is kept in a register.
        const uint32_t sb = sbv, wb1 = win[c1 + best], wb2 = win[c2 + best];
        const bool go2 = c3 > limit && chain > 2;            // ... and after c2
        const int c4 = pvl[l2 && go2 ? c3 : sp];
        const bool cand1 = live && wb1 == sb, cand2 = l2 && wb2 == sb;
        uint32_t x1 = 0, x2 = 0;
        if (cand1) x1 = pm_w4(win, c1) ^ s4;
        if (cand2) x2 = pm_w4(win, c2) ^ s4;
#elif PM_WBSKIP
        // the byte at best only filters (a candidate that differs there cannot beat best); while
        // best < 4 the 4-byte compare decides that exactly, so only lanes with best >= 4 read it
        // (fewer lanes in the random LDS reads, fewer bank conflicts)
        uint32_t x1 = pm_w4(win, c1) ^ s4, x2 = pm_w4(win, c2) ^ s4;
        const bool go2 = c3 > limit && chain > 2;            // ... and after c2
        const int c4 = pvl[l2 && go2 ? c3 : sp];
        bool f1 = true, f2 = true;
        if (best >= 4) {
            const uint32_t sb = win[sp + best];
            f1 = win[c1 + best] == sb;
            f2 = win[c2 + best] == sb;
        }
        const bool cand1 = live && f1, cand2 = l2 && f2;
#elif PM_W8 && PM_WBLATE
        // The byte-at-best filter only decides which candidates enter the long compare: a
        // candidate that beats best agrees at best anyway.  While best < 8 the 8-byte compare
        // decides that exactly too, so the filter bytes are read only for lanes with best >= 8
        // and an 8-byte prefix match, after the compare, and only when some lane has one.
        uint32_t x1, x2, y1, y2;
        pm_w8(win, c1, x1, y1);
        pm_w8(win, c2, x2, y2);
        x1 ^= s4; x2 ^= s4; y1 ^= s4b; y2 ^= s4b;
        const bool go2 = c3 > limit && chain > 2;            // ... and after c2
        const int c4 = pvl[l2 && go2 ? c3 : sp];
        const bool chk1 = live && best >= 8 && (x1 | y1) == 0, chk2 = l2 && best >= 8 && (x2 | y2) == 0;
        bool cand1 = live, cand2 = l2;
        if (__ballot(chk1 || chk2)) {
            if (chk1 || chk2) {
                const uint32_t sb = win[sp + best], wb1 = win[(chk1 ? c1 : sp) + best], wb2 = win[(chk2 ? c2 : sp) + best];
                cand1 = live && wb1 == sb;
                cand2 = l2 && wb2 == sb;
            }
        }
#else
#if PM_SBREG
        const uint32_t sb = sbv, wb1 = win[c1 + best], wb2 = win[c2 + best];
#else
        const uint32_t sb = win[sp + best], wb1 = win[c1 + best], wb2 = win[c2 + best];
#endif
#if PM_W8 && PM_ISSUE
        // both candidates' dwords issued with the link and filter reads, before any use (the
        // scheduler otherwise waited for c1's bytes before issuing c2's reads: a round trip)
        const uint32_t* w32 = (const uint32_t*)win;
        const uint32_t a1 = c1 >> 2, a2 = c2 >> 2;
        const uint32_t d10 = w32[a1], d11 = w32[a1 + 1], d12 = w32[a1 + 2];
        const uint32_t d20 = w32[a2], d21 = w32[a2 + 1], d22 = w32[a2 + 2];
        // then the next link (c4, on the walk's critical path) as soon as c3 is in, then the rest
        __builtin_amdgcn_sched_barrier(0);
        const bool go2 = c3 > limit && chain > 2;            // ... and after c2
        const int c4 = pvl[l2 && go2 ? c3 : sp];
        __builtin_amdgcn_sched_barrier(0);
        uint32_t x1 = __builtin_amdgcn_alignbyte(d11, d10, c1 & 3u) ^ s4, y1 = __builtin_amdgcn_alignbyte(d12, d11, c1 & 3u) ^ s4b;
        uint32_t x2 = __builtin_amdgcn_alignbyte(d21, d20, c2 & 3u) ^ s4, y2 = __builtin_amdgcn_alignbyte(d22, d21, c2 & 3u) ^ s4b;
#elif PM_W8
        uint32_t x1, x2, y1, y2;
        pm_w8(win, c1, x1, y1);
        pm_w8(win, c2, x2, y2);
        x1 ^= s4; x2 ^= s4; y1 ^= s4b; y2 ^= s4b;
#else
        uint32_t x1 = pm_w4(win, c1) ^ s4, x2 = pm_w4(win, c2) ^ s4;
#endif
#if !(PM_W8 && PM_ISSUE)
        const bool go2 = c3 > limit && chain > 2;            // ... and after c2
        const int c4 = pvl[l2 && go2 ? c3 : sp];
#endif
        const bool cand1 = live && wb1 == sb, cand2 = l2 && wb2 == sb;
#endif
#if PM_W8
        // bytes 4-7 in the same round trip (a third aligned dword): matches of 4-7 bytes, most of
        // those that pass the filter, then need no long-compare iteration
        // (as one 64-bit count: no branch)
        const uint64_t v1 = ((uint64_t)y1 << 32) | x1, v2 = ((uint64_t)y2 << 32) | x2;
        int len1 = (int)((v1 ? (uint32_t)__builtin_ctzll(v1) : 64u) >> 3);
        int len2 = (int)((v2 ? (uint32_t)__builtin_ctzll(v2) : 64u) >> 3);
        bool more1 = cand1 && v1 == 0, more2 = cand2 && v2 == 0;
#else
        int len1 = x1 ? (int)(__builtin_ctz(x1) >> 3) : 4;
        int len2 = x2 ? (int)(__builtin_ctz(x2) >> 3) : 4;
        bool more1 = cand1 && x1 == 0, more2 = cand2 && x2 == 0;
#endif
#if PM_SBREG
        uint32_t lb1 = 0, lb2 = 0;                            // the position's byte where a long compare ended
#endif
#if PM_MORE_IF
        // the long-compare loop behind one wave-uniform test: most steps have no lane with a
        // 4-byte prefix match, and the loop's own exit test then costs nothing more
        if (__ballot(more1 || more2)) {
#if PM_COUNT
            if (A.dbg) ++n_lst;
#endif
            do {
#else
        while (__ballot(more1 || more2)) {                   // matches of more than 4 bytes
#endif
            const uint32_t cm = more1 ? c1 : c2;
            const int lm = more1 ? len1 : len2;
#if PM_SBREG
            const uint32_t wsp = pm_w4(win, sp + (uint32_t)lm);
            const uint32_t x = pm_w4(win, cm + (uint32_t)lm) ^ wsp;
#else
            const uint32_t x = pm_w4(win, cm + (uint32_t)lm) ^ pm_w4(win, sp + (uint32_t)lm);
#endif
            const int d = x ? (int)(__builtin_ctz(x) >> 3) : 4;
            const bool m1 = more1, m2 = !more1 && more2;
#if PM_SBREG
            const uint32_t xb = (wsp >> (8 * (d & 3))) & 255u;
            lb1 = m1 ? xb : lb1;
            lb2 = m2 ? xb : lb2;
#endif
#if PM_COUNT
            if (A.dbg) { ++n_it; n_itl += __popcll(__ballot(more1 || more2)); }
#endif
            len1 += m1 ? d : 0;
            len2 += m2 ? d : 0;
            more1 = m1 ? x == 0 && len1 < MAX_MATCH : more1;
            more2 = m2 ? x == 0 && len2 < MAX_MATCH : more2;
#if PM_MORE_IF
            } while (__ballot(more1 || more2));
#endif
        }
        len1 = len1 > MAX_MATCH ? MAX_MATCH : len1;
        len2 = len2 > MAX_MATCH ? MAX_MATCH : len2;
        // c1
        const bool upd1 = cand1 && len1 > best;
        best = upd1 ? len1 : best;
        bpos = upd1 ? cur : bpos;
        const bool cap1 = live && chain == cq;
        qbest = cap1 ? best : qbest;
        qpos = cap1 ? bpos : qpos;
        const bool w2 = l2 && !(upd1 && len1 >= nice);
        // c2
        const bool upd2 = w2 && cand2 && len2 > best;
        best = upd2 ? len2 : best;
        bpos = upd2 ? nxt : bpos;
        const bool cap2 = w2 && chain - 1 == cq;
        qbest = cap2 ? best : qbest;
        qpos = cap2 ? bpos : qpos;
        const bool fin = live && (!w2 || (upd2 && len2 >= nice) || !go2);
#if PM_COUNT
        if (A.dbg) n_upd += __popcll(__ballot(upd1 || upd2));
#endif
#if PM_LAZYW4
        if (upd1 || upd2) sbv = win[sp + best];
#endif
#if PM_SBREG
        // the position's byte at the new best: in the first 8 bytes (registers), else where the
        // long compare that set it ended (a best of MAX_MATCH ends the walk: nice <= MAX_MATCH)
        sbv = best < 8 ? __builtin_amdgcn_perm(s4b, s4, 0x0c0c0c00u | (uint32_t)best) : upd2 ? lb2 : upd1 ? lb1 : sbv;
#endif
        cur = c3;
        nxt = c4;
        pend = pend || fin;                                   // stored at the next refill
        chain = fin ? 0 : chain - 2;
    }
#if PM_COUNT
    if (A.dbg && lane == 0) { atomicAdd(&A.dbg[13], n_live); atomicAdd(&A.dbg[14], n_step); atomicAdd(&A.dbg[15], n_fill); }
    if (A.dbg && lane == 0) { atomicAdd(&A.dbg[16], n_it); atomicAdd(&A.dbg[17], n_itl); atomicAdd(&A.dbg[18], n_lst); atomicAdd(&A.dbg[19], n_upd); }
#endif
}

// ------------------------------------------------------------------ levels 4-9: search over 4-byte chains
// longest_match (deflate.ts:827-946) from best_len = 2 returns the first candidate (most recent)
// of maximal length among the first K = max_chain entries of the hash chain -- each above `limit`
// but the first, which may sit at MAX_DIST -- cut at the first one reaching nice_match.  A
// candidate passes its pre-check only if bytes 0-1 agree, and with an equal 15-bit hash byte 2
// then agrees too (HASH_SHIFT 5: byte 2's bits are the hash's low 5 and, xor'd with byte 1, the
// next 3).  So a result of 4 or more comes from the positions sharing the first 4 bytes, and a
// result of 3 is the first chain entry whose bytes 0-1 agree.  Text chains hold ~3x more entries
// than share 4 bytes (paradiselost.txt at L6: 35.8 candidates per search against 11.4), so:
//   k_dfl_link4  per position x, the first entry of x's chain (within the K that x's own search
//                could visit) that shares x's first 4 bytes, and its rank there (the gap).  Ranks
//                add up along a 4-byte chain -- the chain of link4(x) continues x's chain -- so a
//                walk from p knows each 4-byte candidate's rank in p's chain from the gaps alone,
//                and a link whose gap passes K can never be followed from anywhere;
//                The same walk finds the first entry whose bytes 0-1 agree: the result when no
//                entry of 4+ bytes is in the window (a 4-byte entry is one, so it comes first);
//   k_dfl_match4 per position, the walk over that 4-byte chain with the window and the links
//                (with their gaps) in LDS.
// Both chain lengths come from one walk as in k_dfl_match (the quarter window is ranks <= K/4).
// Link word: (gap - 1) << 16 | distance, 0 if none (k_dfl_match4 stages it packed, m4_pack).
// the record (k_dfl_match's word) of a search whose best is the 3-byte entry f3 (k_dfl_link4); the
// quarter word is written for every position here (k_dfl_match4 reads it back)
__device__ __forceinline__ void m4_rec3(GLB uint32_t* rec, GLB uint32_t* qrec, int p, uint32_t f3, uint32_t lb) {
    const uint32_t d = f3 & 0x7fffu, w = d ? rc_res(3u, d) : 0u, q = (f3 & 0x8000u) ? w : 0u;
    rec[p] = rc_word(w, q, lb);
    qrec[p] = q;
}
__global__ __launch_bounds__(PM_THREADS) void k_dfl_link4(DeflateArgs A) {
    __shared__ __attribute__((aligned(16))) uint8_t win[(PM_WINB + 15) & ~15];
    __shared__ __attribute__((aligned(16))) uint16_t pvl[PM_PV];
    __shared__ int pm_next;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    // four consecutive units (a stream's segments: they share history) on one XCD (block % 8)
    const uint32_t bb = blockIdx.x, u = (bb & ~31u) | ((bb & 7u) << 2) | ((bb >> 3) & 3u);
    if (u >= A.nmseg) return;
    const uint32_t sid = A.mseg[u] >> kRecUnitShift, seg = A.mseg[u] & ((1u << kRecUnitShift) - 1);
    const uint64_t rp = A.rp0[sid];
    if (rp == ~0ull) return;
    const int n = (int)A.in_len[sid];
    const int tail = n > PM_TAIL ? n - PM_TAIL : 0;
    const int s0 = (int)(seg * PM_SEG), e0 = s0 + (A.seg_merge && seg == 0 ? 3 * PM_SEG : PM_SEG);
    const int s1 = e0 < tail ? e0 : tail;
    if (s0 >= s1) return;
    const int ws = s0 > W_SIZE ? s0 - W_SIZE : 0;
    const int we = s1 + MAX_MATCH + 8 < n ? s1 + MAX_MATCH + 8 : n;
    const GLB uint8_t* in = (const GLB uint8_t*)(A.in + A.in_off[sid]);
    const GLB uint16_t* pv = (const GLB uint16_t*)A.pv_buf + rp;
    {                                                      // staging as k_dfl_match
        const int nw = (we - ws) >> 2;
        uint32_t* w32 = (uint32_t*)win;
        for (int i = (int)tid; i < nw; i += PM_THREADS) {
            uint32_t v;
            __builtin_memcpy(&v, (const uint8_t*)(in + ws + 4 * i), 4);
            w32[i] = v;
        }
        for (int i = 4 * nw + (int)tid; i < we - ws; i += PM_THREADS) win[i] = in[ws + i];
        const int np = (s1 - ws) >> 1;
        uint32_t* p32 = (uint32_t*)pvl;
        for (int i = (int)tid; i < np; i += PM_THREADS) {
            const uint32_t v = *(const GLB uint32_t*)(pv + ws + 2 * i);
            const uint32_t lo = v & 0xffffu, hi = v >> 16;
            const uint32_t r0 = 2u * (uint32_t)i, r1 = r0 + 1u;
            p32[i] = (lo && lo < r0 ? r0 - lo : 0u) | ((hi && hi < r1 ? r1 - hi : 0u) << 16);
        }
        for (int i = 2 * np + (int)tid; i < s1 - ws; i += PM_THREADS) {
            const uint32_t v = pv[ws + i];
            pvl[i] = (uint16_t)(v && v < (uint32_t)i ? (uint32_t)i - v : 0u);
        }
        if (tid == 0) pm_next = s0;
    }
    __syncthreads();
    GLB uint32_t* l4 = (GLB uint32_t*)A.l4_buf + rp;
    GLB uint32_t* rec = (GLB uint32_t*)A.rec_buf + rp;
    GLB uint32_t* qrec = (GLB uint32_t*)A.rec_buf + A.qoff + rp;
    const int K = c_config[A.level][3], Kq = K >> 2;
    // Each lane walks one position at a time and takes the next from an LDS counter itself,
    // one step ahead: its first link and 4 bytes are read in the step after the take, beside
    // the running walk's reads, so a new walk starts without a round trip of its own (walks are
    // short -- 7 entries on average at L6 -- and a wave-wide refill ran at nearly every step).
    // Walk: cur (relative) at rank r, res the link word so far, f3 the first entry whose bytes
    // 0-1 agree (the 3-byte match): distance | (rank <= K/4) << 15, 0: none.  The position's
    // record is written here as if no entry of 4+ bytes existed; k_dfl_match4 replaces the
    // halves (chain lengths) in which its walk finds one.
    int sp = 0, cur = 0, r = 0, limit = 0;
    uint32_t s4 = 0, res = 0, f3 = 0;
    bool busy = false;
    int np = 0, ncur = 0, stg = 0;                           // the next position: 0 take, 1 read, 2 ready, 3 none
    uint32_t ns4 = 0;
    unsigned long long n_hop = 0, n_step = 0;                 // SDZ_PHASE_TIMING counters
    for (;;) {
        // reads: the walk's entry, and the taken position's first link and bytes
        const int c = busy ? cur : 0;
        const uint32_t x = pm_w4(win, (uint32_t)c) ^ s4;
        const int nc = pvl[c];
        int pc = 0;
        uint32_t pw = 0;
        if (stg == 1) { pc = pvl[np - ws]; pw = pm_w4(win, (uint32_t)(np - ws)); }
        if (A.dbg) { ++n_step; n_hop += __popcll(__ballot(busy)); }
        if (busy) {                                       // one chain entry
            const bool hit = x == 0;
            res = hit ? ((uint32_t)(r - 1) << 16) | (uint32_t)(sp - cur) : res;
            if (f3 == 0 && (x & 0xffffu) == 0)            // (a 4-byte entry is a 3-byte one too)
                f3 = (uint32_t)(sp - cur) | (r <= Kq ? 0x8000u : 0u);
            const bool fin = hit || nc <= limit || r >= K;    // (nc == 0: the chain ends; limit >= 0)
            cur = nc;
            ++r;
            if (fin) {
                l4[sp + ws] = res;
                m4_rec3(rec, qrec, sp + ws, f3, win[sp + ws > 0 ? sp - 1 : 0]);
                busy = false;
            }
        }
        if (stg == 1) { ncur = pc; ns4 = pw; stg = 2; }
        if (!busy && stg == 2) {                          // start the next walk
            sp = np - ws;
            cur = ncur;
            s4 = ns4;
            res = 0; f3 = 0; r = 1;
            limit = (np > MAX_DIST ? np - MAX_DIST : 0) - ws;
            busy = cur != 0 && sp - cur <= MAX_DIST;      // the first entry (deflate.ts:1092)
            if (!busy) { l4[np] = 0u; m4_rec3(rec, qrec, np, 0u, win[np > 0 ? sp - 1 : 0]); }
            stg = 0;
        }
        if (stg == 0) {
            np = atomicAdd(&pm_next, 1);
            stg = np < s1 ? 1 : 3;
        }
        if (!__ballot(busy || stg != 3)) break;
    }
    if (A.dbg && lane == 0) { atomicAdd(&A.dbg[8], n_hop); atomicAdd(&A.dbg[9], n_step); }
}

#ifndef M4_WALKERS
#define M4_WALKERS 1                                     // 2: measured no faster
#endif
#define M4_WINB (W_SIZE + PM_SEG + MAX_MATCH + 16)
#define M4_ESC 3968                                      // escape side table (fills the LDS)
#define M4_PV (W_SIZE + PM_SEG)
static uint32_t match4_blocks(uint32_t nmseg) { return (nmseg + 127u) & ~127u; }
static uint32_t link4_blocks(uint32_t nmseg) { return (nmseg + 31u) & ~31u; }
// A link staged in LDS as 16 bits: distance << 3 | gap for distances below 8192 and gaps up to 7
// (~94 % of the links walked on text); 0: none; else an escape, (k + 1) << 3 with the word in
// the side table's entry k (m4_pack returns 8 for it; 0x1fff << 3: in HBM, the table full)
__device__ __forceinline__ uint16_t m4_pack(uint32_t v) {
    const uint32_t d = v & 0xffffu, g = (v >> 16) + 1u;
    return (uint16_t)(d == 0u ? 0u : d < 8192u && g <= 7u ? d << 3 | g : 8u);
}
template <bool kHbm>
__device__ __forceinline__ void m4_unpack(uint32_t e, const uint32_t* esc, const GLB uint32_t* l4g, int x, bool live,
                                          int& dist, int& gap) {
    if (e & 7u) { dist = (int)(e >> 3); gap = (int)(e & 7u); return; }
    uint32_t v = 0;
    if (e != 0u && live) v = kHbm && (e >> 3) == 0x1fffu ? l4g[x] : esc[(e >> 3) - 1u];
    dist = (int)(v & 0xffffu);
    gap = (int)(v >> 16) + 1;
}
// window bytes x .. x + 15 as 4 words (5 aligned dword reads)
__device__ __forceinline__ void m4_w16(const uint8_t* w, uint32_t x, uint32_t (&m)[4]) {
    const uint32_t* w32 = (const uint32_t*)w + (x >> 2);
    const uint32_t s = x & 3u;
    uint32_t d[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) d[i] = w32[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) m[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], s);
}
// equal leading bytes of two 16-byte strings, from their xor words (16: all equal)
__device__ __forceinline__ int m4_lcp16(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
    const int k = x0 ? 0 : x1 ? 4 : x2 ? 8 : x3 ? 12 : 16;
    const uint32_t x = x0 ? x0 : x1 ? x1 : x2 ? x2 : x3;
    return k == 16 ? 16 : k + (int)(__builtin_ctz(x) >> 3);
}
// k_dfl_match4's walks (kHbm: the escape table overflowed, some link words stay in HBM)
template <bool kHbm>
__device__ __forceinline__ void m4_walks(const uint8_t* win, const uint16_t* lk, const uint32_t* esc,
                                         const GLB uint32_t* l4g, GLB uint32_t* rec, GLB uint32_t* qrec, int* pm_next, int ws, int s1,
                                         int K, int Kq, int nice, unsigned long long* dbg, uint32_t lane) {
    // Each lane runs M4_WALKERS walks side by side (their LDS round trips overlap) and takes
    // the next position from an LDS counter itself, one step ahead (as k_dfl_link4): the taken
    // position's link and bytes 4-19 are read in the step after the take, beside the running
    // walks' reads; the first walker free takes it.  No HBM loads in the loop (a wait on one
    // would also wait for every record store before it).
    // Walk k: position sp (relative to ws; < 0 none), its limit, the 4-byte candidate cur at rank cum.
    constexpr int W = M4_WALKERS;
    int sp[W], cur[W], cum[W], limit[W], best[W], bpos[W], qbest[W], qpos[W];
    uint32_t pw[W][4];                                       // p's bytes 4-19
    bool busy[W];
#pragma unroll
    for (int k = 0; k < W; ++k) {
        sp[k] = -1; cur[k] = cum[k] = limit[k] = bpos[k] = qpos[k] = 0; best[k] = qbest[k] = 2;
        pw[k][0] = pw[k][1] = pw[k][2] = pw[k][3] = 0u;
        busy[k] = false;
    }
    int np = 0, stg = 0;                                     // the next position: 0 take, 1 read, 2 ready, 3 none
    uint32_t ne = 0, npw[4] = { 0, 0, 0, 0 };
    unsigned long long n_cand = 0, n_step = 0;               // SDZ_PHASE_TIMING counters
    for (;;) {
        // reads: each candidate's link and bytes 4-19; the taken position's link, bytes, 3-byte entry
        uint32_t e[W], m[W][4];
#pragma unroll
        for (int k = 0; k < W; ++k) {
            const int c = busy[k] ? cur[k] : 0;
            e[k] = lk[c];
            m4_w16(win, (uint32_t)(c + 4), m[k]);
        }
        uint32_t pe = 0, ppw[4] = { 0, 0, 0, 0 };
        if (stg == 1) {
            pe = lk[np - ws];
            m4_w16(win, (uint32_t)(np - ws + 4), ppw);
        }
        if (dbg) {
            ++n_step;
#pragma unroll
            for (int k = 0; k < W; ++k) n_cand += __popcll(__ballot(busy[k]));
        }
        int len[W], nl[W], ng[W];
        bool more[W];
#pragma unroll
        for (int k = 0; k < W; ++k) {
            nl[k] = ng[k] = 0;
            m4_unpack<kHbm>(e[k], esc, l4g, cur[k], busy[k], nl[k], ng[k]);
            len[k] = 4 + m4_lcp16(m[k][0] ^ pw[k][0], m[k][1] ^ pw[k][1], m[k][2] ^ pw[k][2], m[k][3] ^ pw[k][3]);
            more[k] = busy[k] && len[k] == 20;
        }
        for (;;) {                                           // matches past 20 bytes
            bool any = false;
#pragma unroll
            for (int k = 0; k < W; ++k) any = any || more[k];
            if (!__ballot(any)) break;
#pragma unroll
            for (int k = 0; k < W; ++k) {
                if (more[k]) {
                    uint32_t a[4], b[4];
                    m4_w16(win, (uint32_t)(cur[k] + len[k]), a);
                    m4_w16(win, (uint32_t)(sp[k] + len[k]), b);
                    const int d = m4_lcp16(a[0] ^ b[0], a[1] ^ b[1], a[2] ^ b[2], a[3] ^ b[3]);
                    len[k] += d;
                    more[k] = d == 16 && len[k] < MAX_MATCH;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < W; ++k) {
            const int ln = len[k] > MAX_MATCH ? MAX_MATCH : len[k];
            const bool upd = busy[k] && ln > best[k];
            best[k] = upd ? ln : best[k];
            bpos[k] = upd ? cur[k] : bpos[k];
            const bool cap = busy[k] && cum[k] <= Kq;
            qbest[k] = cap ? best[k] : qbest[k];
            qpos[k] = cap ? bpos[k] : qpos[k];
            const int ncur = cur[k] - nl[k], ncum = cum[k] + ng[k];
            const bool fin = (upd && ln >= nice) || nl[k] == 0 || ncum > K || ncur <= limit[k];
            cur[k] = busy[k] ? ncur : cur[k];
            cum[k] = busy[k] ? ncum : cum[k];
            busy[k] = busy[k] && !fin;
        }
        if (stg == 1) { ne = pe; npw[0] = ppw[0]; npw[1] = ppw[1]; npw[2] = ppw[2]; npw[3] = ppw[3]; stg = 2; }
#pragma unroll
        for (int k = 0; k < W; ++k) {
            if (!busy[k] && sp[k] >= 0) {                    // a walk ended: the halves it improves
                // (k_dfl_link4 wrote the record of the 3-byte entry, and its quarter word)
                if (best[k] >= 4 || qbest[k] >= 4) {
                    const int pp = sp[k] + ws;
                    const uint32_t lb = win[pp > 0 ? sp[k] - 1 : 0];
                    const uint32_t o = rec[pp], oq = qrec[pp];
                    const uint32_t full = best[k] >= 4 ? rc_res((uint32_t)best[k], (uint32_t)(sp[k] - bpos[k])) : o & 0x7fffffu;
                    const uint32_t quarter = qbest[k] >= 4 ? rc_res((uint32_t)qbest[k], (uint32_t)(sp[k] - qpos[k])) : oq;
                    rec[pp] = rc_word(full, quarter, lb);
                    qrec[pp] = quarter;
                }
                sp[k] = -1;
            }
            if (sp[k] < 0 && stg == 2) {                     // start the taken position
                sp[k] = np - ws;
                pw[k][0] = npw[0]; pw[k][1] = npw[1]; pw[k][2] = npw[2]; pw[k][3] = npw[3];
                limit[k] = (np > MAX_DIST ? np - MAX_DIST : 0) - ws;
                best[k] = 2; bpos[k] = 0; qbest[k] = 2; qpos[k] = 0;
                int l = 0, g = 0;
                m4_unpack<kHbm>(ne, esc, l4g, sp[k], true, l, g);  // (no search at p: no link, deflate.ts:1092)
                cur[k] = sp[k] - l;
                cum[k] = g;
                busy[k] = l != 0 && g <= K && (g == 1 || cur[k] > limit[k]);
                stg = 0;
            }
        }
        if (stg == 0) {
            np = atomicAdd(pm_next, 1);
            stg = np < s1 ? 1 : 3;
        }
        bool act = stg != 3;
#pragma unroll
        for (int k = 0; k < W; ++k) act = act || busy[k] || sp[k] >= 0;
        if (!__ballot(act)) break;
    }
    if (dbg && lane == 0) { atomicAdd(&dbg[11], n_cand); atomicAdd(&dbg[12], n_step); }
}
__global__ __launch_bounds__(PM_THREADS) void k_dfl_match4(DeflateArgs A) {
    __shared__ __attribute__((aligned(16))) uint8_t win[(M4_WINB + 15) & ~15];
    __shared__ __attribute__((aligned(16))) uint16_t lk[M4_PV];   // m4_pack words
    __shared__ uint32_t esc[M4_ESC];                               // link words of the escapes
    __shared__ int pm_next, esc_n;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    // block -> unit: of each 128 blocks, the 16 on XCD x (block % 8) take units 16 x .. 16 x + 15
    const uint32_t bb = blockIdx.x, item = (bb & ~127u) | ((bb & 7u) << 4) | ((bb >> 3) & 15u);
    const uint32_t u = item;
    if (u >= A.nmseg) return;
    const uint32_t sid = A.mseg[u] >> kRecUnitShift, seg = A.mseg[u] & ((1u << kRecUnitShift) - 1);
    const uint64_t rp = A.rp0[sid];
    if (rp == ~0ull) return;
    const int n = (int)A.in_len[sid];
    const int tail = n > PM_TAIL ? n - PM_TAIL : 0;
    const int ge = (int)(seg * PM_SEG) + (A.seg_merge && seg == 0 ? 3 * PM_SEG : PM_SEG);
    const int g1 = ge < tail ? ge : tail;
    const int s0 = (int)(seg * PM_SEG), s1 = g1;
    if (s0 >= s1) return;
    const int ws = s0 > W_SIZE ? s0 - W_SIZE : 0;
    const int we = s1 + MAX_MATCH + 8 < n ? s1 + MAX_MATCH + 8 : n;
    const GLB uint8_t* in = (const GLB uint8_t*)(A.in + A.in_off[sid]);
    const GLB uint32_t* l4g = (const GLB uint32_t*)A.l4_buf + rp + ws;   // relative to ws
    if (tid == 0) esc_n = 0;
    __syncthreads();
    {
        const int nw = (we - ws) >> 2;
        uint32_t* w32 = (uint32_t*)win;
        for (int i = (int)tid; i < nw; i += PM_THREADS) {
            uint32_t v;
            __builtin_memcpy(&v, (const uint8_t*)(in + ws + 4 * i), 4);
            w32[i] = v;
        }
        for (int i = 4 * nw + (int)tid; i < we - ws; i += PM_THREADS) win[i] = in[ws + i];
        for (int i = (int)tid; i < s1 - ws; i += PM_THREADS) {
            const uint32_t v = l4g[i];
            uint32_t e = m4_pack(v);
            if (e == 8u) {                                     // an escape: its word in the side table
                const int k = atomicAdd(&esc_n, 1);
                if (k < M4_ESC) { esc[k] = v; e = (uint32_t)(k + 1) << 3; }
                else e = 0x1fffu << 3;                         // (table full: the word stays in HBM)
            }
            lk[i] = (uint16_t)e;
        }
        if (tid == 0) pm_next = s0;
    }
    __syncthreads();
    GLB uint32_t* rec = (GLB uint32_t*)A.rec_buf + rp;
    GLB uint32_t* qrec = (GLB uint32_t*)A.rec_buf + A.qoff + rp;
    const int K = c_config[A.level][3], Kq = K >> 2, nice = c_config[A.level][2];
    if (esc_n > M4_ESC) m4_walks<true>(win, lk, esc, l4g, rec, qrec, &pm_next, ws, s1, K, Kq, nice, A.dbg, lane);
    else m4_walks<false>(win, lk, esc, l4g, rec, qrec, &pm_next, ws, s1, K, Kq, nice, A.dbg, lane);
}

// ------------------------------------------------------------------ record path: tail, parse, trees, encode
// After k_dfl_chain / k_dfl_match the rest of deflate_slow is split by what it depends on:
//   k_dfl_tail   records of the last PM_TAIL positions (the reference's longest_match itself);
//   k_dfl_parse  the lazy parse (deflate.ts:1054-1182) and _tr_tally (deflate.ts:488-524):
//                serial per stream but only registers + one round trip per position; emits
//                the symbols and where each block ends (the flush points);
//   k_dfl_trees  per block: frequencies, build_tree / build_bl_tree, the block type choice of
//                _tr_flush_block (deflate.ts:614-674), the code table and the header bits;
//   k_dfl_encode per stream: bit layout of its blocks, then the symbols of each block packed
//                by all threads at prefix-summed bit offsets (compress_block, deflate.ts:527-571).
// A stream leaves the path (flag) where the reference's output would not be the plain
// bitstream -- its pending_buf overlay overtaken by the output, a pending_buf or
// output slot overflow -- and is redone by the serial kernel (k_deflate, A.fast).

// The window at the end of the input, in the reference's coordinates (deflate.ts:690-766): the
// window (64 KiB, zero-filled at construction, deflate.ts:119) slides by 32 KiB when
// fill_window finds strstart >= 65274 with lookahead < MIN_LOOKAHEAD; a slide copies the
// upper half down and leaves the upper half as it was (stale), and fill_window then reads
// input greedily.  After e slides (off = 32 Ki e) window index i holds input byte
// i + off if i < F_e = min(64 Ki, n - off); otherwise what the same index held before the
// last slide (index i + 32 Ki for the lower half, i for the upper half), back to zeros.
// Only the last positions' searches (lookahead < MAX_MATCH) read past the input.
__device__ uint32_t win_byte(const GLB uint8_t* in, int64_t n, int64_t off, int64_t i) {
    for (int64_t e = off / W_SIZE;; --e) {
        const int64_t base = e * W_SIZE;
        const int64_t F = n - base < WINDOW_SIZE ? n - base : WINDOW_SIZE;
        if (i < F) return in[base + i];
        if (e == 0) return 0u;
        if (i < W_SIZE) i += W_SIZE;
    }
}
// window offset when the parse is at original position P: slide e happens at the first
// visited position with strstart >= 65274 and lookahead < MIN_LOOKAHEAD in epoch e - 1 (both
// grow with P, so every visited P has the offset this loop finds)
__device__ __forceinline__ int64_t slide_off(int64_t n, int64_t P) {
    int64_t off = 0;
    // the slides with the window's end still inside the input happen at P - off >= 65275
    // (fe - P < MIN_LOOKAHEAD with fe = off + 64 Ki): taken in one go, the loop does the rest
    if (P >= WINDOW_SIZE - MIN_LOOKAHEAD + 1 && n >= WINDOW_SIZE) {
        const int64_t e = (P - (WINDOW_SIZE - MIN_LOOKAHEAD + 1)) / W_SIZE + 1, emid = (n - WINDOW_SIZE) / W_SIZE + 1;
        off = (int64_t)W_SIZE * (e < emid ? e : emid);
    }
    for (;;) {
        const int64_t fe = n < off + WINDOW_SIZE ? n : off + WINDOW_SIZE;
        if (fe - P < MIN_LOOKAHEAD && P - off >= WINDOW_SIZE - MIN_LOOKAHEAD) off += W_SIZE;
        else return off;
    }
}
// deflate.ts:827-946 at original position P (lookahead >= MIN_MATCH), from best_len = 2, for
// chain_length and chain_length >> 2 in one walk: the shorter walk is the longer one's first
// qchain candidates.  Record word as in k_dfl_match (quarter in the high half).  The search
// runs in the window coordinates the reference has at P; pv holds each position's distance
// to its previous same-hash position (0: none), and the reference's rebased links (0 below
// the window) end a walk exactly where these would pass `limit`.
__device__ uint64_t tail_search(const GLB uint8_t* in, const GLB uint16_t* pv, int64_t n, int64_t P, int chain_length,
                                int nice) {
    const int64_t off = slide_off(n, P);
    const int strstart = (int)(P - off);
    auto prev_of = [&](int64_t q) -> int {                // window index of q's predecessor (0: none)
        const uint32_t d = pv[q];
        const int64_t r = q - (int64_t)d;
        return d && r > off ? (int)(r - off) : 0;
    };
    auto wb = [&](int i) -> uint32_t { return win_byte(in, n, off, i); };
    int cur = prev_of(P);
    if (cur == 0 || ((strstart - cur) & 0xffff) > MAX_DIST) return 0u;      // no search (deflate.ts:1092)
    const int lookahead = (int)(n - P);
    if (nice > lookahead) nice = lookahead;
    const int limit = strstart > MAX_DIST ? strstart - MAX_DIST : 0;
    const int qchain = chain_length >> 2;
    int best = MIN_MATCH - 1, bstart = 0, qbest = -1, qstart = 0, k = 0;
    uint32_t scan_end1 = wb(strstart + best - 1), scan_end = wb(strstart + best);
    const uint32_t c0 = wb(strstart), c1 = wb(strstart + 1);
    // The link and the four checked bytes of a candidate are loaded together, and a long
    // compare takes 4 byte pairs per step, so the walk waits on one memory round trip per
    // candidate rather than on one per load.
    do {
        const int match = cur;
        const int nx = prev_of(match + off);
        const uint32_t e0 = wb(match + best), e1 = wb(match + best - 1);
        const uint32_t m0 = wb(match), m1 = wb(match + 1);
        if ((e0 == scan_end) & (e1 == scan_end1) & (m0 == c0) & (m1 == c1)) {
            int len = 3;                      // byte 2 is not compared (equal hash, deflate.ts:891-897)
            for (bool go = true; go && len < MAX_MATCH;) {
                uint32_t x[4], y[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    x[i] = wb(strstart + len + i);
                    y[i] = wb(match + len + i);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (go && len < MAX_MATCH && x[i] == y[i]) ++len;
                    else go = false;
                }
            }
            if (len > best) {
                bstart = match;
                best = len;
                if (len >= nice) break;
                scan_end1 = wb(strstart + best - 1);
                scan_end = wb(strstart + best);
            }
        }
        if (++k == qchain) { qbest = best; qstart = bstart; }
        cur = nx;
    } while (cur > limit && --chain_length != 0);
    if (qbest < 0) { qbest = best; qstart = bstart; }
    const uint32_t full = best > MIN_MATCH - 1 ? ((uint32_t)best << 16) | (uint32_t)(strstart - bstart) : 0u;
    const uint32_t quarter = qbest > MIN_MATCH - 1 ? ((uint32_t)qbest << 16) | (uint32_t)(strstart - qstart) : 0u;
    return ((uint64_t)quarter << 32) | full;
}
__global__ __launch_bounds__(256) void k_dfl_tail(DeflateArgs A) {
    const uint32_t sid = blockIdx.x;
    if (sid >= A.n) return;
    const uint64_t rp = A.rp0[sid];
    if (rp == ~0ull) return;
    const int64_t n = (int64_t)A.in_len[sid], tail = n > PM_TAIL ? n - PM_TAIL : 0;
    const GLB uint8_t* in = (const GLB uint8_t*)(A.in + A.in_off[sid]);
    const GLB uint16_t* pv = (const GLB uint16_t*)A.pv_buf + rp;
    GLB uint32_t* rec = (GLB uint32_t*)A.rec_buf + rp;
    GLB uint32_t* qrec = (GLB uint32_t*)A.rec_buf + A.qoff + rp;
    const int max_chain = c_config[A.level][3], nice = c_config[A.level][2];
    // with A.tail_in_match, k_dfl_match searched the larger window-offset group already (a stream
    // with match segments, tail > 0); the last MIN_MATCH - 1 positions are not searched, their
    // records carry only the byte
    TailGroups tg = { n, n, 0 };
    if (A.tail_in_match && tail > 0) tg = tail_groups(n, tail);
    for (int64_t P = tail + (int64_t)threadIdx.x; P < n; P += 256) {
        if (P >= tg.mlo && P < tg.mhi) continue;
        const uint64_t r = P <= n - MIN_MATCH ? tail_search(in, pv, n, P, max_chain, nice) : 0ull;
        const uint32_t full = rc_from16((uint32_t)r), quarter = rc_from16((uint32_t)(r >> 32));
        rec[P] = rc_word(full, quarter, in[P > 0 ? P - 1 : 0]);
        if (quarter != full) qrec[P] = quarter;
    }
}

// k_dfl_parse: the reference's loop (deflate_slow, deflate.ts:1054-1182) with its scalars in
// registers, one record load per step.  At each position the record gives
// longest_match(prev_length): the record's candidate if it is longer than prev_length, else
// prev_length, clamped to the lookahead.  (In the tail with prev_length >= min(nice,
// lookahead) the reference returns the lookahead, and so does this; otherwise its walk stops
// at the same candidate as the record's.)  Positions with lookahead < MIN_MATCH are not
// searched here: the reference's result there is <= 2 either way and nothing downstream
// tells the values apart.
// Positions are original (absolute) ones.  The reference's window slides when fill_window
// finds strstart >= 65274 with lookahead < MIN_LOOKAHEAD (deflate.ts:708-737); that changes
// no decision (a search reads no byte past the input unless lookahead < MAX_MATCH, and
// lookahead is n - P whenever it matters), only the window coordinates a flush records
// (block_start < 0: no stored block, deflate.ts:648).
// Symbols go to the stream's symbol buffer -- the front of its record buffer: symbol k is
// written after record k/2 has been read -- as lc | dist << 8 (dist 0: literal lc).
struct PState {
    int n, level, good, max_lazy;
    int strstart, match_length, match_start, match_available, block_start;
    int64_t off;
    uint32_t last_lit, matches, lx, nblk, sym0, nbcap;
    // TRUNCATE_BLOCK's estimate needs only sum over the block's matches of 5 + extra bits of
    // the distance code (deflate.ts:503-506), kept as a running sum: extra bits of distance
    // d + 1 are 0 for d < 4, else floor(log2 d) - 1 (no dist_code table, no per-code counts)
    uint32_t dxb;
    GLB uint32_t* sym;
    uint32_t* stg;                // null, or an LDS stage of PS_STG symbols written as whole 64-B pieces
    uint8_t* blk;                 // this stream's first block slot
};
#define PS_STG 16
__device__ __forceinline__ void ps_init(PState& st, const DeflateArgs& A, uint32_t sid, int n) {
    st.n = n; st.level = A.level; st.good = c_config[A.level][0]; st.max_lazy = c_config[A.level][1];
    st.strstart = 0; st.match_length = MIN_MATCH - 1; st.match_start = 0; st.match_available = 0;
    st.block_start = 0; st.off = 0;
    st.last_lit = 0; st.matches = 0; st.lx = 0; st.nblk = 0; st.sym0 = 0; st.dxb = 0;
    st.sym = (GLB uint32_t*)A.sym_buf + A.rp0[sid];
    st.stg = nullptr;
    st.blk = A.blk + (uint64_t)A.tb0[sid] * FB_SLOT;
    st.nbcap = A.tb0[sid + 1] - A.tb0[sid];
}
// the staged symbols [lx & ~(PS_STG - 1), lx) to the symbol buffer
__device__ __forceinline__ void ps_drain(PState& st) {
    const uint32_t k0 = st.lx & ~(PS_STG - 1u);
    for (uint32_t k = k0; k < st.lx; ++k) st.sym[k] = st.stg[k - k0];
}
__device__ __forceinline__ bool ps_tally(PState& st, int dist, int lc) {      // _tr_tally, deflate.ts:488-524
    const uint32_t v = (uint32_t)lc | ((uint32_t)dist << 8);
    if (st.stg) {
        // staged: a lane's symbols leave in 64-byte pieces (4-byte stores of 64 lanes to 64 streams
        // wrote ~2.4x the symbol bytes to HBM: partial lines evicted before they filled)
        st.stg[st.lx & (PS_STG - 1u)] = v;
        if ((++st.lx & (PS_STG - 1u)) == 0) {
            const uint2* q = (const uint2*)st.stg;
            uint2* d = (uint2*)(uint32_t*)(st.sym + st.lx - PS_STG);   // (8-byte aligned: rp0 is a multiple of 64)
#pragma unroll
            for (int k = 0; k < PS_STG / 2; ++k) d[k] = q[k];
        }
    } else {
        st.sym[st.lx++] = v;
    }
    st.last_lit++;
    if (dist) {
        st.matches++;
        const uint32_t d = (uint32_t)(dist - 1);
        st.dxb += 5u + (d < 4u ? 0u : 30u - (uint32_t)__builtin_clz(d));
    }
    if ((st.last_lit & 0x1fff) == 0 && st.level > 2) {                       // TRUNCATE_BLOCK
        uint32_t out_length = st.last_lit * 8 + st.dxb;
        const int in_length = st.strstart - st.block_start;
        out_length >>= 3;
        if (st.matches < st.last_lit / 2 && (int)out_length < in_length / 2) return true;
    }
    return st.last_lit == LIT_BUFSIZE - 1;
}
__device__ __forceinline__ void ps_flush(PState& st, uint32_t eof) {          // flush_block_only's bookkeeping
    if (st.nblk < st.nbcap) {
        GLB FBlock* B = (GLB FBlock*)(st.blk + (uint64_t)st.nblk * FB_SLOT);
        B->sym0 = st.sym0; B->nsym = st.last_lit;
        B->block_start = (int32_t)(st.block_start - st.off); B->strstart = (int32_t)(st.strstart - st.off);
        B->off = st.off; B->eof = eof;
    }
    st.nblk++;
    st.sym0 = st.lx; st.last_lit = 0; st.matches = 0; st.dxb = 0;
    st.block_start = st.strstart;
}
// the step's fill_window: true when the input is used up (lookahead == 0)
__device__ __forceinline__ bool ps_fill(PState& st) {
    const int64_t fe = (int64_t)st.n < st.off + WINDOW_SIZE ? (int64_t)st.n : st.off + WINDOW_SIZE;
    if (fe - st.strstart < MIN_LOOKAHEAD) {
        if (st.strstart - st.off >= WINDOW_SIZE - MIN_LOOKAHEAD) st.off += W_SIZE;   // the slide
        if (st.strstart == st.n) return true;
    }
    return false;
}
// one step at position strstart with its record r (rc_word) and, when prev_length >= good_match,
// the quarter word q there (ps_qload: loaded beside the record, not after it)
__device__ __forceinline__ uint32_t ps_qload(const PState& st, const GLB uint32_t* qrec) {
    return st.match_length >= st.good ? qrec[st.strstart] : 0u;
}
__device__ __forceinline__ void ps_step(PState& st, uint32_t r, uint32_t q) {
    const uint32_t lb = r >> 24;
    const int lookahead = st.n - st.strstart;
    const int prev_length = st.match_length, prev_match = st.match_start;
    st.match_length = MIN_MATCH - 1;
    // The reference also requires hash_head != 0 and (strstart - hash_head) <= MAX_DIST
    // (deflate.ts:1092).  Where that fails the record is 0 (k_dfl_match / k_dfl_tail test
    // the same), and a 0 record gives the step the same outcome as no search: match_length
    // ends <= prev_length, so with prev_length >= MIN_MATCH the previous match is emitted
    // either way, and otherwise it stays MIN_MATCH - 1.  So the link load is not needed.
    if (lookahead >= MIN_MATCH && prev_length < st.max_lazy) {
        const uint32_t e = prev_length >= st.good && (r & (1u << 23)) ? q : r;
        const int len = (int)rc_len(e);
        int ml = prev_length;
        if (len > prev_length) { ml = len; st.match_start = st.strstart - (int)(e & 0x7fffu); }
        st.match_length = ml < lookahead ? ml : lookahead;
        if (st.match_length <= 5 && st.match_length == MIN_MATCH && st.strstart - st.match_start > 4096)
            st.match_length = MIN_MATCH - 1;
    }
    if (prev_length >= MIN_MATCH && st.match_length <= prev_length) {
        const bool bflush = ps_tally(st, st.strstart - 1 - prev_match, prev_length - MIN_MATCH);
        // strstart+1 .. strstart+prev_length-2 are inserted (up to max_insert); their links
        // are already in the chain buffer (k_dfl_chain), and the records carry the search
        // test, so nothing is read here
        st.strstart += prev_length - 1;
        st.match_available = 0;
        st.match_length = MIN_MATCH - 1;
        if (bflush) ps_flush(st, 0);
    } else if (st.match_available) {
        const bool bflush = ps_tally(st, 0, (int)lb);
        if (bflush) ps_flush(st, 0);
        st.strstart++;
    } else {
        st.match_available = 1;
        st.strstart++;
    }
}
__device__ __forceinline__ void ps_finish(PState& st, const GLB uint8_t* in, GLB FStream* F) {
    if (st.match_available) ps_tally(st, 0, in[st.strstart - 1]);
    if (st.stg) ps_drain(st);
    ps_flush(st, 1);
    F->nblk = st.nblk;
    F->flag = st.nblk > st.nbcap ? 1u : 0u;
}
// many streams: one lane each
__global__ __launch_bounds__(64) void k_dfl_parse(DeflateArgs A) {
    const uint32_t lane = threadIdx.x, sid = blockIdx.x * 64 + lane;
    if (sid >= A.n) return;
    GLB DSlab* S = (GLB DSlab*)(A.state + (uint64_t)sid * SLAB_BYTES);
    GLB FStream* F = (GLB FStream*)S->window;
    const uint64_t in_len = A.in_len[sid];
    if (in_len == 0 || A.rp0[sid] == ~0ull) { F->nblk = 0; F->flag = 1; return; }
    const GLB uint8_t* in = (const GLB uint8_t*)(A.in + A.in_off[sid]);
    const GLB uint32_t* rec = (const GLB uint32_t*)A.rec_buf + A.rp0[sid];
    const GLB uint32_t* qrec = (const GLB uint32_t*)A.rec_buf + A.qoff + A.rp0[sid];
    __shared__ __attribute__((aligned(16))) uint32_t stage[64 * PS_STG];
    PState st;
    ps_init(st, A, sid, (int)in_len);
    st.stg = stage + lane * PS_STG;
    for (;;) {
        if (ps_fill(st)) break;
        uint32_t r = rec[st.strstart];                        // the step's one load (rc_word) ...
        uint32_t q = ps_qload(st, qrec);                      // ... and beside it the quarter word it may use
        asm volatile("" : "+v"(r), "+v"(q));                  // here, not sunk into the branches
        ps_step(st, r, q);
    }
    ps_finish(st, in, F);
}
// few long streams (the facade's one-buffer deflate()): one workgroup per stream; waves 1..3
// stage the records in LDS chunks ahead of lane 0, which parses from LDS (a lone lane waits
// on every dependent HBM load otherwise)
#define PW_THREADS 256
#ifndef PW_UNIFORM
#define PW_UNIFORM 1
#endif
#define PW_CHUNK 4096                                    // records per LDS chunk (>= MAX_MATCH)
#ifdef DT_PROF
#define PW_T(k) do { if (blockIdx.x == 0 && tid == 0) tw[k] = wall_clock64(); } while (0)
#else
#define PW_T(k) do { } while (0)
#endif
__global__ __launch_bounds__(PW_THREADS) void k_dfl_parse_wide(DeflateArgs A) {
    __shared__ uint32_t buf[2][PW_CHUNK];
    const uint32_t sid = blockIdx.x, tid = threadIdx.x;
#ifdef DT_PROF
    uint64_t tw[6] = {};
#endif
    PW_T(0);
    if (sid >= A.n) return;
    GLB DSlab* S = (GLB DSlab*)(A.state + (uint64_t)sid * SLAB_BYTES);
    GLB FStream* F = (GLB FStream*)S->window;
    const uint64_t in_len = A.in_len[sid];
    if (in_len == 0 || A.rp0[sid] == ~0ull) { if (tid == 0) { F->nblk = 0; F->flag = 1; } return; }
    const int n = (int)in_len;
    const GLB uint8_t* in = (const GLB uint8_t*)(A.in + A.in_off[sid]);
    const GLB uint32_t* rec = (const GLB uint32_t*)A.rec_buf + A.rp0[sid];
    const GLB uint32_t* qrec = (const GLB uint32_t*)A.rec_buf + A.qoff + A.rp0[sid];
    const int nch = (n + PW_CHUNK - 1) / PW_CHUNK;
    for (int i = (int)tid; i < PW_CHUNK && i < n; i += PW_THREADS) buf[0][i] = rec[i];
    __syncthreads();
    PW_T(1);
    PState st;
    bool done = false;
#if PW_UNIFORM
    // wave 0 runs the parse with every lane on the same values: the state is wave-uniform
    // (scalar registers, scalar branches) instead of lane 0's masked vector code; the
    // symbol and block stores are made by all 64 lanes to one address
    const bool parser = __builtin_amdgcn_readfirstlane(tid) < 64;
#else
    const bool parser = tid == 0;
#endif
    if (parser) ps_init(st, A, sid, n);
    PW_T(2);
    for (int c = 0; c < nch; ++c) {
        const int c1 = c + 1;
        if (tid >= 64 && c1 < nch) {                    // stage the next chunk
            const int b0 = c1 * PW_CHUNK, m = n - b0 < PW_CHUNK ? n - b0 : PW_CHUNK;
            for (int i = (int)tid - 64; i < m; i += PW_THREADS - 64) buf[c1 & 1][i] = rec[b0 + i];
        }
        if (parser && !done) {
            const int end = (c + 1) * PW_CHUNK, b0 = c * PW_CHUNK;
            const uint32_t* cb = buf[c & 1];
#if PW_UNIFORM
            // the records of positions rb .. rb + 63 in lane order (one LDS read per 64
            // positions); a step takes its record with readlane instead of waiting on LDS
            int rb = -(1 << 30);
            uint32_t rlo = 0;
#endif
            for (;;) {
                if (st.strstart >= end) break;             // the next chunk (a step moves <= MAX_MATCH)
                if (ps_fill(st)) { done = true; break; }
#if PW_UNIFORM
                int o = st.strstart - rb;
                if ((uint32_t)o >= 64u) {
                    rb = st.strstart;
                    o = 0;
                    const int i = rb - b0 + (int)tid;
                    rlo = i < PW_CHUNK ? cb[i] : 0u;
                }
                const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)rlo, o);
#else
                const uint32_t r = cb[st.strstart - b0];
#endif
                ps_step(st, r, ps_qload(st, qrec));
            }
        }
        __syncthreads();
    }
    PW_T(3);
    if (parser) {
        // (the records past the last chunk: none -- a stream's positions end at n)
        ps_finish(st, in, F);
    }
    PW_T(4);
#ifdef DT_PROF
    if (sid == 0 && tid == 0)
        printf("PW_PROF n %d | stage %lu init %lu loop %lu finish %lu [x10ns]\n", n, tw[1] - tw[0], tw[2] - tw[1],
               tw[3] - tw[2], tw[4] - tw[3]);
#endif
}

// ------------------------------------------------------------------ segment-parallel lazy parse
// deflate_slow's parse (deflate.ts:1054-1182) is a walk over step positions whose state between
// steps is (prev_length, prev_match, match_available) and whose step reads one record.  Block
// flushes do not feed back into it (they only cut the symbol sequence: _tr_tally's verdict,
// deflate.ts:488-524), so the symbols are found first and cut into blocks afterwards:
//   k_lz_spec    one lane per segment (2^lz_shift positions) parses it from a fresh state
//                (prev_length 2, nothing pending) -- a guess -- and records, by position, the
//                state before each step and the symbol the step emits;
//   k_lz_join    one lane per segment boundary carries the previous segment's parse on into
//                the segment until it stands on a position the segment's own parse visited in
//                the same state: both are one parse from there (lazy parses fall back into step
//                within a few symbols, so that is a handful of steps);
//   k_lz_fix     one lane per stream takes the boundaries in order: where a join crossed a
//                whole segment without meeting its parse (long matches out of phase: runs),
//                the true parse entering the next segment is that join's carry, and the next
//                join is redone from it;
//   k_lz_count / k_lz_scan / k_lz_emit   the symbols in order into the stream's symbol buffer;
//   k_lz_blocks  one workgroup per stream cuts them into blocks where _tr_tally would flush
//                (TRUNCATE_BLOCK at 8192 symbols, LIT_BUFSIZE - 1), the sums it tests reduced
//                over the block's symbols.
// The result is the serial parse's (k_dfl_parse) symbol for symbol, block for block.
struct LzSt {
    int s, ml, ms, avail;           // step position; prev_length, prev_match, match_available
};
#define LZ_SYM 0x80000000u          // a step's symbol word: emitted flag | lc | dist << 8
#define LZ_THREADS 64
// the state as compared between parses: prev_match only matters with prev_length >= MIN_MATCH
__device__ __forceinline__ uint32_t lz_pack(const LzSt& t) {
    return t.ml >= MIN_MATCH ? (uint32_t)t.ml | ((uint32_t)(t.s - t.ms) << 9) | ((uint32_t)t.avail << 25)
                             : (uint32_t)(MIN_MATCH - 1) | ((uint32_t)t.avail << 25);
}
__device__ __forceinline__ uint64_t lz_save(const LzSt& t) { return (uint64_t)(uint32_t)t.s | ((uint64_t)lz_pack(t) << 32); }
__device__ __forceinline__ LzSt lz_load(uint64_t v) {
    const uint32_t p = (uint32_t)(v >> 32);
    LzSt t;
    t.s = (int)(uint32_t)v;
    t.ml = (int)(p & 511u);
    t.ms = t.s - (int)((p >> 9) & 0xffffu);
    t.avail = (int)((p >> 25) & 1u);
    return t;
}
// one step of deflate_slow at t.s with the record r there (as ps_step); returns the symbol
// it emits (LZ_SYM set) or 0
__device__ __forceinline__ uint32_t lz_step(LzSt& t, uint32_t r, const GLB uint32_t* qrec, int n, int good, int max_lazy) {
    const int lookahead = n - t.s;
    const int prev_length = t.ml, prev_match = t.ms;
    int ml = MIN_MATCH - 1, ms = t.ms;
    if (lookahead >= MIN_MATCH && prev_length < max_lazy) {
        const uint32_t e = prev_length >= good && (r & (1u << 23)) ? qrec[t.s] : r;
        const int len = (int)rc_len(e);
        ml = prev_length;
        if (len > prev_length) { ml = len; ms = t.s - (int)(e & 0x7fffu); }
        ml = ml < lookahead ? ml : lookahead;
        if (ml == MIN_MATCH && t.s - ms > 4096) ml = MIN_MATCH - 1;           // TOO_FAR
    }
    if (prev_length >= MIN_MATCH && ml <= prev_length) {
        const uint32_t sym = (uint32_t)(prev_length - MIN_MATCH) | ((uint32_t)(t.s - 1 - prev_match) << 8) | LZ_SYM;
        t.s += prev_length - 1;
        t.avail = 0; t.ml = MIN_MATCH - 1; t.ms = 0;
        return sym;
    }
    const uint32_t lb = r >> 24;
    const uint32_t sym = t.avail ? (lb | LZ_SYM) : 0u;
    t.avail = 1; t.ml = ml; t.ms = ms;
    t.s += 1;
    return sym;
}
struct LzSeg {
    uint32_t k, j;                  // stream, segment within it
    uint64_t rp;
    int n, g, h;                    // stream length; the segment's positions [g, h)
};
__device__ __forceinline__ LzSeg lz_seg(const DeflateArgs& A, uint32_t seg) {
    LzSeg q;
    q.k = A.lz_seg[seg];
    q.j = seg - A.lz_sg0[q.k];
    q.rp = A.rp0[q.k];
    q.n = (int)A.in_len[q.k];
    q.g = (int)(q.j << A.lz_shift);
    // deflate(NO_FLUSH) steps while lookahead >= MIN_LOOKAHEAD (deflate.ts:1060-1066)
    const int nend = A.noflush ? (q.n >= MIN_LOOKAHEAD ? q.n - MIN_LOOKAHEAD + 1 : 0) : q.n;
    q.h = q.g + (1 << A.lz_shift) < nend ? q.g + (1 << A.lz_shift) : nend;
    return q;
}
__global__ __launch_bounds__(LZ_THREADS) void k_lz_spec(DeflateArgs A) {
    const uint32_t seg = blockIdx.x * LZ_THREADS + threadIdx.x;
    if (seg >= A.nlseg) return;
    const LzSeg q = lz_seg(A, seg);
    const int good = c_config[A.level][0], max_lazy = c_config[A.level][1];
    const GLB uint32_t* rec = (const GLB uint32_t*)A.rec_buf + q.rp;
    const GLB uint32_t* qrec = (const GLB uint32_t*)A.rec_buf + A.qoff + q.rp;
    GLB uint64_t* w = (GLB uint64_t*)A.lz_w + q.rp;
    GLB uint64_t* v1 = (GLB uint64_t*)A.lz_v1 + (q.rp >> 6);
    GLB uint64_t* e1 = (GLB uint64_t*)A.lz_e1 + (q.rp >> 6);
    LzSt t{q.g, MIN_MATCH - 1, 0, 0};
    uint64_t va = 0, ea = 0;
    int wc = q.g >> 6;
    auto one = [&](int s, uint32_t r) {
        for (; (s >> 6) != wc; ++wc) { v1[wc] = va; e1[wc] = ea; va = 0; ea = 0; }
        const uint32_t st = lz_pack(t);
        const uint32_t sym = lz_step(t, r, qrec, q.n, good, max_lazy);
        va |= 1ull << (s & 63);
        if (sym) ea |= 1ull << (s & 63);
        w[s] = (uint64_t)st | ((uint64_t)sym << 32);
    };
    while (t.s < q.h) {
        // two records per round trip: a step moves on by one position except after a match
        const int s = t.s;
        const uint32_t r0 = rec[s], r1 = rec[s + 1 < q.n ? s + 1 : s];
        one(s, r0);
        if (t.s == s + 1 && t.s < q.h) one(s + 1, r1);
    }
    for (; wc <= ((q.h - 1) >> 6); ++wc) { v1[wc] = va; e1[wc] = ea; va = 0; ea = 0; }
    A.lz_end[seg] = lz_save(t);
    if (q.j == 0) A.lz_c[seg] = 0;                            // the first segment's parse is the true one
}
// carry the parse t on through segment q until it meets the segment's phase-1 parse (same
// position, same state); returns that position, or q.h (t then is the state leaving the
// segment).  Writes the symbols of its steps (lz_s2, lz_e2 words [g, returned position)).
__device__ int lz_join_run(const DeflateArgs& A, const LzSeg& q, LzSt& t, int good, int max_lazy) {
    const GLB uint32_t* rec = (const GLB uint32_t*)A.rec_buf + q.rp;
    const GLB uint32_t* qrec = (const GLB uint32_t*)A.rec_buf + A.qoff + q.rp;
    const GLB uint64_t* w = (const GLB uint64_t*)A.lz_w + q.rp;
    const GLB uint64_t* v1 = (const GLB uint64_t*)A.lz_v1 + (q.rp >> 6);
    GLB uint32_t* s2 = (GLB uint32_t*)A.lz_s2 + q.rp;
    GLB uint64_t* e2 = (GLB uint64_t*)A.lz_e2 + (q.rp >> 6);
    uint64_t ea = 0;
    int wc = q.g >> 6;
    uint64_t vw = t.s < q.h ? v1[t.s >> 6] : 0ull;
    int c = q.h;
    while (t.s < q.h) {
        const int s = t.s;
        if ((s >> 6) != wc) {
            for (; (s >> 6) != wc; ++wc) { e2[wc] = ea; ea = 0; }
            vw = v1[wc];
        }
        const uint32_t r = rec[s];
        if (((vw >> (s & 63)) & 1ull) && (uint32_t)w[s] == lz_pack(t)) { c = s; break; }
        const uint32_t sym = lz_step(t, r, qrec, q.n, good, max_lazy);
        if (sym) { ea |= 1ull << (s & 63); s2[s] = sym; }
    }
    if (c > q.g)
        for (; wc <= ((c - 1) >> 6); ++wc) { e2[wc] = ea; ea = 0; }
    return c;
}
__global__ __launch_bounds__(LZ_THREADS) void k_lz_join(DeflateArgs A) {
    const uint32_t seg = blockIdx.x * LZ_THREADS + threadIdx.x;
    if (seg >= A.nlseg) return;
    const LzSeg q = lz_seg(A, seg);
    if (q.j == 0) return;
    LzSt t = lz_load(A.lz_end[seg - 1]);
    A.lz_c[seg] = (uint32_t)lz_join_run(A, q, t, c_config[A.level][0], c_config[A.level][1]);
    A.lz_carry[seg] = lz_save(t);
}
__global__ __launch_bounds__(64) void k_lz_fix(DeflateArgs A) {      // one wave per stream (as k_fz_fix)
    const uint32_t k = blockIdx.x, lane = threadIdx.x;
    if (k >= A.n || A.rp0[k] == ~0ull) return;
    const uint32_t base = A.lz_sg0[k], K = A.lz_sg0[k + 1] - base;
    if (K == 0) return;
    const int good = c_config[A.level][0], max_lazy = c_config[A.level][1];
    bool ok = true;                                            // the last segment's parse is true at its end
    LzSt t{0, 0, 0, 0};
    uint32_t j = 1;
    while (j < K) {
        uint32_t found = K;
        for (; j < K; j += 64) {
            const uint32_t jj = j + lane;
            const bool un = jj < K && (int)A.lz_c[base + jj] >= lz_seg(A, base + jj).h;
            const uint64_t m = __ballot(un);
            if (m) { found = j + (uint32_t)__builtin_ctzll(m); break; }
        }
        if (found >= K) break;
        uint32_t next = K;
        if (lane == 0) {
            t = lz_load(A.lz_carry[base + found]);             // crossed its segment: the carry is true
            ok = false;
            uint32_t jj = found + 1;
            for (; jj < K; ++jj) {
                const LzSeg q = lz_seg(A, base + jj);
                const int c = lz_join_run(A, q, t, good, max_lazy);
                A.lz_c[base + jj] = (uint32_t)c;
                if (c < q.h) { ok = true; break; }
            }
            next = jj + 1;
        }
        j = __shfl(next, 0);
    }
    if (lane == 0) {
        const LzSt f = ok ? lz_load(A.lz_end[base + K - 1]) : t;
        // deflate_slow's last literal (deflate.ts:1172) -- not under NO_FLUSH: it stays pending
        A.lz_fin[k] = A.noflush ? 0u : (uint32_t)f.avail;
        ((GLB FStream*)((GLB DSlab*)(A.state + (uint64_t)k * SLAB_BYTES))->window)->pad[0] = (uint32_t)f.s;
    }
}
// bits of word wi that belong to positions [a, b)
__device__ __forceinline__ uint64_t lz_range(int wi, int a, int b) {
    const int lo = wi << 6;
    const uint64_t ma = a <= lo ? ~0ull : a >= lo + 64 ? 0ull : ~0ull << (a - lo);
    const uint64_t mb = b >= lo + 64 ? ~0ull : b <= lo ? 0ull : ~(~0ull << (b - lo));
    return ma & mb;
}
__global__ __launch_bounds__(LZ_THREADS) void k_lz_count(DeflateArgs A) {
    const uint32_t seg = blockIdx.x * LZ_THREADS + threadIdx.x;
    if (seg >= A.nlseg) return;
    const LzSeg q = lz_seg(A, seg);
    const int c = (int)A.lz_c[seg];
    const GLB uint64_t* e1 = (const GLB uint64_t*)A.lz_e1 + (q.rp >> 6);
    const GLB uint64_t* e2 = (const GLB uint64_t*)A.lz_e2 + (q.rp >> 6);
    uint32_t cnt = 0;
    for (int wi = q.g >> 6; wi <= ((q.h - 1) >> 6); ++wi) {
        const uint64_t m2 = lz_range(wi, q.g, c), m1 = lz_range(wi, c, q.h);
        cnt += (uint32_t)__popcll((m2 ? e2[wi] : 0ull) & m2) + (uint32_t)__popcll(e1[wi] & m1);
    }
    if (seg + 1 == A.lz_sg0[q.k + 1]) cnt += A.lz_fin[q.k] & 1u;
    A.lz_cnt[seg] = cnt;
}
// one workgroup per stream: the exclusive scan of its segments' symbol counts, 256 at a time
// (a lane walking a long stream's ~1,000 segments serially took 0.3 ms of a one-buffer deflate)
#define LS_THREADS 256
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t ls_dpp_add(uint32_t x) {
    return x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, false);
}
__global__ __launch_bounds__(LS_THREADS) void k_lz_scan(DeflateArgs A) {
    __shared__ uint32_t wsum[LS_THREADS / 64];
    const uint32_t k = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    if (k >= A.n || A.rp0[k] == ~0ull) return;              // (block-uniform)
    const uint32_t s0 = A.lz_sg0[k], s1 = A.lz_sg0[k + 1];
    uint32_t o = 0;
    for (uint32_t b = s0; b < s1; b += LS_THREADS) {
        const uint32_t s = b + tid;
        const uint32_t c = s < s1 ? A.lz_cnt[s] : 0u;
        uint32_t x = c;                                     // inclusive wave scan (DPP)
        x = ls_dpp_add<0x111, 0xf>(x);
        x = ls_dpp_add<0x112, 0xf>(x);
        x = ls_dpp_add<0x114, 0xf>(x);
        x = ls_dpp_add<0x118, 0xf>(x);
        x = ls_dpp_add<0x142, 0xa>(x);
        x = ls_dpp_add<0x143, 0xc>(x);
        if (lane == 63) wsum[wv] = x;
        __syncthreads();
        uint32_t base = 0, all = 0;
#pragma unroll
        for (uint32_t w = 0; w < LS_THREADS / 64; ++w) {
            const uint32_t t = wsum[w];
            base += w < wv ? t : 0u;
            all += t;
        }
        if (s < s1) A.lz_cnt[s] = o + base + x - c;
        o += all;
        __syncthreads();                                    // (wsum is rewritten next)
    }
    if (tid == 0) {
        // (no segment: NO_FLUSH before MIN_LOOKAHEAD bytes, nothing parsed)
        const uint32_t fin = s1 > s0 ? (A.lz_fin[k] & 1u) : 0u;
        if (s1 == s0) ((GLB FStream*)((GLB DSlab*)(A.state + (uint64_t)k * SLAB_BYTES))->window)->pad[0] = 0u;
        A.lz_fin[k] = fin | (o << 1);
    }
}
// symbols to the front of the stream's record buffer (no record is read any more)
__global__ __launch_bounds__(LZ_THREADS) void k_lz_emit(DeflateArgs A) {
    const uint32_t seg = blockIdx.x * LZ_THREADS + threadIdx.x;
    if (seg >= A.nlseg) return;
    const LzSeg q = lz_seg(A, seg);
    const int c = (int)A.lz_c[seg];
    const GLB uint64_t* w = (const GLB uint64_t*)A.lz_w + q.rp;
    const GLB uint32_t* s2 = (const GLB uint32_t*)A.lz_s2 + q.rp;
    const GLB uint64_t* e1 = (const GLB uint64_t*)A.lz_e1 + (q.rp >> 6);
    const GLB uint64_t* e2 = (const GLB uint64_t*)A.lz_e2 + (q.rp >> 6);
    GLB uint32_t* sym = (GLB uint32_t*)A.sym_buf + q.rp;
    uint32_t o = A.lz_cnt[seg];
    for (int wi = q.g >> 6; wi <= ((q.h - 1) >> 6); ++wi) {
        const uint64_t m2 = lz_range(wi, q.g, c), m1 = lz_range(wi, c, q.h);
        uint64_t b2 = (m2 ? e2[wi] : 0ull) & m2, b1 = e1[wi] & m1;
        for (uint64_t b = b1 | b2; b; b &= b - 1) {
            const int p = (wi << 6) + __builtin_ctzll(b);
            const uint32_t v = p < c ? s2[p] : (uint32_t)(w[p] >> 32);
            sym[o++] = v & ~LZ_SYM;
        }
    }
    if (seg + 1 == A.lz_sg0[q.k + 1] && (A.lz_fin[q.k] & 1u))
        sym[o] = ((const GLB uint8_t*)A.in)[A.in_off[q.k] + (uint64_t)q.n - 1];
}
// block cuts: _tr_tally returns true at last_lit == 8192 when TRUNCATE_BLOCK's estimate says
// so (level > 2), and at last_lit == LIT_BUFSIZE - 1; the final literal's verdict is ignored
// (deflate.ts:1172-1176).  At a cut, strstart - block_start is the block's bytes, less the
// cutting match's length - 1 (its tally precedes strstart += prev_length - 1).
#define LB_THREADS 256                                // (batches; few streams: 1024, k_lz_blocks_t<1024>)
struct LzSums { uint32_t mat, dxb, cov, last; };
// sums over symbols [a, b): matches, extra-bit estimate, bytes covered by [a, b - 1), and by b - 1;
// the four reduced together (one pair of barriers)
template <int NT>
__device__ LzSums lb_sums(const GLB uint32_t* sym, uint32_t a, uint32_t b, uint4* red) {
    uint32_t mat = 0, dxb = 0, cov = 0, last = 0;
    for (uint32_t i = a + threadIdx.x; i < b; i += NT) {
        const uint32_t v = sym[i], dist = v >> 8;
        const uint32_t len = dist ? (v & 255u) + MIN_MATCH : 1u;
        if (dist) {
            const uint32_t d = dist - 1;
            mat += 1;
            dxb += 5u + (d < 4u ? 0u : 30u - (uint32_t)__builtin_clz(d));
        }
        if (i + 1 < b) cov += len;
        else last = len;
    }
    for (int o = 32; o > 0; o >>= 1) {
        mat += __shfl_xor(mat, o);
        dxb += __shfl_xor(dxb, o);
        cov += __shfl_xor(cov, o);
        last += __shfl_xor(last, o);
    }
    const uint32_t wv = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[wv] = make_uint4(mat, dxb, cov, last);
    __syncthreads();
    LzSums r{0, 0, 0, 0};
#pragma unroll
    for (uint32_t i = 0; i < NT / 64; ++i) {
        const uint4 t = red[i];
        r.mat += t.x; r.dxb += t.y; r.cov += t.z; r.last += t.w;
    }
    return r;
}
template <int NT>
__global__ __launch_bounds__(NT) void k_lz_blocks_t(DeflateArgs A) {
    __shared__ uint4 red[NT / 64];
    const uint32_t sid = blockIdx.x;
    if (sid >= A.n) return;
    GLB DSlab* S = (GLB DSlab*)(A.state + (uint64_t)sid * SLAB_BYTES);
    GLB FStream* F = (GLB FStream*)S->window;
    const uint64_t in_len = A.in_len[sid];
    if (in_len == 0 || A.rp0[sid] == ~0ull) {
        if (threadIdx.x == 0) { F->nblk = 0; F->flag = 1; }
        return;
    }
    if (A.lz_act && (A.lz_act[sid] & 1u)) {                    // fast levels: not settled, serial kernel
        if (threadIdx.x == 0) { F->nblk = 0; F->flag = 1; }
        return;
    }
    const int64_t n = (int64_t)in_len;
    // deflate_slow tallies a literal or match one step after its position (the cutting step is
    // one past the bytes before it), deflate_fast at it; TRUNCATE_BLOCK only above level 2
    const int64_t plus = A.level >= 4 ? 1 : 0;
    const bool trunc = A.level > 2;
    const uint32_t fin = A.lz_fin[sid], nsym = fin >> 1, nchk = nsym - (fin & 1u);
    const GLB uint32_t* sym = (const GLB uint32_t*)A.sym_buf + A.rp0[sid];
    GLB uint8_t* slots = (GLB uint8_t*)(A.blk + (uint64_t)A.tb0[sid] * FB_SLOT);
    const uint32_t nbcap = A.tb0[sid + 1] - A.tb0[sid];
    uint32_t nb = 0, b0 = 0;
    int64_t block_start = 0;
    for (;;) {
        uint32_t cnt = 0, eof = 0;
        int64_t step = n, strstart = n;                        // the cutting step's position; strstart after it
        if (b0 + 8192 <= nchk) {
            const LzSums a = lb_sums<NT>(sym, b0, b0 + 8192, red);
            const int64_t in_length = a.cov + plus;
            const uint32_t out_length = (8192u * 8u + a.dxb) >> 3;
            if (trunc && a.mat < 4096 && (int64_t)out_length < in_length / 2) {
                cnt = 8192;
                step = block_start + in_length;
                strstart = block_start + a.cov + a.last;
            } else if (b0 + LIT_BUFSIZE - 1 <= nchk) {
                const LzSums b = lb_sums<NT>(sym, b0 + 8192, b0 + LIT_BUFSIZE - 1, red);
                cnt = LIT_BUFSIZE - 1;
                const int64_t before = (int64_t)a.cov + a.last + b.cov;   // symbols [b0, b0 + 16382)
                step = block_start + before + plus;
                strstart = block_start + before + b.last;
            }
        }
        if (cnt == 0) {
            if (A.noflush) break;                              // the open block stays pending
            cnt = nsym - b0; eof = 1;
        }
        if (threadIdx.x == 0 && nb < nbcap) {
            const int64_t off = slide_off(n, step);
            GLB FBlock* B = (GLB FBlock*)(slots + (uint64_t)nb * FB_SLOT);
            B->sym0 = b0; B->nsym = cnt;
            B->block_start = (int32_t)(block_start - off); B->strstart = (int32_t)(strstart - off);
            B->off = off; B->eof = eof;
        }
        nb++;
        b0 += cnt;
        block_start = strstart;
        if (eof) break;
    }
    if (threadIdx.x == 0) {
        F->nblk = nb;
        F->flag = nb > nbcap ? 1u : 0u;
    }
}

// ------------------------------------------------------------------ fast levels on the record path
// deflate_fast (deflate.ts:953-1049) inserts the string at every step with lookahead >=
// MIN_MATCH and at the positions inside a match of at most max_lazy_match bytes, but not inside
// longer matches: its hash chains depend on its own parse.  The positions it inserts are the
// unique fixed point of  I -> the parse whose searches walk the chains of I -> the positions
// that parse inserts  (a step at s reads I below s only, so by induction over positions any
// fixed point is the reference's), and iterating from I = every position reaches it: a round
// settles at least everything before the first difference, and the changes of a round are
// local (10-50 rounds on text, each touching fewer positions).  A round: k_fz_match (every
// position's search on the links of k_dfl_chain, stepping over positions outside I),
// the segment-parallel parse of k_lz_* with the step position as its whole state
// (k_fz_spec / k_fz_join / k_fz_fix), k_fz_merge (the next I, and whether it changed) and
// k_fz_roll (streams whose I did not change are settled and leave the rounds).  The symbols of
// their last round then take the slow levels' way (k_lz_count / scan / emit / blocks).
__device__ __forceinline__ bool fz_in(const GLB uint64_t* I, int64_t q) { return (I[q >> 6] >> (q & 63)) & 1ull; }
// bits of one bitmap set in increasing position order, words written as they are left behind
struct BitW {
    GLB uint64_t* dst;
    int wc;
    uint64_t acc;
    __device__ void to(int p) { for (; (p >> 6) != wc; ++wc) { dst[wc] = acc; acc = 0; } }
    __device__ void set(int p) { to(p); acc |= 1ull << (p & 63); }
    __device__ void end(int g, int e) {                      // write the words up to position e - 1
        if (e > g)
            for (; wc <= ((e - 1) >> 6); ++wc) { dst[wc] = acc; acc = 0; }
    }
};
// common prefix of in[a ..] and in[b ..] (a < b, b + MAX_MATCH <= input length), <= MAX_MATCH
__device__ __forceinline__ int fz_len(const GLB uint8_t* in, int a, int b) {
    int l = 0;
    for (; l < MAX_MATCH - 2; l += 4) {
        uint32_t x, y;
        __builtin_memcpy(&x, (const uint8_t*)(in + a + l), 4);
        __builtin_memcpy(&y, (const uint8_t*)(in + b + l), 4);
        if (x ^ y) return l + (int)(__builtin_ctz(x ^ y) >> 3);
    }
    while (l < MAX_MATCH && in[a + l] == in[b + l]) ++l;
    return l;
}
// the previous position of I on q's hash chain above `lo` (0: none)
__device__ __forceinline__ int fz_prev(const GLB uint16_t* pv, const GLB uint64_t* I, int q, int lo) {
    for (;;) {
        const uint32_t d = pv[q];
        q -= (int)d;
        if (!d || q <= lo) return 0;
        if (fz_in(I, q)) return q;
    }
}
// longest_match (deflate.ts:827-946) as deflate_fast calls it at P (best_len from
// MIN_MATCH - 1, every candidate of the chain of I counted) with P + MIN_LOOKAHEAD <= n: only
// input bytes are read.  Record: len << 16 | dist, 0 below MIN_MATCH.
__device__ uint32_t fz_search(const GLB uint8_t* in, const GLB uint16_t* pv, const GLB uint64_t* I, int P, int chain,
                              int nice) {
    // hash_head: not 0, within MAX_DIST (deflate.ts:986); the walk continues above limit
    int cur = fz_prev(pv, I, P, P > MAX_DIST ? P - MAX_DIST - 1 : 0);
    if (cur == 0) return 0u;
    const int limit = P > MAX_DIST ? P - MAX_DIST : 0;
    int best = MIN_MATCH - 1, bpos = 0;
    for (;;) {
        const int len = fz_len(in, cur, P);
        if (len > best) {
            best = len; bpos = cur;
            if (len >= nice) break;
        }
        if (--chain == 0) break;
        cur = fz_prev(pv, I, cur, limit);
        if (cur == 0) break;
    }
    return best >= MIN_MATCH ? ((uint32_t)best << 16) | (uint32_t)(P - bpos) : 0u;
}
// the same for the last positions (lookahead < MIN_LOOKAHEAD), in the window the reference
// has there (stale bytes past the input: see tail_search)
__device__ uint32_t fz_tail(const GLB uint8_t* in, const GLB uint16_t* pv, const GLB uint64_t* I, int64_t n, int64_t P,
                            int chain_length, int nice) {
    const int64_t off = slide_off(n, P);
    const int strstart = (int)(P - off);
    auto prev_of = [&](int64_t q, int lo) -> int {       // window index of the previous position of I above lo
        for (;;) {
            const uint32_t d = pv[q];
            q -= (int64_t)d;
            if (!d || q - off <= lo) return 0;
            if (fz_in(I, q)) return (int)(q - off);
        }
    };
    auto wb = [&](int i) -> uint32_t { return win_byte(in, n, off, i); };
    int cur = prev_of(P, strstart > MAX_DIST ? strstart - MAX_DIST - 1 : 0);
    if (cur == 0) return 0u;
    const int lookahead = (int)(n - P);
    if (nice > lookahead) nice = lookahead;
    const int limit = strstart > MAX_DIST ? strstart - MAX_DIST : 0;
    int best = MIN_MATCH - 1, bstart = 0;
    uint32_t scan_end1 = wb(strstart + best - 1), scan_end = wb(strstart + best);
    const uint32_t c0 = wb(strstart), c1 = wb(strstart + 1);
    do {
        const int match = cur;
        const int nx = prev_of(match + off, limit);
        const uint32_t e0 = wb(match + best), e1 = wb(match + best - 1);
        const uint32_t m0 = wb(match), m1 = wb(match + 1);
        if ((e0 == scan_end) & (e1 == scan_end1) & (m0 == c0) & (m1 == c1)) {
            int len = 3;                      // byte 2 is not compared (equal hash, deflate.ts:891-897)
            while (len < MAX_MATCH && wb(strstart + len) == wb(match + len)) ++len;
            if (len > best) {
                bstart = match;
                best = len;
                if (len >= nice) break;
                scan_end1 = wb(strstart + best - 1);
                scan_end = wb(strstart + best);
            }
        }
        cur = nx;
    } while (cur > limit && --chain_length != 0);
    if (best > lookahead) best = lookahead;
    return best >= MIN_MATCH ? ((uint32_t)best << 16) | (uint32_t)(strstart - bstart) : 0u;
}
__global__ __launch_bounds__(256) void k_fz_init(DeflateArgs A) {     // I = every position with lookahead >= 3
    const uint32_t seg = blockIdx.x * 256 + threadIdx.x;
    if (seg >= A.nlseg) return;
    const LzSeg q = lz_seg(A, seg);
    GLB uint64_t* I = (GLB uint64_t*)A.lz_i + (q.rp >> 6);
    for (int wi = q.g >> 6; wi <= ((q.h - 1) >> 6); ++wi) I[wi] = lz_range(wi, q.g, q.n - MIN_MATCH + 1);
    A.fz_rc[seg] = 0; A.fz_chg[seg] = 0; A.fz_fx[seg] = 0;
    if (q.j == 0) A.lz_act[q.k] = 1u;
}
// A round recomputes only what the last round's changes of I can reach: a segment's
// searches read I over the 32 KiB before it, its parse reads its own records, a join its own
// and the previous segment's parse.
__global__ __launch_bounds__(256) void k_fz_match(DeflateArgs A) {
    __shared__ int any;
    const uint32_t seg = blockIdx.x;
    if (seg >= A.nlseg) return;
    const LzSeg q = lz_seg(A, seg);
    if (!(A.lz_act[q.k] & 1u)) return;
    if (A.lz_round > 1) {
        if (threadIdx.x == 0) any = 0;
        __syncthreads();
        const uint32_t w = ((uint32_t)(W_SIZE + MAX_MATCH) >> A.lz_shift) + 1u;
        const uint32_t j0 = q.j > w ? q.j - w : 0u;
        for (uint32_t jj = j0 + threadIdx.x; jj <= q.j; jj += blockDim.x)
            if (A.fz_chg[seg - q.j + jj] == A.lz_round - 1) any = 1;
        __syncthreads();
        if (!any) return;
    }
    if (threadIdx.x == 0) A.fz_rc[seg] = A.lz_round;
    const GLB uint8_t* in = (const GLB uint8_t*)(A.in + A.in_off[q.k]);
    const GLB uint16_t* pv = (const GLB uint16_t*)A.pv_buf + q.rp;
    const GLB uint64_t* I = (const GLB uint64_t*)A.lz_i + (q.rp >> 6);
    GLB uint32_t* rec = (GLB uint32_t*)A.rec_buf + q.rp;       // (the slow levels' layout: u32 at rp0 + p)
    const int nice = c_config[A.level][2], chain = c_config[A.level][3];
    for (int p = q.g + (int)threadIdx.x; p < q.h; p += (int)blockDim.x) {
        uint32_t r = 0;
        if (q.n - p >= MIN_MATCH)
            r = p + MIN_LOOKAHEAD <= q.n ? fz_search(in, pv, I, p, chain, nice) : fz_tail(in, pv, I, q.n, p, chain, nice);
        rec[p] = r;
    }
}
// one deflate_fast step at s (deflate.ts:974-1033): its symbol, the positions it inserts
// (I.set), the next step position; *iin: the positions inside its match are inserted
__device__ __forceinline__ uint32_t fz_step(int& s, uint32_t r, uint32_t lit, int n, int max_ins, BitW& I, bool& iin) {
    const int lookahead = n - s;
    if (lookahead >= MIN_MATCH) I.set(s);
    const int len = (int)(r >> 16);
    if (len >= MIN_MATCH) {
        iin = len <= max_ins && lookahead - len >= MIN_MATCH;
        if (iin)
            for (int i = 1; i < len; ++i) I.set(s + i);
        const uint32_t sym = (uint32_t)(len - MIN_MATCH) | ((r & 0xffffu) << 8) | LZ_SYM;
        s += len;
        return sym;
    }
    iin = false;
    s += 1;
    return lit | LZ_SYM;
}
__global__ __launch_bounds__(LZ_THREADS) void k_fz_spec(DeflateArgs A) {
    const uint32_t seg = blockIdx.x * LZ_THREADS + threadIdx.x;
    if (seg >= A.nlseg) return;
    const LzSeg q = lz_seg(A, seg);
    if (!(A.lz_act[q.k] & 1u) || A.fz_rc[seg] != A.lz_round) return;
    const GLB uint8_t* in = (const GLB uint8_t*)(A.in + A.in_off[q.k]);
    const GLB uint32_t* rec = (const GLB uint32_t*)A.rec_buf + q.rp;
    GLB uint64_t* w = (GLB uint64_t*)A.lz_w + q.rp;
    const int max_ins = c_config[A.level][1];
    BitW V{(GLB uint64_t*)A.lz_v1 + (q.rp >> 6), q.g >> 6, 0};
    BitW I{(GLB uint64_t*)A.lz_i1 + (q.rp >> 6), q.g >> 6, 0};
    int s = q.g;
    bool iin = false;
    // records and bytes of 4 positions per round trip: a literal moves on by one
    int wb0 = -0x40000000;
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, lw = 0;
    while (s < q.h) {
        const int p = s;
        if (p - wb0 >= 4) {
            wb0 = p;
            const int last = q.n - 1;
            r0 = rec[p];
            r1 = rec[p + 1 < last ? p + 1 : last];
            r2 = rec[p + 2 < last ? p + 2 : last];
            r3 = rec[p + 3 < last ? p + 3 : last];
            if (p + 4 <= q.n) __builtin_memcpy(&lw, (const uint8_t*)(in + p), 4);
            else {
                lw = 0;
                for (int i = 0; p + i < q.n; ++i) lw |= (uint32_t)in[p + i] << (8 * i);
            }
        }
        const int o = p - wb0;
        const uint32_t r = o == 0 ? r0 : o == 1 ? r1 : o == 2 ? r2 : r3;
        V.set(p);
        const uint32_t sym = fz_step(s, r, (lw >> (8 * o)) & 255u, q.n, max_ins, I, iin);
        w[p] = (uint64_t)sym << 32;
    }
    // (interior bits past h belong to the next segment's join: BitW.end stops at h)
    I.acc &= (I.wc << 6) + 64 <= q.h ? ~0ull : lz_range(I.wc, q.g, q.h);
    V.end(q.g, q.h);
    I.end(q.g, q.h);
    A.lz_end[seg] = (uint64_t)(uint32_t)s | ((uint64_t)(iin ? 1u : 0u) << 32);
    if (q.j == 0) A.lz_c[seg] = 0;
}
// carry the parse at s on through segment q until it stands on a step position of the
// segment's own parse (the step position is the whole state); positions [g, s) lie inside the
// match crossing in (inserted iff cin).  Returns the meeting position or q.h.
__device__ int fz_join_run(const DeflateArgs& A, const LzSeg& q, int& s, bool& cin, int max_ins) {
    const GLB uint8_t* in = (const GLB uint8_t*)(A.in + A.in_off[q.k]);
    const GLB uint32_t* rec = (const GLB uint32_t*)A.rec_buf + q.rp;
    const GLB uint64_t* v1 = (const GLB uint64_t*)A.lz_v1 + (q.rp >> 6);
    GLB uint32_t* s2 = (GLB uint32_t*)A.lz_s2 + q.rp;
    BitW E{(GLB uint64_t*)A.lz_e2 + (q.rp >> 6), q.g >> 6, 0};
    BitW I{(GLB uint64_t*)A.lz_i2 + (q.rp >> 6), q.g >> 6, 0};
    if (cin)
        for (int p = q.g; p < s && p < q.h; ++p) I.set(p);
    int c = q.h, vwc = -1;
    uint64_t vw = 0;
    while (s < q.h) {
        if ((s >> 6) != vwc) { vwc = s >> 6; vw = v1[vwc]; }
        if ((vw >> (s & 63)) & 1ull) { c = s; break; }
        const int p = s;
        const uint32_t r = rec[p];
        E.set(p);
        s2[p] = fz_step(s, r, in[p], q.n, max_ins, I, cin);
    }
    if (c == q.h) I.acc &= (I.wc << 6) + 64 <= q.h ? ~0ull : lz_range(I.wc, q.g, q.h);
    E.end(q.g, c);
    I.end(q.g, c);
    return c;
}
__global__ __launch_bounds__(LZ_THREADS) void k_fz_join(DeflateArgs A) {
    const uint32_t seg = blockIdx.x * LZ_THREADS + threadIdx.x;
    if (seg >= A.nlseg) return;
    const LzSeg q = lz_seg(A, seg);
    if (q.j == 0 || !(A.lz_act[q.k] & 1u)) return;
    if (A.fz_rc[seg] != A.lz_round && A.fz_rc[seg - 1] != A.lz_round) return;
    const uint64_t e = A.lz_end[seg - 1];
    int s = (int)(uint32_t)e;
    bool cin = (e >> 32) != 0;
    A.lz_c[seg] = (uint32_t)fz_join_run(A, q, s, cin, c_config[A.level][1]);
    A.lz_carry[seg] = (uint64_t)(uint32_t)s | ((uint64_t)(cin ? 1u : 0u) << 32);
}
// one wave per stream: the boundaries whose join crossed its segment are found 64 at a time;
// from each, lane 0 redoes the following joins until one meets its segment's parse
__global__ __launch_bounds__(64) void k_fz_fix(DeflateArgs A) {
    const uint32_t k = blockIdx.x, lane = threadIdx.x;
    if (k >= A.n || A.rp0[k] == ~0ull || !(A.lz_act[k] & 1u)) return;
    const uint32_t base = A.lz_sg0[k], K = A.lz_sg0[k + 1] - base;
    const int max_ins = c_config[A.level][1];
    bool fok = true;                                            // (lane 0) the last chain met its segment
    int fs = 0;                                                 // (lane 0) else where it ended
    uint32_t j = 1;
    while (j < K) {
        uint32_t found = K;
        for (; j < K; j += 64) {
            const uint32_t jj = j + lane;
            const bool un = jj < K && (int)A.lz_c[base + jj] >= lz_seg(A, base + jj).h;
            const uint64_t m = __ballot(un);
            if (m) { found = j + (uint32_t)__builtin_ctzll(m); break; }
        }
        if (found >= K) break;
        uint32_t next = K;
        if (lane == 0) {
            const uint64_t e = A.lz_carry[base + found];
            int s = (int)(uint32_t)e;
            bool cin = (e >> 32) != 0;
            uint32_t jj = found + 1;
            fs = s;
            fok = false;
            for (; jj < K; ++jj) {
                const LzSeg q = lz_seg(A, base + jj);
                const int c = fz_join_run(A, q, s, cin, max_ins);
                A.lz_c[base + jj] = (uint32_t)c;
                A.fz_fx[base + jj] = A.lz_round;
                if (c < q.h) { fok = true; break; }
            }
            fs = s;
            next = jj + 1;
        }
        j = __shfl(next, 0);
    }
    if (lane == 0) {
        A.lz_fin[k] = 0;                                        // deflate_fast leaves no pending literal
        const int f = fok && K ? (int)(uint32_t)A.lz_end[base + K - 1] : fs;
        ((GLB FStream*)((GLB DSlab*)(A.state + (uint64_t)k * SLAB_BYTES))->window)->pad[0] = (uint32_t)f;
    }
}
// the next I of each segment ([g, c) from the join, [c, h) from its own parse); a stream
// whose I changed anywhere goes another round
__global__ __launch_bounds__(LZ_THREADS) void k_fz_merge(DeflateArgs A) {
    const uint32_t seg = blockIdx.x * LZ_THREADS + threadIdx.x;
    if (seg == 0) *A.lz_nact = 0;                          // k_fz_roll counts into it next (no memset launch)
    if (seg >= A.nlseg) return;
    const LzSeg q = lz_seg(A, seg);
    if (!(A.lz_act[q.k] & 1u)) return;
    if (A.fz_rc[seg] != A.lz_round && (q.j == 0 || A.fz_rc[seg - 1] != A.lz_round) && A.fz_fx[seg] != A.lz_round)
        return;
    const int c = (int)A.lz_c[seg];
    GLB uint64_t* I = (GLB uint64_t*)A.lz_i + (q.rp >> 6);
    const GLB uint64_t* i1 = (const GLB uint64_t*)A.lz_i1 + (q.rp >> 6);
    const GLB uint64_t* i2 = (const GLB uint64_t*)A.lz_i2 + (q.rp >> 6);
    bool changed = false;
    for (int wi = q.g >> 6; wi <= ((q.h - 1) >> 6); ++wi) {
        const uint64_t m2 = lz_range(wi, q.g, c), m1 = lz_range(wi, c, q.h);
        const uint64_t nw = ((m2 ? i2[wi] : 0ull) & m2) | (i1[wi] & m1);
        if (nw != I[wi]) { changed = true; I[wi] = nw; }
    }
    if (changed) {
        A.fz_chg[seg] = A.lz_round;
        atomicOr(&A.lz_act[q.k], 2u);
    }
}
__global__ __launch_bounds__(256) void k_fz_roll(DeflateArgs A) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= A.n) return;
    const uint32_t a = A.lz_act[k];
    if (!(a & 1u)) return;
    A.lz_act[k] = (a >> 1) & 1u;
    if (a & 2u) atomicAdd(A.lz_nact, 1u);
}

// tree context of the record path: LDS arrays, header bits into LDS words
struct LTreeCtx {
    uint16_t *heap, *depth, *bl_count, *next_code, *bltree;
    int heap_len, heap_max, opt_len, static_len;
    uint32_t* hdr;
    uint32_t nb;
    __device__ void bits(uint32_t v, int len) {
        const uint32_t w = nb >> 5, sh = nb & 31;
        hdr[w] |= v << sh;
        if (sh + (uint32_t)len > 32) hdr[w + 1] |= v >> (32 - sh);
        nb += (uint32_t)len;
    }
};

#ifndef DT_WAVE
#define DT_WAVE 1                         // wave-cooperative k_dfl_trees (round 5; 0: lane 0 alone)
#endif
#if DT_WAVE
// k_dfl_trees, wave-cooperative: the same trees and header as _tr_flush_block
// (deftree.ts:190-267 build_tree, 60-132 gen_bitlen, 155-182 gen_codes, deflate.ts:267-429
// scan_tree / send_tree), with only the heap (pqdownheap and the merge loop, whose tie
// order decides the code lengths) left to one lane.  A lone lane pays the full LDS or HBM
// latency on every dependent access, so everything that is not the heap is spread over the
// wave or kept in registers:
// - the heap holds packed keys freq << 16 | depth << 10 | node, so smaller() (deftree.ts /
//   deflate.ts:233-238: freq, then depth, ties taken as "smaller") is one compare of key >> 10
//   with no indirection through tree[] and depth[], and both children come in one 8-byte load;
// - gen_bitlen: every node's depth below the root by chasing its parent links, all lanes at
//   once; Len = min(depth, max_length) and overflow = #nodes deeper than max_length are what
//   the reference's top-down loop computes (Len[dad] is already clamped there); the overflow
//   repair (rare) is the reference's loop on lane 0;
// - gen_codes: next_code[len] plus the symbol's rank among the same-length symbols below it
//   (ballots), as the reference's in-order next_code[len]++;
// - scan_tree / send_tree: the code lengths read 64 at a time into a register and taken
//   lane by lane (readlane), the bit-length counts in a lane-indexed register, the header
//   bits in a register accumulator stored a word at a time;
// - the static trees and extra-bit tables are staged in LDS (global loads of a lone lane
//   were most of this kernel's time on a one-block call: 149 us on simple.txt).
#define DT_NODE_BITS 10                   // node ids < 573
#ifdef DT_PROF                            // development: phase clocks of the first (stream, block), printf
#define DT_T(a, k) do { if (a) (a)[k] = wall_clock64(); } while (0)
#else
#define DT_T(a, k) do { } while (0)
#endif
#define DT_KEY(f, d, n) (((uint32_t)(f) << 16) | ((uint32_t)(d) << DT_NODE_BITS) | (uint32_t)(n))
struct WTree {
    uint16_t* order;                      // the reference's heap[heap_max..HEAP_SIZE-1]: node order
    uint32_t* hk;                         // heap of packed keys, [1..heap_len] (8-byte aligned)
    uint32_t* blc;                        // bl_count[0..15]
    int* xch;                             // lane 0 -> wave
    int opt_len, static_len;              // wave-uniform
};
__device__ __forceinline__ int dt_rdl(uint32_t v, int i) { return __builtin_amdgcn_readlane((int)v, i); }
__device__ __forceinline__ int dt_sum(int v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ void dt_down(uint32_t* hk, int len, int k) {   // pqdownheap, deflate.ts:241-263
    const uint32_t v = hk[k];
    int j = k << 1;
    while (j <= len) {
        const uint2 ab = *(const uint2*)(hk + j);                  // j even: both children
        uint32_t c = ab.x;
        if (j < len && (ab.y >> DT_NODE_BITS) <= (ab.x >> DT_NODE_BITS)) { c = ab.y; j++; }
        if ((v >> DT_NODE_BITS) <= (c >> DT_NODE_BITS)) break;
        hk[k] = c;
        k = j;
        j <<= 1;
    }
    hk[k] = v;
}
#ifndef DT_RHEAP
#define DT_RHEAP 1                        // heaps of <= 62 entries in one register (0: all in LDS)
#endif
// A heap of at most 62 entries in one register: entry i at lane i, read with readlane at a
// wave-uniform index and written with a lane compare and select; the compares run on scalars.
// In LDS each level of a pqdownheap is a dependent load (23 us of a one-block call's ~25-leaf
// heap, DT_PROF); a 5-register heap for all sizes (the index's register picked by a switch)
// measured twice as slow as LDS: its branches cost more than the loads.
__device__ __forceinline__ void dt_down_1(int& H, int len, int k) {   // pqdownheap, deflate.ts:241-263
    const int me = (int)threadIdx.x;
    const uint32_t v = (uint32_t)__builtin_amdgcn_readlane(H, k);
    int j = k << 1;
    while (j <= len) {
        uint32_t c = (uint32_t)__builtin_amdgcn_readlane(H, j);
        if (j < len) {
            const uint32_t c1 = (uint32_t)__builtin_amdgcn_readlane(H, j + 1);
            if ((c1 >> DT_NODE_BITS) <= (c >> DT_NODE_BITS)) { c = c1; j++; }
        }
        if ((v >> DT_NODE_BITS) <= (c >> DT_NODE_BITS)) break;
        H = me == k ? (int)c : H;
        k = j;
        j <<= 1;
    }
    H = me == k ? (int)v : H;
}
// build_tree (deftree.ts:190-267) with gen_bitlen and gen_codes; returns max_code.  tree:
// LDS, tsize entries; stree: the static tree (LDS) or null; called by the whole wave.
__device__ int dt_build(WTree& W, uint16_t* tree, const uint16_t* stree, const uint8_t* extra, int base,
                        int elems, int max_length, uint64_t* tp = nullptr) {
    const uint32_t lane = threadIdx.x;
    const uint64_t below = (1ull << lane) - 1ull;
    int heap_len = 0, max_code = -1;
    for (int cb = 0; cb < elems; cb += 64) {                      // the leaves in symbol order
        const int n = cb + (int)lane;
        const uint32_t f = n < elems ? tree[n * 2] : 0u;
        const uint64_t m = __ballot(f != 0);
        if (f) W.hk[heap_len + 1 + (int)__popcll(m & below)] = DT_KEY(f, 0, n);
        else if (n < elems) tree[n * 2 + 1] = 0;
        heap_len += (int)__popcll(m);
        if (m) max_code = cb + 63 - (int)__clzll(m);
    }
    while (heap_len < 2) {                                        // at least two codes
        const int node = max_code < 2 ? ++max_code : 0;
        ++heap_len;
        if (lane == 0) { W.hk[heap_len] = DT_KEY(1, 0, node); tree[node * 2] = 1; }
        W.opt_len--;
        if (stree) W.static_len -= stree[node * 2 + 1];
    }
    const int nodes = 2 * heap_len - 1, hmax = HEAP_SIZE - nodes;
    __syncthreads();
    DT_T(tp, 0);
#if DT_RHEAP
    if (heap_len <= 62) {
        int H = (int)W.hk[lane];
        int len = heap_len, node = elems, hm = HEAP_SIZE;
        for (int k = len / 2; k >= 1; --k) dt_down_1(H, len, k);
        do {
            const uint32_t a = (uint32_t)__builtin_amdgcn_readlane(H, 1);
            const int tl = __builtin_amdgcn_readlane(H, len--);
            H = lane == 1 ? tl : H;
            dt_down_1(H, len, 1);
            const uint32_t b = (uint32_t)__builtin_amdgcn_readlane(H, 1);
            const uint32_t na = a & 1023u, nb = b & 1023u;
            hm -= 2;
            const uint32_t da = (a >> DT_NODE_BITS) & 63u, db = (b >> DT_NODE_BITS) & 63u;
            const uint32_t f = (a >> 16) + (b >> 16);
            if (lane == 0) {
                W.order[hm + 1] = (uint16_t)na;
                W.order[hm] = (uint16_t)nb;
                tree[node * 2] = (uint16_t)f;
                tree[na * 2 + 1] = tree[nb * 2 + 1] = (uint16_t)node;   // Dad
            }
            H = lane == 1 ? (int)DT_KEY(f, (da > db ? da : db) + 1u, node) : H;
            node++;
            dt_down_1(H, len, 1);
        } while (len >= 2);
        if (lane == 0) W.order[hm - 1] = (uint16_t)((uint32_t)__builtin_amdgcn_readlane(H, 1) & 1023u);
    } else
#endif
    if (lane == 0) {
        int len = heap_len, node = elems, hm = HEAP_SIZE;
        for (int k = len / 2; k >= 1; --k) dt_down(W.hk, len, k);
        do {
            const uint32_t a = W.hk[1];
            W.hk[1] = W.hk[len--];
            dt_down(W.hk, len, 1);
            const uint32_t b = W.hk[1];
            const uint32_t na = a & 1023u, nb = b & 1023u;
            W.order[--hm] = (uint16_t)na;
            W.order[--hm] = (uint16_t)nb;
            const uint32_t da = (a >> DT_NODE_BITS) & 63u, db = (b >> DT_NODE_BITS) & 63u;
            const uint32_t f = (a >> 16) + (b >> 16);
            tree[node * 2] = (uint16_t)f;
            tree[na * 2 + 1] = tree[nb * 2 + 1] = (uint16_t)node;       // Dad
            W.hk[1] = DT_KEY(f, (da > db ? da : db) + 1u, node);
            node++;
            dt_down(W.hk, len, 1);
        } while (len >= 2);
        W.order[--hm] = (uint16_t)(W.hk[1] & 1023u);
    }
    __syncthreads();
    DT_T(tp, 1);
    // gen_bitlen: depths below the root, then Len, bl_count, opt_len, static_len
    const int root = W.order[hmax];
    if (lane < 16) W.blc[lane] = 0;
    constexpr int NC = (HEAP_SIZE + 63) / 64;
    int nd[NC], dp[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int h = hmax + 1 + c * 64 + (int)lane;
        nd[c] = h < HEAP_SIZE ? W.order[h] : root;
        dp[c] = 0;
    }
    {
        int x[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) x[c] = nd[c];
        for (;;) {
            bool live = false;
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (x[c] != root) { x[c] = tree[x[c] * 2 + 1]; dp[c]++; live = true; }
            if (!__ballot(live)) break;
        }
    }
    __syncthreads();                                              // every chase done before Len
    DT_T(tp, 2);
    int ovf = 0, opt = 0, stl = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int h = hmax + 1 + c * 64 + (int)lane;
        if (h < HEAP_SIZE) {
            const int n = nd[c], bits = dp[c] > max_length ? max_length : dp[c];
            ovf += dp[c] > max_length;
            tree[n * 2 + 1] = (uint16_t)bits;
            if (n <= max_code) {
                atomicAdd(&W.blc[bits], 1u);
                const int xb = n >= base ? extra[n - base] : 0, f = tree[n * 2];
                opt += f * (bits + xb);
                if (stree) stl += f * (stree[n * 2 + 1] + xb);
            }
        }
    }
    if (lane == 0) tree[root * 2 + 1] = 0;
    const int overflow = dt_sum(ovf);
    W.opt_len += dt_sum(opt);
    W.static_len += dt_sum(stl);
    __syncthreads();
    if (overflow) {                                               // deftree.ts:98-131, as written
        if (lane == 0) {
            int ov = overflow, bits, d = 0;
            do {
                bits = max_length - 1;
                while (W.blc[bits] == 0) bits--;
                W.blc[bits]--;
                W.blc[bits + 1] += 2;
                W.blc[max_length]--;
                ov -= 2;
            } while (ov > 0);
            int h = HEAP_SIZE;
            for (bits = max_length; bits != 0; bits--) {
                int k = (int)W.blc[bits];
                while (k != 0) {
                    const int m = W.order[--h];
                    if (m > max_code) continue;
                    const int t = tree[m * 2 + 1];
                    if (t != bits) { d += (bits - t) * (int)tree[m * 2]; tree[m * 2 + 1] = (uint16_t)bits; }
                    k--;
                }
            }
            *W.xch = d;
        }
        __syncthreads();
        W.opt_len += *W.xch;
        __syncthreads();
    }
    DT_T(tp, 3);
    // gen_codes: lane L holds next_code[L]
    const uint32_t blc = lane < 16 ? W.blc[lane] : 0u;
    uint32_t ncv = 0, code = 0;
    for (int b = 1; b <= max_length; ++b) {
        code = (code + (uint32_t)dt_rdl(blc, b - 1)) << 1;
        if ((int)lane == b) ncv = code;
    }
    for (int cb = 0; cb <= max_code; cb += 64) {
        const int n = cb + (int)lane;
        const int len = n <= max_code ? tree[n * 2 + 1] : 0;
        uint32_t cd = 0;
        for (int L = 1; L <= max_length; ++L) {
            const uint64_t m = __ballot(len == L);
            if (!m) continue;
            const uint32_t b0 = (uint32_t)dt_rdl(ncv, L);
            if (len == L) cd = b0 + (uint32_t)__popcll(m & below);
            if ((int)lane == L) ncv += (uint32_t)__popcll(m);
        }
        if (len) tree[n * 2] = (uint16_t)bitrev_n(cd, len);
    }
    __syncthreads();
    DT_T(tp, 4);
    return max_code;
}
// the code lengths tree[0..max_code + 1] (with the guard), 64 at a time: lenat(i), i ascending
struct DtLens {
    const uint16_t* tree;
    int tsize, c = -1;
    uint32_t v = 0;
    __device__ int at(int i) {
        const int k = i >> 6;
        if (k != c) {
            c = k;
            const int j = (k * 64 + (int)threadIdx.x) * 2 + 1;
            v = j < tsize ? tree[j] : 0u;
        }
        return dt_rdl(v, i & 63);
    }
};
// scan_tree (deflate.ts:267-312): the bit-length counts into blv (lane j: code j)
__device__ void dt_scan(uint16_t* tree, int tsize, int max_code, uint32_t& blv) {
    const uint32_t lane = threadIdx.x;
    if (lane == 0) tree[(max_code + 1) * 2 + 1] = 0xffff;
    __syncthreads();
    DtLens L{tree, tsize};
    int prevlen = -1, curlen, nextlen = L.at(0), count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = L.at(n + 1);
        if (++count < max_count && curlen == nextlen) continue;
        else if (count < min_count) blv += (int)lane == curlen ? (uint32_t)count : 0u;
        else if (curlen != 0) { if (curlen != prevlen) blv += (int)lane == curlen; blv += lane == 16; }
        else if (count <= 10) blv += lane == 17;
        else blv += lane == 18;
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}
// the block header's bits: a register accumulator, stored a 32-bit word at a time (lane 0)
struct DtBits {
    uint32_t* hdr;
    uint64_t acc = 0;
    uint32_t n = 0, nb = 0, w = 0;
    __device__ void bits(uint32_t v, int len) {
        acc |= (uint64_t)v << n;
        n += (uint32_t)len;
        nb += (uint32_t)len;
        if (n >= 32) {
            if (threadIdx.x == 0) hdr[w] = (uint32_t)acc;
            ++w;
            acc >>= 32;
            n -= 32;
        }
    }
    __device__ void flush() { if (n && threadIdx.x == 0) hdr[w] = (uint32_t)acc; }
    // bits up to bit position p were OR-ed into hdr (zero past them): go on from p
    __device__ void resume(uint32_t p) {
        nb = p;
        w = p >> 5;
        n = p & 31u;
        acc = n ? (uint64_t)hdr[w] : 0ull;
    }
};
#ifndef DT_PAR
#define DT_PAR 1                          // scan_tree / send_tree over the wave (0: one lane's loop)
#endif
// scan_tree and send_tree cut each run of equal code lengths into the same pieces: a run of
// zeros into pieces of up to 138; any other run into a first piece of up to 7, then pieces of
// up to 6 (the max_count / min_count they set after each piece: 138 / 3 when the next length
// is 0, 6 / 3 when the run goes on, 7 / 4 when a new nonzero run starts).  So a length at
// offset t of its run starts a piece iff t % 138 == 0 (zeros), or t == 0 or (t - 7) % 6 == 0,
// and the piece's size is min(138 | 7 | 6, the rest of the run).  dt_pieces finds every
// position's run (start and end from per-chunk ballots of "differs from the previous length",
// with the guard at max_code + 1 ending the last run) and hands f, chunk by chunk with the
// whole wave: (piece start?, length, piece size, first piece of its run?).
template <class F>
__device__ __forceinline__ void dt_pieces(const uint16_t* tree, int max_code, F f) {
    const int lane = (int)threadIdx.x;
    const int nch = (max_code + 2 + 63) >> 6;                     // positions 0 .. max_code + 1
    uint32_t lv[5];
    uint64_t S[5];
    int fsa[5];
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        const int i = c * 64 + lane;
        lv[c] = c < nch && i <= max_code ? (uint32_t)tree[i * 2 + 1] : 0xffffu;
    }
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        uint32_t prev = (uint32_t)__shfl_up((int)lv[c], 1);
        if (lane == 0) prev = c ? (uint32_t)dt_rdl(lv[c ? c - 1 : 0], 63) : 0xfffeu;
        S[c] = c < nch ? __ballot(lv[c] != prev) : 0ull;
    }
    int nxt = 0;
#pragma unroll
    for (int c = 4; c >= 0; --c) {
        fsa[c] = nxt;
        if (S[c]) nxt = c * 64 + (int)__builtin_ctzll(S[c]);
    }
    int ls = 0;
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        if (c < nch) {
            const int n = c * 64 + lane;
            const uint64_t le = (2ull << lane) - 1ull;               // positions <= n (lane 63: all)
            const uint64_t mb = S[c] & le, ma = S[c] & ~le;
            const int st = mb ? c * 64 + 63 - (int)__clzll(mb) : ls;
            const int en = ma ? c * 64 + (int)__builtin_ctzll(ma) : fsa[c];
            const int v = (int)lv[c], t = n - st;
            const bool first = t == 0;
            const bool pc = n <= max_code && (v == 0 ? t % 138 == 0 : (first || (t >= 7 && (t - 7) % 6 == 0)));
            const int P = v == 0 ? 138 : first ? 7 : 6;
            f(pc, v & 31, min(P, en - n), first);
            if (S[c]) ls = c * 64 + 63 - (int)__clzll(S[c]);
        }
    }
}
// scan_tree (deflate.ts:267-312): each piece's bit-length codes counted into blacc (LDS)
__device__ void dt_scan_par(uint16_t* tree, int max_code, uint32_t* blacc) {
    if (threadIdx.x == 0) tree[(max_code + 1) * 2 + 1] = 0xffff;   // the reference's guard (kept as it leaves it)
    dt_pieces(tree, max_code, [&](bool pc, int v, int q, bool first) {
        if (!pc) return;
        if (v == 0) {
            if (q < 3) atomicAdd(&blacc[0], (uint32_t)q);
            else atomicAdd(&blacc[q <= 10 ? 17 : 18], 1u);
        } else if (q < (first ? 4 : 3)) atomicAdd(&blacc[v], (uint32_t)q);
        else {
            if (first) atomicAdd(&blacc[v], 1u);
            atomicAdd(&blacc[16], 1u);
        }
    });
    __syncthreads();
}
// send_tree (deflate.ts:378-429): each piece's bits (<= 21) at its prefix-summed offset from
// bit o.nb, OR-ed into the zeroed header words; blc: lane j holds bl code j as code | len << 16
__device__ void dt_send_par(DtBits& o, const uint16_t* tree, int max_code, uint32_t blc) {
    const int lane = (int)threadIdx.x;
    o.flush();
    __syncthreads();
    const uint32_t e16 = (uint32_t)dt_rdl(blc, 16), e17 = (uint32_t)dt_rdl(blc, 17), e18 = (uint32_t)dt_rdl(blc, 18);
    uint32_t base = o.nb;
    dt_pieces(tree, max_code, [&](bool pc, int v, int q, bool first) {
        const uint32_t ev = (uint32_t)__shfl((int)blc, v);
        uint32_t b = 0, nbits = 0;
        if (pc) {
            const uint32_t cv = ev & 0xffffu, lv = ev >> 16;
            if (q < (v == 0 || !first ? 3 : 4)) {
                for (int i = 0; i < q; ++i) b |= cv << (i * lv);
                nbits = (uint32_t)q * lv;
            } else if (v != 0) {
                const uint32_t c16 = e16 & 0xffffu, l16 = e16 >> 16;
                if (first) { b = cv | (c16 << lv) | ((uint32_t)(q - 4) << (lv + l16)); nbits = lv + l16 + 2; }
                else { b = c16 | ((uint32_t)(q - 3) << l16); nbits = l16 + 2; }
            } else if (q <= 10) { b = (e17 & 0xffffu) | ((uint32_t)(q - 3) << (e17 >> 16)); nbits = (e17 >> 16) + 3; }
            else { b = (e18 & 0xffffu) | ((uint32_t)(q - 11) << (e18 >> 16)); nbits = (e18 >> 16) + 7; }
        }
        uint32_t x = nbits;                                       // inclusive scan over the wave
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, d);
            if (lane >= d) x += y;
        }
        if (nbits) {
            const uint32_t off = base + x - nbits, w = off >> 5, sh = off & 31u;
            atomicOr(&o.hdr[w], b << sh);
            if (sh + nbits > 32) atomicOr(&o.hdr[w + 1], b >> (32 - sh));
        }
        base += (uint32_t)dt_rdl(x, 63);
    });
    __syncthreads();
    o.resume(base);
}
// send_tree (deflate.ts:378-429); blc: lane j holds bl code j as code | len << 16
__device__ void dt_send(DtBits& o, const uint16_t* tree, int tsize, int max_code, uint32_t blc) {
    DtLens L{tree, tsize};
    auto put = [&](int c) { const uint32_t e = (uint32_t)dt_rdl(blc, c); o.bits(e & 0xffffu, (int)(e >> 16)); };
    int prevlen = -1, curlen, nextlen = L.at(0), count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = L.at(n + 1);
        if (++count < max_count && curlen == nextlen) continue;
        else if (count < min_count) { do { put(curlen); } while (--count != 0); }
        else if (curlen != 0) {
            if (curlen != prevlen) { put(curlen); count--; }
            put(16);
            o.bits((uint32_t)(count - 3), 2);
        } else if (count <= 10) { put(17); o.bits((uint32_t)(count - 3), 3); }
        else { put(18); o.bits((uint32_t)(count - 11), 7); }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}
// k_dfl_trees: one wave per (stream, block), blocks y, y + ny, ...  Frequencies from the
// symbols (LDS atomics), the trees and the block type choice of _tr_flush_block
// (deftree.ts:1044-1108), the code table (code | len << 16) and the header bits out.
__global__ __launch_bounds__(64) void k_dfl_trees(DeflateArgs A) {
    __shared__ uint16_t ltree[HEAP_SIZE * 2], dtree[(2 * D_CODES + 1) * 2], bltree[(2 * BL_CODES + 1) * 2];
    __shared__ uint16_t order[HEAP_SIZE];
    __shared__ __attribute__((aligned(8))) uint32_t hk[L_CODES + 2];
    __shared__ uint32_t blcnt[16], blacc[32], hist[L_CODES + D_CODES], hdr[FB_HDR_WORDS];
    __shared__ int xch;
    __shared__ uint16_t s_sl[288 * 2], s_sd[30 * 2];
    __shared__ uint8_t s_xl[32], s_xd[32], s_xbl[32], lcode_t[256], dcode_t[512];
    const uint32_t sid = blockIdx.x, lane = threadIdx.x;
#ifdef DT_PROF
    uint64_t tk[16] = {}, tb[5] = {};
    uint64_t* const tpk = sid == 0 && blockIdx.y == 0 ? tk : nullptr;
    uint64_t* const tpb = sid == 0 && blockIdx.y == 0 ? tb : nullptr;
#else
    uint64_t* const tpk = nullptr;
    uint64_t* const tpb = nullptr;
    (void)tpk;
#endif
    DT_T(tpk, 0);
    if (sid >= A.n) return;
    GLB DSlab* S = (GLB DSlab*)(A.state + (uint64_t)sid * SLAB_BYTES);
    GLB FStream* F = (GLB FStream*)S->window;
    // the stream's words and the tables in one round trip (a lone wave waits for each)
    const uint32_t flag = F->flag, nblk = F->nblk;
    const uint64_t rp0 = A.rp0[sid], tb0 = A.tb0[sid];
    const GLB DTables* T = (const GLB DTables*)&g_dt;
    for (int i = (int)lane; i < 256; i += 64) lcode_t[i] = T->length_code[i];
    for (int i = (int)lane; i < 512; i += 64) dcode_t[i] = T->dist_code[i];
    for (int i = (int)lane; i < 288 * 2; i += 64) s_sl[i] = T->static_ltree[i];
    if (lane < 60) s_sd[lane] = T->static_dtree[lane];
    if (lane < 29) s_xl[lane] = T->extra_lbits[lane];
    if (lane < 30) s_xd[lane] = T->extra_dbits[lane];
    if (lane < 19) s_xbl[lane] = T->extra_blbits[lane];
    if (flag) return;
    const GLB uint32_t* sym = (const GLB uint32_t*)A.sym_buf + rp0;
    for (uint32_t b = blockIdx.y; b < nblk; b += gridDim.y) {
        GLB FBlock* Bk = (GLB FBlock*)(A.blk + (tb0 + b) * FB_SLOT);
        const uint32_t sym0 = Bk->sym0, nsym = Bk->nsym, eof = Bk->eof;
        const int block_start = Bk->block_start, strstart = Bk->strstart;
        for (int i = (int)lane; i < L_CODES + D_CODES; i += 64) hist[i] = 0;
        for (int i = (int)lane; i < HEAP_SIZE * 2; i += 64) ltree[i] = 0;
        for (int i = (int)lane; i < (2 * D_CODES + 1) * 2; i += 64) dtree[i] = 0;
        for (int i = (int)lane; i < (2 * BL_CODES + 1) * 2; i += 64) bltree[i] = 0;
        for (int i = (int)lane; i < FB_HDR_WORDS; i += 64) hdr[i] = 0;
        if (lane < 32) blacc[lane] = 0;
        __syncthreads();
        for (uint32_t i = lane; i < nsym; i += 64) {
            const uint32_t s = sym[sym0 + i], lc = s & 255u, dist = s >> 8;
            if (dist == 0) atomicAdd(&hist[lc], 1u);
            else {
                const uint32_t d = dist - 1;
                atomicAdd(&hist[257 + lcode_t[lc]], 1u);
                atomicAdd(&hist[L_CODES + (d < 256 ? dcode_t[d] : dcode_t[256 + (d >> 7)])], 1u);
            }
        }
        __syncthreads();
        if (lane == 0) hist[END_BLOCK] += 1;                 // init_block's END_BLOCK count
        __syncthreads();
        for (int i = (int)lane; i < L_CODES; i += 64) ltree[i * 2] = (uint16_t)hist[i];
        for (int i = (int)lane; i < D_CODES; i += 64) dtree[i * 2] = (uint16_t)hist[L_CODES + i];
        __syncthreads();
        WTree W{order, hk, blcnt, &xch, 0, 0};
        DT_T(tpk, 1);
        const int l_max = dt_build(W, ltree, s_sl, s_xl, 257, L_CODES, 15, tpb);
        DT_T(tpk, 2);
        const int d_max = dt_build(W, dtree, s_sd, s_xd, 0, D_CODES, 15);
        DT_T(tpk, 3);
#if DT_PAR
        dt_scan_par(ltree, l_max, blacc);
        dt_scan_par(dtree, d_max, blacc);
        if (lane < BL_CODES) bltree[lane * 2] = (uint16_t)blacc[lane];
#else
        uint32_t blv = 0;
        dt_scan(ltree, HEAP_SIZE * 2, l_max, blv);
        dt_scan(dtree, (2 * D_CODES + 1) * 2, d_max, blv);
        if (lane < BL_CODES) bltree[lane * 2] = (uint16_t)blv;
#endif
        __syncthreads();
        DT_T(tpk, 4);
        dt_build(W, bltree, (const uint16_t*)nullptr, s_xbl, 0, BL_CODES, 7);
        DT_T(tpk, 5);
        const uint32_t blc = lane < BL_CODES ? (uint32_t)bltree[lane * 2] | ((uint32_t)bltree[lane * 2 + 1] << 16) : 0u;
        int max_blindex;
        for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
            if (dt_rdl(blc, c_bl_order[max_blindex]) >> 16) break;
        const int opt_len = W.opt_len + 3 * (max_blindex + 1) + 5 + 5 + 4;
        uint32_t opt_lenb = (uint32_t)(opt_len + 3 + 7) >> 3;
        const uint32_t static_lenb = (uint32_t)(W.static_len + 3 + 7) >> 3;
        if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
        const int stored_len = strstart - block_start;
        DtBits o{hdr};
        uint32_t type;
        if ((uint32_t)(stored_len + 4) <= opt_lenb && block_start >= 0) {
            type = 0;
            o.bits(eof, 3);
        } else {
            type = static_lenb == opt_lenb ? 1 : 2;
            if (type == 1) o.bits(2u + eof, 3);
            else {
                o.bits(4u + eof, 3);
                const int lcodes = l_max + 1, dcodes = d_max + 1, blcodes = max_blindex + 1;
                o.bits((uint32_t)(lcodes - 257), 5);
                o.bits((uint32_t)(dcodes - 1), 5);
                o.bits((uint32_t)(blcodes - 4), 4);
                for (int rank = 0; rank < blcodes; rank++) o.bits((uint32_t)dt_rdl(blc, c_bl_order[rank]) >> 16, 3);
#if DT_PAR
                dt_send_par(o, ltree, lcodes - 1, blc);
                dt_send_par(o, dtree, dcodes - 1, blc);
#else
                dt_send(o, ltree, HEAP_SIZE * 2, lcodes - 1, blc);
                dt_send(o, dtree, (2 * D_CODES + 1) * 2, dcodes - 1, blc);
#endif
            }
        }
        o.flush();
        DT_T(tpk, 6);
        // the data bits of the block (codes and extra bits; compress_block's length)
        uint32_t db = 0;
        if (type != 0) {
            const bool st = type == 1;
            for (int i = (int)lane; i < L_CODES; i += 64) {
                const uint32_t h = hist[i];
                if (h) db += h * (uint32_t)(st ? s_sl[i * 2 + 1] : ltree[i * 2 + 1]);
                if (i >= 257) db += h * s_xl[i - 257];
            }
            if (lane < D_CODES) {
                const uint32_t h = hist[L_CODES + lane];
                if (h) db += h * ((uint32_t)(st ? 5 : dtree[lane * 2 + 1]) + s_xd[lane]);
            }
        }
        const uint32_t dbits = (uint32_t)dt_sum((int)db), hbits = o.nb;
        GLB uint32_t* tab = (GLB uint32_t*)((GLB uint8_t*)Bk + 64);
        if (type != 0)
            for (int i = (int)lane; i < L_CODES + D_CODES; i += 64) {
                uint32_t e;
                if (i < L_CODES) e = type == 2 ? (uint32_t)ltree[i * 2] | ((uint32_t)ltree[i * 2 + 1] << 16)
                                               : (uint32_t)s_sl[i * 2] | ((uint32_t)s_sl[i * 2 + 1] << 16);
                else {
                    const int d = i - L_CODES;
                    e = type == 2 ? (uint32_t)dtree[d * 2] | ((uint32_t)dtree[d * 2 + 1] << 16)
                                  : (uint32_t)s_sd[d * 2] | ((uint32_t)s_sd[d * 2 + 1] << 16);
                }
                tab[i] = e;
            }
        __syncthreads();                                      // the header words (lane 0) stored
        for (uint32_t i = lane; i < (hbits + 31) / 32; i += 64) tab[FB_HDR_OFF / 4 + i] = hdr[i];
        if (lane == 0) {
            Bk->type = type; Bk->hbits = hbits; Bk->dbits = dbits; Bk->stored_len = (uint32_t)stored_len;
        }
        __syncthreads();
        DT_T(tpk, 7);
#ifdef DT_PROF
        if (tpk && lane == 0)
            printf("DT_PROF lmax %d type %u | setup %lu ltree %lu (leaves %lu heap %lu chase %lu len %lu codes %lu) dtree %lu scan %lu bltree %lu hdr %lu out %lu [x10ns]\n",
                   l_max, type, tk[1] - tk[0], tk[2] - tk[1], tb[0] - tk[1], tb[1] - tb[0], tb[2] - tb[1], tb[3] - tb[2],
                   tb[4] - tb[3], tk[3] - tk[2], tk[4] - tk[3], tk[5] - tk[4], tk[6] - tk[5], tk[7] - tk[6]);
#endif
    }
}
#else
// k_dfl_trees: one wave per stream, its blocks in turn.  Frequencies from the symbols (LDS
// atomics), then lane 0 runs build_tree / scan_tree / build_bl_tree and the block type choice
// exactly as _tr_flush_block does, and the wave exports the code table (code | len << 16)
// and the block header bits.
__global__ __launch_bounds__(64) void k_dfl_trees(DeflateArgs A) {   // grid (n, ny): blocks y, y + ny, ...
    __shared__ uint16_t ltree[HEAP_SIZE * 2], dtree[(2 * D_CODES + 1) * 2], bltree[(2 * BL_CODES + 1) * 2];
    __shared__ uint16_t depth[2 * L_CODES + 1], heap[2 * L_CODES + 1], bl_count[16], next_code[16];
    __shared__ uint32_t hist[L_CODES + D_CODES];
    __shared__ uint32_t hdr[FB_HDR_WORDS];
    __shared__ uint32_t info[4];
    __shared__ uint8_t lcode_t[256], dcode_t[512];
    const uint32_t sid = blockIdx.x, lane = threadIdx.x;
    if (sid >= A.n) return;
    GLB DSlab* S = (GLB DSlab*)(A.state + (uint64_t)sid * SLAB_BYTES);
    GLB FStream* F = (GLB FStream*)S->window;
    if (F->flag) return;
    const GLB DTables* T = (const GLB DTables*)&g_dt;
    for (int i = (int)lane; i < 256; i += 64) lcode_t[i] = T->length_code[i];
    for (int i = (int)lane; i < 512; i += 64) dcode_t[i] = T->dist_code[i];
    const GLB uint32_t* sym = (const GLB uint32_t*)A.sym_buf + A.rp0[sid];
    const uint32_t nblk = F->nblk;
    for (uint32_t b = blockIdx.y; b < nblk; b += gridDim.y) {
        GLB FBlock* Bk = (GLB FBlock*)(A.blk + ((uint64_t)A.tb0[sid] + b) * FB_SLOT);
        const uint32_t sym0 = Bk->sym0, nsym = Bk->nsym, eof = Bk->eof;
        const int block_start = Bk->block_start, strstart = Bk->strstart;
        for (int i = (int)lane; i < L_CODES + D_CODES; i += 64) hist[i] = 0;
        for (int i = (int)lane; i < FB_HDR_WORDS; i += 64) hdr[i] = 0;
        for (int i = (int)lane; i < HEAP_SIZE * 2; i += 64) ltree[i] = 0;
        for (int i = (int)lane; i < (2 * D_CODES + 1) * 2; i += 64) dtree[i] = 0;
        for (int i = (int)lane; i < (2 * BL_CODES + 1) * 2; i += 64) bltree[i] = 0;
        __syncthreads();
        for (uint32_t i = lane; i < nsym; i += 64) {
            const uint32_t s = sym[sym0 + i], lc = s & 255u, dist = s >> 8;
            if (dist == 0) atomicAdd(&hist[lc], 1u);
            else {
                const uint32_t d = dist - 1;
                atomicAdd(&hist[257 + lcode_t[lc]], 1u);
                atomicAdd(&hist[L_CODES + (d < 256 ? dcode_t[d] : dcode_t[256 + (d >> 7)])], 1u);
            }
        }
        __syncthreads();
        if (lane == 0) hist[END_BLOCK] += 1;                 // init_block's END_BLOCK count
        __syncthreads();
        for (int i = (int)lane; i < L_CODES; i += 64) ltree[i * 2] = (uint16_t)hist[i];
        for (int i = (int)lane; i < D_CODES; i += 64) dtree[i * 2] = (uint16_t)hist[L_CODES + i];
        __syncthreads();
        if (lane == 0) {
            LTreeCtx c{heap, depth, bl_count, next_code, bltree, 0, 0, 0, 0, hdr, 0};
            const int l_max = build_tree(c, ltree, T->static_ltree, T->extra_lbits, 257, L_CODES, 15);
            const int d_max = build_tree(c, dtree, T->static_dtree, T->extra_dbits, 0, D_CODES, 15);
            scan_tree(c, ltree, l_max);
            scan_tree(c, dtree, d_max);
            build_tree(c, bltree, (const GLB uint16_t*)nullptr, T->extra_blbits, 0, BL_CODES, 7);
            int max_blindex;
            for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
                if (bltree[c_bl_order[max_blindex] * 2 + 1] != 0) break;
            c.opt_len += 3 * (max_blindex + 1) + 5 + 5 + 4;
            uint32_t opt_lenb = (uint32_t)(c.opt_len + 3 + 7) >> 3;
            const uint32_t static_lenb = (uint32_t)(c.static_len + 3 + 7) >> 3;
            if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
            const int stored_len = strstart - block_start;
            uint32_t type, dbits = 0;
            if ((uint32_t)(stored_len + 4) <= opt_lenb && block_start >= 0) {
                type = 0;
                c.bits(eof, 3);
            } else {
                const bool st = static_lenb == opt_lenb;
                type = st ? 1 : 2;
                if (st) c.bits(2u + eof, 3);
                else {
                    c.bits(4u + eof, 3);
                    const int lcodes = l_max + 1, dcodes = d_max + 1, blcodes = max_blindex + 1;
                    c.bits((uint32_t)(lcodes - 257), 5);
                    c.bits((uint32_t)(dcodes - 1), 5);
                    c.bits((uint32_t)(blcodes - 4), 4);
                    for (int rank = 0; rank < blcodes; rank++) c.bits(bltree[c_bl_order[rank] * 2 + 1], 3);
                    send_tree(c, ltree, lcodes - 1);
                    send_tree(c, dtree, dcodes - 1);
                }
                for (int i = 0; i < L_CODES; ++i)
                    if (hist[i]) dbits += hist[i] * (uint32_t)(st ? T->static_ltree[i * 2 + 1] : ltree[i * 2 + 1]);
                for (int i = 0; i < 29; ++i) dbits += hist[257 + i] * c_extra_lbits[i];
                for (int i = 0; i < D_CODES; ++i)
                    if (hist[L_CODES + i])
                        dbits += hist[L_CODES + i] * ((uint32_t)(st ? 5 : dtree[i * 2 + 1]) + c_extra_dbits[i]);
            }
            info[0] = type; info[1] = c.nb; info[2] = dbits; info[3] = (uint32_t)stored_len;
        }
        __syncthreads();
        const uint32_t type = info[0], hbits = info[1];
        GLB uint32_t* tab = (GLB uint32_t*)((GLB uint8_t*)Bk + 64);
        if (type != 0)
            for (int i = (int)lane; i < L_CODES + D_CODES; i += 64) {
                uint32_t code, len;
                if (i < L_CODES) {
                    code = type == 2 ? ltree[i * 2] : T->static_ltree[i * 2];
                    len = type == 2 ? ltree[i * 2 + 1] : T->static_ltree[i * 2 + 1];
                } else {
                    const int d = i - L_CODES;
                    code = type == 2 ? dtree[d * 2] : T->static_dtree[d * 2];
                    len = type == 2 ? dtree[d * 2 + 1] : T->static_dtree[d * 2 + 1];
                }
                tab[i] = (code & 0xffffu) | ((len & 0xffffu) << 16);
            }
        for (uint32_t i = lane; i < (hbits + 31) / 32; i += 64) tab[FB_HDR_OFF / 4 + i] = hdr[i];
        if (lane == 0) {
            Bk->type = type; Bk->hbits = hbits; Bk->dbits = info[2]; Bk->stored_len = info[3];
        }
        __syncthreads();
    }
}
#endif

// k_dfl_encode: one workgroup per stream.  Thread 0 lays the blocks out (bit offsets; the
// 16-bit pending units behind the overlay check; stored blocks' byte alignment), the group
// zeroes the output slot, then for each block every thread packs a run of symbols at its
// prefix-summed bit offset: whole words are stored, the partial words at run edges OR-ed.
#define EN_THREADS 256                                // (batches; few streams: 1024, k_dfl_encode_t<1024>)
#define EN_STG_WORDS_T(NT) ((NT) * 48 / 32 + 2)       // one row's bits (<= 48 per symbol)
template <int NT>
__device__ __forceinline__ uint32_t en_scan(uint32_t v, uint32_t* wsum, uint32_t& total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    uint32_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t base = 0, all = 0;
    for (uint32_t w = 0; w < NT / 64; ++w) { base += w < wv ? wsum[w] : 0u; all += wsum[w]; }
    __syncthreads();
    total = all;
    return base + x - v;
}
#ifndef EN_V2
#define EN_V2 1                           // encode rows: DPP scan, double-buffered stage and sums (2 barriers per row, not 4)
#endif
#if EN_V2
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t en_dpp_add(uint32_t x) {
    return x + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, false);
}
// the row's exclusive prefix of v over the workgroup and its total: an inclusive wave scan
// with DPP row shifts / broadcasts, the wave sums through wsum (this row's half of a double
// buffer: the next row writes the other half, so one barrier per row suffices)
template <int NT>
__device__ __forceinline__ uint32_t en_scan2(uint32_t v, uint32_t* wsum, uint32_t& total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    uint32_t x = v;
    x = en_dpp_add<0x111, 0xf>(x);                        // row_shr:1
    x = en_dpp_add<0x112, 0xf>(x);                        // row_shr:2
    x = en_dpp_add<0x114, 0xf>(x);                        // row_shr:4
    x = en_dpp_add<0x118, 0xf>(x);                        // row_shr:8
    x = en_dpp_add<0x142, 0xa>(x);                        // row_bcast:15 -> rows 1, 3
    x = en_dpp_add<0x143, 0xc>(x);                        // row_bcast:31 -> rows 2, 3
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t base = 0, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < NT / 64; ++w) {
        const uint32_t t = wsum[w];
        base += w < wv ? t : 0u;
        all += t;
    }
    total = all;
    return base + x - v;
}
#endif
template <int NT>
__global__ __launch_bounds__(NT) void k_dfl_encode_t(DeflateArgs A) {
    __shared__ uint32_t codes[L_CODES + D_CODES];
    __shared__ uint8_t lcode_t[256], dcode_t[512];
    __shared__ uint16_t lbase[29], dbase[30];
#if EN_V2
    __shared__ uint8_t xl_t[32], xd_t[32];
    __shared__ uint32_t wsum2[2][NT / 64];
    __shared__ uint32_t stg2[2][EN_STG_WORDS_T(NT)];
#else
    __shared__ uint32_t wsum[NT / 64];
    __shared__ uint32_t stg[EN_STG_WORDS_T(NT)];
#endif
    __shared__ uint64_t sh_end, sh_al;
    __shared__ uint32_t sh_bad;
    const uint32_t sid = blockIdx.x, tid = threadIdx.x;
    if (sid >= A.n) return;
    GLB DSlab* S = (GLB DSlab*)(A.state + (uint64_t)sid * SLAB_BYTES);
    GLB FStream* F = (GLB FStream*)S->window;
    if (F->flag) return;
    const GLB DTables* T = (const GLB DTables*)&g_dt;
    for (uint32_t i = tid; i < 256; i += NT) lcode_t[i] = T->length_code[i];
    for (uint32_t i = tid; i < 512; i += NT) dcode_t[i] = T->dist_code[i];
    if (tid < 29) lbase[tid] = T->base_length[tid];
    if (tid < 30) dbase[tid] = T->base_dist[tid];
#if EN_V2
    if (tid < 29) xl_t[tid] = T->extra_lbits[tid];
    if (tid < 30) xd_t[tid] = T->extra_dbits[tid];
    for (uint32_t i = tid; i < 2 * EN_STG_WORDS_T(NT); i += NT) (&stg2[0][0])[i] = 0;
    uint32_t rowpar = 0;                                     // which half of the double buffers
#define EN_XL(c) xl_t[c]
#define EN_XD(c) xd_t[c]
#else
#define EN_XL(c) c_extra_lbits[c]
#define EN_XD(c) c_extra_dbits[c]
#endif
    const uint32_t nblk = F->nblk;
    const bool gzip = A.format == SDZ_DEFLATE_GZIP;
    const uint32_t hdr_bytes = A.format == SDZ_DEFLATE_ZLIB ? 2 : gzip ? 10 + (A.fname_len ? A.fname_len + 1 : 0) : 0;
    const uint32_t trl_bytes = A.noflush ? 0u : A.format == SDZ_DEFLATE_ZLIB ? 4 : gzip ? 8 : 0;
    const uint64_t in_len = A.in_len[sid];
    GLB uint8_t* slots = (GLB uint8_t*)(A.blk + (uint64_t)A.tb0[sid] * FB_SLOT);
    auto blk_at = [&](uint32_t b) { return (GLB FBlock*)(slots + (uint64_t)b * FB_SLOT); };
    if (tid == 0) {
        uint64_t Tb = 8ull * hdr_bytes, al = Tb;             // bit position; last byte alignment
        uint32_t bad = 0;
        for (uint32_t b = 0; b < nblk; ++b) {
            GLB FBlock* Bk = blk_at(b);
            Bk->bstart = Tb;
            const uint32_t carry = (uint32_t)((Tb - al) & 15);  // bi_valid at the block's start
            Bk->carry = carry;
            if (Bk->type == 0) {
                const uint32_t K = carry + 3, rem = K & 15;
                const uint32_t pend = 2 * (K >> 4) + (rem > 8 ? 2 : rem > 0 ? 1 : 0) + 4;
                if (pend + Bk->stored_len > PENDING_SIZE) bad = 1;
                Tb = ((Tb + 3 + 7) & ~7ull) + 32 + 8ull * Bk->stored_len;
                al = Tb;
            } else {
                Tb += Bk->hbits + Bk->dbits;
            }
            if (Bk->eof) { Tb = (Tb + 7) & ~7ull; al = Tb; }
        }
        if ((Tb + 7) / 8 + trl_bytes > A.out_cap[sid]) bad = 1;
        sh_end = Tb;
        sh_al = al;
        sh_bad = bad;
    }
    __threadfence();                                         // (block layout: read by all threads)
    __syncthreads();
    if (sh_bad) { if (tid == 0) F->flag = 1; return; }
    const uint64_t total = (sh_end + 7) / 8 + trl_bytes;   // (NO_FLUSH: the last partial byte too)
    GLB uint8_t* out = (GLB uint8_t*)(A.out + A.out_off[sid]);
    {                                                        // zero the slot's bytes [0, total)
        const uint64_t mis = (4 - ((uintptr_t)out & 3)) & 3, head = mis < total ? mis : total;
        if (tid < head) out[tid] = 0;
        const uint64_t nw = (total - head) / 4;
        GLB uint32_t* w = (GLB uint32_t*)(out + head);
        for (uint64_t i = tid; i < nw; i += NT) w[i] = 0;
        for (uint64_t i = head + 4 * nw + tid; i < total; i += NT) out[i] = 0;
    }
    __threadfence();
    __syncthreads();
    GLB uint32_t* ow = (GLB uint32_t*)((uintptr_t)out & ~(uintptr_t)3);
    const uint64_t bias = ((uintptr_t)out & 3) * 8;
    auto orbits = [&](uint64_t bit, uint32_t v) {           // OR 32 bits of v at bit (slot-relative)
        bit += bias;
        const uint64_t w = bit >> 5;
        const uint32_t sh = (uint32_t)(bit & 31);
        if (v << sh) atomicOr((uint32_t*)&ow[w], v << sh);
        if (sh && (v >> (32 - sh))) atomicOr((uint32_t*)&ow[w + 1], v >> (32 - sh));
    };
    if (tid == 0) {                                          // container header (sd-deflate.ts:98-152)
        if (A.format == SDZ_DEFLATE_ZLIB) orbits(0, 0x0178u);
        else if (gzip) {
            orbits(0, 0x00088b1fu | ((A.fname_len ? 8u : 0u) << 24));
            orbits(32, A.mtime);
            orbits(64, 0xff00u);
            for (uint32_t i = 0; i < A.fname_len; i++) orbits(80 + 8 * i, A.fname[i]);
        }
    }
    const GLB uint32_t* sym = (const GLB uint32_t*)A.sym_buf + A.rp0[sid];
    uint32_t bad = 0;
    for (uint32_t b = 0; b < nblk; ++b) {
        const GLB FBlock* Bk = blk_at(b);
        const uint32_t type = Bk->type, hbits = Bk->hbits;
        const GLB uint32_t* tab = (const GLB uint32_t*)((const GLB uint8_t*)Bk + 64);
        const uint64_t b0 = Bk->bstart;
        for (uint32_t i = tid; i < (hbits + 31) / 32; i += NT) orbits(b0 + 32 * i, tab[FB_HDR_OFF / 4 + i]);
        if (type == 0) {                                     // _tr_stored_block: aligned LEN NLEN bytes
            const uint32_t len = Bk->stored_len;
            const uint64_t pay = ((b0 + 3 + 7) & ~7ull) / 8;
            const GLB uint8_t* src = (const GLB uint8_t*)(A.in + A.in_off[sid]) + Bk->off + Bk->block_start;
            for (uint32_t i = tid; i < 4 + len; i += NT) {
                uint8_t v;
                if (i < 4) v = (uint8_t)((i < 2 ? len : ~len) >> (8 * (i & 1)));
                else v = src[i - 4];
                out[pay + i] = v;
            }
            __syncthreads();
            continue;
        }
        for (uint32_t i = tid; i < L_CODES + D_CODES; i += NT) codes[i] = tab[i];
        __syncthreads();
        const uint32_t sym0 = Bk->sym0, nsym = Bk->nsym, items = nsym + 1;   // + END_BLOCK
        auto sym_bits = [&](uint32_t j, uint32_t& lo, uint32_t& nlo, uint32_t& hi, uint32_t& nhi) {
            if (j == nsym) { const uint32_t c = codes[END_BLOCK]; lo = c & 0xffffu; nlo = c >> 16; nhi = 0; hi = 0; return; }
            const uint32_t s = sym[sym0 + j], lc = s & 255u, dist = s >> 8;
            if (dist == 0) { const uint32_t c = codes[lc]; lo = c & 0xffffu; nlo = c >> 16; nhi = 0; hi = 0; return; }
            const uint32_t lcode = lcode_t[lc], c = codes[257 + lcode], cl = c >> 16, xl = EN_XL(lcode);
            lo = (c & 0xffffu) | (xl ? (lc - lbase[lcode]) << cl : 0u);   // code 28 (258): no extra bits
            nlo = cl + xl;
            const uint32_t d = dist - 1, dc = d < 256 ? dcode_t[d] : dcode_t[256 + (d >> 7)];
            const uint32_t e = codes[L_CODES + dc], el = e >> 16;
            hi = (e & 0xffffu) | ((d - dbase[dc]) << el);
            nhi = el + EN_XD(dc);
        };
        // rows of NT symbols (coalesced reads): scan the bit counts, OR each symbol's
        // bits into an LDS image of the row, write the image out (edge words OR-ed)
        const uint32_t carry = Bk->carry;
        uint64_t rowbit = b0 + hbits;                        // slot-relative bit of the row's start
        for (uint32_t r0 = 0; r0 < items; r0 += NT) {
            const uint32_t j = r0 + tid;
            uint32_t lo = 0, nlo = 0, hi = 0, nhi = 0;
            if (j < items) sym_bits(j, lo, nlo, hi, nhi);
            uint32_t tot;
#if EN_V2
            // stg2[rowpar] is all zero here: the row that used it last zeroed what it wrote
            uint32_t* stg = stg2[rowpar];
            const uint32_t excl = en_scan2<NT>(nlo + nhi, wsum2[rowpar], tot);
            rowpar ^= 1u;
#else
            const uint32_t excl = en_scan<NT>(nlo + nhi, wsum, tot);
#endif
            // pending_buf bytes written before symbol j is read (SURVEY A7 overlay)
            const uint64_t pend = 2 * ((carry + (rowbit + excl - b0)) >> 4);
            if (j < nsym && pend > (uint64_t)D_BUF + 2 * j) bad = 1;
            const uint64_t a0 = rowbit + bias, wbase = a0 >> 5;
            const uint32_t nw = (uint32_t)(((a0 + tot + 31) >> 5) - wbase);
#if !EN_V2
            for (uint32_t i = tid; i < nw; i += NT) stg[i] = 0;
            __syncthreads();
#endif
            const uint32_t at = (uint32_t)(a0 - wbase * 32) + excl;
            if (nlo) {
                const uint32_t w = at >> 5, sh = at & 31;
                atomicOr(&stg[w], lo << sh);
                if (sh + nlo > 32) atomicOr(&stg[w + 1], lo >> (32 - sh));
            }
            if (nhi) {
                const uint32_t a2 = at + nlo, w = a2 >> 5, sh = a2 & 31;
                atomicOr(&stg[w], hi << sh);
                if (sh + nhi > 32) atomicOr(&stg[w + 1], hi >> (32 - sh));
            }
            __syncthreads();
            for (uint32_t i = tid; i < nw; i += NT) {
                const uint32_t v = stg[i];
#if EN_V2
                stg[i] = 0;                                  // (for the row after next)
#endif
                const bool edge = (i == 0 && (a0 & 31)) || (i == nw - 1 && ((a0 + tot) & 31));
                if (!edge) ow[wbase + i] = v;
                else if (v) atomicOr((uint32_t*)&ow[wbase + i], v);
            }
#if !EN_V2
            __syncthreads();
#endif
            rowbit += tot;
        }
    }
    if (bad) atomicOr(&sh_bad, 1u);
    __syncthreads();
    if (tid == 0) {
        if (sh_bad) { F->flag = 1; return; }
        const uint32_t cks = A.cks_in ? (uint32_t)*A.cks_in : (uint32_t)A.cks[sid];
        const uint64_t e = sh_end;
        sdz_deflate_record R;
        R.status = SDZ_OK; R.checksum = (int32_t)cks; R.out_len = total; R.reserved = 0;
        if (A.noflush) {
            // what deflate(NO_FLUSH) has put in pending_buf: bytes up to the last byte-aligned
            // point, then the 16-bit units send_bits filled -- it writes a unit once a value
            // overflows it, so up to 16 bits stay in bi_buf (deflate.ts:347-366)
            const uint64_t al = sh_al;
            R.out_len = al / 8 + (e > al ? 2 * ((e - al - 1) / 16) : 0);
            R.reserved = F->pad[0];
        } else if (A.format == SDZ_DEFLATE_ZLIB) {
            orbits(e, ((cks >> 24) & 0xff) | ((cks >> 8) & 0xff00) | ((cks << 8) & 0xff0000) | (cks << 24));
        } else if (gzip) {
            orbits(e, cks); orbits(e + 32, (uint32_t)in_len);
        }
        A.rec[sid] = R;
    }
}

__global__ void k_max_u64(const uint64_t* v, uint32_t n, unsigned long long* out) {
    unsigned long long m = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        m = v[i] > m ? v[i] : m;
    for (int o = 32; o > 0; o >>= 1) { unsigned long long x = __shfl_xor(m, o); m = x > m ? x : m; }
    if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}
__global__ void k_sum_u64(const uint64_t* v, uint32_t n, unsigned long long* out) {
    unsigned long long m = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) m += v[i];
    for (int o = 32; o > 0; o >>= 1) m += __shfl_xor(m, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, m);
}
int device_sum_u64(const uint64_t* v, uint32_t n, unsigned long long* d_slot, uint64_t* out, hipStream_t st) {
    bool ok = hipMemsetAsync(d_slot, 0, sizeof *d_slot, st) == hipSuccess;
    hipLaunchKernelGGL(k_sum_u64, dim3(64), dim3(256), 0, st, v, n, d_slot);
    unsigned long long h = 0;
    ok = ok && hipGetLastError() == hipSuccess;
    ok = ok && hipMemcpyAsync(&h, d_slot, sizeof h, hipMemcpyDeviceToHost, st) == hipSuccess;
    ok = ok && hipStreamSynchronize(st) == hipSuccess;
    *out = h;
    return ok ? 0 : -1;
}
int device_max_u64(const uint64_t* v, uint32_t n, unsigned long long* d_slot, uint64_t* out, hipStream_t st) {
    bool ok = hipMemsetAsync(d_slot, 0, sizeof *d_slot, st) == hipSuccess;
    hipLaunchKernelGGL(k_max_u64, dim3(64), dim3(256), 0, st, v, n, d_slot);
    unsigned long long h = 0;
    ok = ok && hipGetLastError() == hipSuccess;
    ok = ok && hipMemcpyAsync(&h, d_slot, sizeof h, hipMemcpyDeviceToHost, st) == hipSuccess;
    ok = ok && hipStreamSynchronize(st) == hipSuccess;
    *out = h;
    return ok ? 0 : -1;
}

static bool c_config_host_fast(int level) { return level >= 1 && level <= 3; }
constexpr uint32_t kFzRounds = 1024;                       // then the unsettled streams go serial

// side/ev (optional): a second stream and an event for it.  The input checksum depends on
// nothing else: it runs on the side stream beside the parse and the trees, which are
// latency-bound (one lane per stream) and leave the CUs nearly idle; the encoder waits for
// it.  (k_dfl_tail beside k_dfl_match, the other candidate, slowed match by more than the
// tail's own 14 ms: C3 413 -> 438 ms of match.)
void launch_deflate(const DeflateArgs& a, hipStream_t st, hipStream_t side, hipEvent_t ev) {
    if (a.n == 0) return;
    dim3 grid((a.n + DF_THREADS - 1) / DF_THREADS);
    dt_ready(st);
    const bool fastlv = c_config_host_fast(a.level);
    if (a.rec_buf && (!fastlv || (a.lz_shift && (a.nlseg || a.noflush)))) {
        const int ck_kind = a.format == SDZ_DEFLATE_GZIP ? 1 : 0;
        if (a.ncunit)
            hipLaunchKernelGGL(k_dfl_chain, dim3((a.ncunit + CH_WAVES - 1) / CH_WAVES), dim3(64 * CH_WAVES), 0, st, a);
        if (!fastlv) {
            if (a.nmseg && a.l4_buf) {                        // the 4-byte chains
                hipLaunchKernelGGL(k_dfl_link4, dim3(link4_blocks(a.nmseg)), dim3(PM_THREADS), 0, st, a);
                hipLaunchKernelGGL(k_dfl_match4, dim3(match4_blocks(a.nmseg)), dim3(PM_THREADS), 0, st, a);
            } else if (a.nmseg) hipLaunchKernelGGL(k_dfl_match, dim3(a.nmseg), dim3(PM_THREADS), 0, st, a);
            hipLaunchKernelGGL(k_dfl_tail, dim3(a.n), dim3(256), 0, st, a);
        }
        const bool fork = side && ev && hipEventRecord(ev, st) == hipSuccess &&
                          hipStreamWaitEvent(side, ev, 0) == hipSuccess;
        if (fork) {
            launch_checksum(a.in, a.in_off, a.in_len, nullptr, a.cks, a.n, ck_kind, side);
            (void)hipEventRecord(ev, side);
        }
        if (a.lz_shift && (a.nlseg || a.noflush)) {       // (NO_FLUSH may have nothing to parse yet)
            const dim3 gseg((a.nlseg + LZ_THREADS - 1) / LZ_THREADS), gstr((a.n + LZ_THREADS - 1) / LZ_THREADS);
            if (fastlv) (void)hipMemsetAsync(a.lz_act, 0, (size_t)a.n * 4, st);
            if (!a.nlseg) {
            } else if (fastlv) {
                // rounds of the inserted-position fixed point; the host reads the number of
                // streams still moving after each (one small copy + sync per round)
                hipLaunchKernelGGL(k_fz_init, dim3((a.nlseg + 255) / 256), dim3(256), 0, st, a);
                // rounds are queued in batches of 1, 2, 4, then 8 between reads (a settled
                // stream's kernels return at once, so the rounds past the end cost launches only)
                for (uint32_t round = 1; round <= kFzRounds;) {
                    const uint32_t batch = round < 8 ? round : 8;
                    for (uint32_t b = 0; b < batch && round <= kFzRounds; ++b, ++round) {
                        DeflateArgs r = a;
                        r.lz_round = round;
                        hipLaunchKernelGGL(k_fz_match, dim3(a.nlseg), dim3(a.lz_shift >= 8 ? 256 : 1u << a.lz_shift), 0, st, r);
                        hipLaunchKernelGGL(k_fz_spec, gseg, dim3(LZ_THREADS), 0, st, r);
                        hipLaunchKernelGGL(k_fz_join, gseg, dim3(LZ_THREADS), 0, st, r);
                        hipLaunchKernelGGL(k_fz_fix, dim3(a.n), dim3(64), 0, st, r);
                        hipLaunchKernelGGL(k_fz_merge, gseg, dim3(LZ_THREADS), 0, st, r);
                        hipLaunchKernelGGL(k_fz_roll, dim3((a.n + 255) / 256), dim3(256), 0, st, r);
                    }
                    uint32_t moving_pageable = 0;
                    uint32_t* const pw = rt_pinned_words();
                    uint32_t& moving = pw ? pw[1] : moving_pageable;
                    moving = 0;
                    if (hipMemcpyAsync(&moving, a.lz_nact, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                        hipStreamSynchronize(st) != hipSuccess || moving == 0)
                        break;
                }
            } else {
                hipLaunchKernelGGL(k_lz_spec, gseg, dim3(LZ_THREADS), 0, st, a);
                hipLaunchKernelGGL(k_lz_join, gseg, dim3(LZ_THREADS), 0, st, a);
                hipLaunchKernelGGL(k_lz_fix, dim3(a.n), dim3(64), 0, st, a);
            }
            if (a.nlseg) hipLaunchKernelGGL(k_lz_count, gseg, dim3(LZ_THREADS), 0, st, a);
            hipLaunchKernelGGL(k_lz_scan, dim3(a.n), dim3(LS_THREADS), 0, st, a);
            if (a.nlseg) hipLaunchKernelGGL(k_lz_emit, gseg, dim3(LZ_THREADS), 0, st, a);
            if (a.n <= 16) hipLaunchKernelGGL(k_lz_blocks_t<1024>, dim3(a.n), dim3(1024), 0, st, a);
            else hipLaunchKernelGGL(k_lz_blocks_t<LB_THREADS>, dim3(a.n), dim3(LB_THREADS), 0, st, a);
        } else if (a.wide) hipLaunchKernelGGL(k_dfl_parse_wide, dim3(a.n), dim3(PW_THREADS), 0, st, a);
        else hipLaunchKernelGGL(k_dfl_parse, grid, dim3(64), 0, st, a);
        hipLaunchKernelGGL(k_dfl_trees, dim3(a.n, a.nbmax < 32 ? (a.nbmax ? a.nbmax : 1) : 32), dim3(64), 0, st, a);
        if (fork) (void)hipStreamWaitEvent(st, ev, 0);
        else launch_checksum(a.in, a.in_off, a.in_len, nullptr, a.cks, a.n, ck_kind, st);
        // few streams (one-buffer calls): 1,024 threads, a quarter of the rows (each row's fixed
        // scan and barriers were most of a 481 KB stream's 0.46 ms on 256 threads)
        if (a.n <= 16) hipLaunchKernelGGL(k_dfl_encode_t<1024>, dim3(a.n), dim3(1024), 0, st, a);
        else hipLaunchKernelGGL(k_dfl_encode_t<EN_THREADS>, dim3(a.n), dim3(EN_THREADS), 0, st, a);
        if (a.noflush) return;                               // (the caller redoes a flagged stream)
        DeflateArgs f = a;
        f.fast = 1;                                          // streams the record path handed back
        hipLaunchKernelGGL(k_deflate, grid, dim3(DF_THREADS), 0, st, f);
        return;
    }
    hipLaunchKernelGGL(k_deflate, grid, dim3(DF_THREADS), 0, st, a);
}

}  // namespace sdz
