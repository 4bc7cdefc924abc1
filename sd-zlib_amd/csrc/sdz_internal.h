// sdz_internal.h -- shared between the runtime (sdz_runtime.cpp) and the HIP kernels.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "sdz.h"
#include "split.h"

namespace sdz {

// z.msg reason codes (texts in sdz_runtime.cpp)
enum ZMsg : int32_t {
    ZM_NONE = 0, ZM_INVALID_GZIP_ID, ZM_UNKNOWN_METHOD, ZM_INVALID_WINDOW, ZM_HEADER_CHECK,
    ZM_NEED_DICT, ZM_BLOCK_TYPE, ZM_STORED_LENS, ZM_TOO_MANY_SYMS, ZM_BL_REPEAT,
    ZM_BL_OVERSUB, ZM_BL_INCOMPLETE, ZM_LL_OVERSUB, ZM_LL_INCOMPLETE, ZM_D_OVERSUB,
    ZM_D_INCOMPLETE, ZM_D_EMPTY, ZM_INVALID_DIST, ZM_INVALID_LITLEN, ZM_COUNT
};

// bytes of per-stream global scratch used by the inflate kernel (code lengths)
constexpr uint64_t kInflateScratchPerStream = 320;
// the wave decoder's provisional token slots per stream (64 lanes x WD_CAP tokens, then a dummy
// slot per lane for the compaction's masked-off stores)
constexpr uint64_t kWdProvTokens = 64 * 512 + 64;
#define IS_WIN 32768u                 // incremental mode: window bytes per stream

struct InflateArgs {
    const uint8_t* in;
    const uint64_t* in_off;
    const uint64_t* in_len;
    uint8_t* out;
    const uint64_t* out_off;
    const uint64_t* out_cap;
    sdz_inflate_record* rec;
    uint8_t* scratch;            // n * kInflateScratchPerStream
    const uint8_t* dict;         // preset dictionary (last <= 32767 bytes used), may be null
    uint32_t dict_len;
    int32_t dict_adler;          // adler32.ts of the full dictionary (when dict_adler_dev is null)
    const int32_t* dict_adler_dev;  // ... or computed on the device by this call (no host sync)
    uint32_t n;
    int32_t format;
    // round machinery (phase 1 -> tokens -> phase 2)
    void* dsave;                 // n * decode state
    void* rsave;                 // n * resolve state (inside the same slab, after dsave)
    uint32_t* tokens;            // n * round_tokens
    uint32_t round_tokens;
    uint32_t* ntok;              // n
    uint32_t* flags;             // n: 0 more rounds, 1 finished this round, 2 finished earlier
    uint32_t* active;            // 1 counter
    uint32_t wave;               // 1: this one-shot call decodes with the wave decoder (inflate_wave_policy)
    uint32_t* wdprov;            // ... whose provisional tokens: n * kWdProvTokens
    unsigned long long* dbg;     // phase cycle counters (SDZ_PHASE_TIMING), normally null
    // incremental mode (sdz_inflate_append_batch_device): input may continue in a later
    // call, so streams stall at the end of their input instead of ending TRUNCATED
    uint32_t streaming;
    uint8_t* window;             // n * 32 KiB: the 32 KiB before this call's output
    uint8_t* carry;              // n * SDZ_INFLATE_CARRY: input carried to the next call
    // block-parallel decode of long streams (k_split.hip, split.h)
    const SplitPlan* split_plan; // host pointer: this call's split pre-pass, or null
    uint32_t* split_state;       // per stream SPS_* (split.h): whether the rounds decode it
    uint32_t fallback_pass;      // 1: this round-0 decode runs the SPS_FALLBACK streams only
    uint32_t segmode;            // 1: this decode launch runs segments, one lane per segment
    const SegInfo* seg;          // segment mode: start bit, token buffer, stream per segment
    const SplitInfo* spinfo;     // segment mode: the split streams (candidate counts)
    const uint64_t* cand;        // segment mode: sorted candidates, SP_CAND_MAX per split stream
    uint32_t* segtok;            // segment mode: the segment token pool
    // host-side hints (host pointers / flags; kernels never read them)
    const uint64_t* host_len;    // the n input lengths, when the caller has them on the host
    uint32_t one_round;          // every stream finishes in one round: no active-count read-back
    uint64_t host_cap_max;       // the largest out_cap when the caller has them on the host (0: unknown)
    uint32_t no_gzip;            // the caller saw every input: none is a gzip stream (no crc32 finalize)
};

uint64_t inflate_dsave_bytes();  // per stream decode state
// one-shot batches: decode with the wave decoder (k_inflate_wdec, a wave per stream) rather than the
// lane decoder (k_inflate_decode, a lane per stream)?  SDZ_WDEC=1 / 0 forces it.  By default when
// the batch's compressed bytes are at most kWdAutoRatio times its longest stream's (the lane
// decoder's time is its longest stream's serial decode, ~3.7 MB/s per lane; the wave decoder's the
// batch's total at ~133 GB/s: equal at ~36,000 equal streams, measured crossover 32,768 on
// paradiselost copies and on distinct 64 KiB streams, tools/wdec_sweep.sh), for at most
// kWdAutoStreams streams of at most kWdAutoBytes each, and when the longest is at least
// kWdAutoMinBytes (shorter ones decode in a few lane steps, and the lane decoder's single decode +
// resolve launch keeps small calls' latency)
constexpr uint32_t kWdAutoStreams = 65536;
constexpr uint64_t kWdAutoRatio = 24576;
constexpr uint64_t kWdAutoBytes = 4ull << 20;
constexpr uint64_t kWdAutoMinBytes = 16ull << 10;
// wave decoder: alternations of k_inflate_wcold / k_inflate_wdec per round before the lane decoder
// finishes the round's remaining streams (one alternation per block otherwise)
constexpr uint32_t kWdLaneAfter = 16;
constexpr int kWdRestart = 1000;   // run_inflate_rounds: start the call over without the wave decoder
int inflate_wdec_mode();         // SDZ_WDEC: -1 unset, 0 off, 1 on
bool inflate_wave_policy(uint32_t n, const uint64_t* host_len, const uint64_t* dev_len, void* stream);
uint64_t inflate_rsave_bytes();  // per stream resolve state
// hook (optional): called once on the host right after the first round's decode is queued
// (the split pre-pass's second half); a nonzero return ends the rounds with that code
int run_inflate_rounds(const InflateArgs& a, hipStream_t s, uint32_t* host_active, float* kernel_ms,
                       int (*hook)(void*) = nullptr, void* hook_ctx = nullptr);
// incremental mode: fresh state / stage carry + chunk contiguously (k_istream.hip)
void launch_istate_reset(uint8_t* dsave, uint8_t* rsave, uint32_t n, hipStream_t s);
// block-parallel decode of long streams (k_split.hip)
void launch_split_find(const uint8_t* in, const uint64_t* in_off, SplitInfo* sp, uint32_t nsplit, uint64_t* cand,
                       uint64_t total_lanes, uint64_t* surv, uint32_t* nsurv, uint32_t cap, hipStream_t s);
// candidates of the split streams packed in stream order (SplitInfo.cand0), count in *total
void launch_split_pack(SplitInfo* sp, uint32_t nsplit, const uint64_t* cand, uint64_t* packed, uint32_t* total,
                       hipStream_t s);
void launch_seg_decode(const InflateArgs& a, hipStream_t s);
void launch_seg_chain(const InflateArgs& a, SplitInfo* sp, uint32_t nsplit, const SegInfo* seg, const uint64_t* cand,
                      const void* segD, uint32_t* chain, uint64_t* chain_tok, uint32_t* split_state, hipStream_t s);
void launch_seg_feed(const InflateArgs& a, uint32_t round, hipStream_t s);
// st_off: the staging slots (prefix sums of SDZ_INFLATE_CARRY + in_len + 64, 256-aligned)
void launch_istate_stage(const InflateArgs& a, const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                         uint8_t* stage, uint64_t* st_off, uint64_t* st_len, hipStream_t s);

struct DeflateArgs {
    const uint8_t* in;
    const uint64_t* in_off;
    const uint64_t* in_len;
    uint8_t* out;
    const uint64_t* out_off;
    const uint64_t* out_cap;
    sdz_deflate_record* rec;
    uint8_t* state;              // n * deflate_state_bytes()
    const uint8_t* fname;
    uint32_t fname_len;
    uint32_t mtime;
    uint32_t n;
    int32_t level;
    int32_t format;
    // record path (levels 4-9, inputs <= kDeflateRecMax; host plan, sdz_runtime.cpp): stream k
    // owns positions [rp0[k], rp0[k] + in_len) of the record and link buffers (rp0[k] = ~0: not
    // on the record path) and block slots [tb0[k], tb0[k + 1]); the match and chain kernels
    // run over work-unit lists (k << kRecUnitShift | unit)
    uint64_t* rec_buf;           // match records, a u32 per position at rp0[k] + p (null: classic path only)
    uint64_t qoff;               // ... and the differing quarter-chain results at qoff + rp0[k] + p (u32 units)
    uint16_t* pv_buf;            // hash chain links: distance to the previous same-hash position
    uint32_t* l4_buf;            // levels 4-9 (null: k_dfl_match): per position the 4-byte chain link
                                 // and its rank in the hash chain (k_dfl_link4)
    uint32_t* sym_buf;           // the parse's symbols, u32 index rp0[k] (normally rec_buf itself:
                                 // records are dead once parsed; a Deflater keeps its records)
    const uint64_t* rp0;         // n + 1 entries
    const uint32_t* tb0;         // n + 1 entries
    uint8_t* blk;                // block slots (FB_SLOT bytes each)
    const uint32_t* mseg;        // match segments (PM_SEG positions each)
    uint32_t nmseg;
    uint32_t seg_merge;          // match kernels: a stream's segment 0 also covers segments 1-2
    uint32_t pm_seg;             // k_dfl_match: positions per segment (0: PM_SEG; smaller for few streams)
    const uint32_t* cunit;       // chain units (k_dfl_chain)
    uint32_t ncunit;
    uint32_t nbmax;              // most block slots of one stream (k_dfl_trees grid)
    uint32_t wide;               // k_dfl_parse: one workgroup per stream (few, long streams)
    uint32_t tail_in_match;      // k_dfl_match searches the last positions too (in its last segment's
                                 // LDS window); k_dfl_tail does only those of the other window offset
    // segment-parallel lazy parse (k_lz_*, k_deflate.hip): stream k's positions cut into
    // segments of 1 << lz_shift, global segment ids [lz_sg0[k], lz_sg0[k + 1])
    uint32_t lz_shift;           // 0: the serial parse kernels instead
    uint32_t nlseg;
    const uint32_t* lz_sg0;      // n + 1 entries
    const uint32_t* lz_seg;      // nlseg entries: the stream of each segment
    uint64_t* lz_w;              // per position (rp0 + p): phase-1 state before the step | symbol << 32
    uint32_t* lz_s2;             // per position: the join / fix symbols
    uint64_t* lz_v1;             // bitmaps, word (rp0 + p) >> 6: phase-1 step positions,
    uint64_t* lz_e1;             //   phase-1 symbols,
    uint64_t* lz_e2;             //   join / fix symbols
    uint64_t* lz_end;            // per segment: the phase-1 parse's state where it left the segment
    uint64_t* lz_carry;          // per segment: the join's state where it left the segment
    uint32_t* lz_c;              // per segment: first position whose phase-1 parse is the true one
    uint32_t* lz_cnt;            // per segment: symbols, then their exclusive prefix in the stream
    uint32_t* lz_fin;            // per stream: bit 0 the final literal, bits 1.. the symbol count
    // fast levels (1-3, k_fz_*): the inserted-position fixed point, iterated per stream
    uint64_t* lz_i;              // bitmap: positions inserted into the hash chains (current guess)
    uint64_t* lz_i1;             // bitmaps of the next guess: phase-1 parses,
    uint64_t* lz_i2;             //   joins / fixes
    uint32_t* lz_act;            // per stream: bit 0 still iterating, bit 1 changed this round
    uint32_t* lz_nact;           // one counter: streams still iterating after a round
    uint32_t lz_round;           // the round (from 1); per segment, the last round that
    uint32_t* fz_rc;             //   recomputed its records,
    uint32_t* fz_chg;            //   changed its part of I,
    uint32_t* fz_fx;             //   had its join redone by k_fz_fix
    // Deflater.append on the record path (sdz_deflater_*): deflate(NO_FLUSH) -- the parse
    // stops at the first step with lookahead < MIN_LOOKAHEAD, only the blocks cut before it are
    // flushed, no trailer; the record's out_len is what the reference's pending buffer holds
    // then, its `reserved` field the stop position.  Flagged streams are not redone here.
    uint32_t noflush;
    const int32_t* cks_in;       // the running checksum (chunk-wise, as sd-deflate.ts:185-190), or null
    int32_t* cks;                // n input checksums (record path)
    uint32_t fast;               // set by launch_deflate: k_deflate redoes flagged streams only
    const uint8_t* dict;         // preset dictionary (deflateSetDictionary), may be null
    uint32_t dict_len;
    int32_t dict_adler;          // adler32.ts of the whole dictionary: the zlib header's DICTID
    const int32_t* dict_adler_dev;  // ... or computed on the device by this call (no host sync)
    unsigned long long* dbg;     // phase cycle counters (SDZ_PHASE_TIMING), normally null
};

uint64_t deflate_state_bytes();
void launch_deflate(const DeflateArgs& a, hipStream_t s, hipStream_t side = nullptr, hipEvent_t ev = nullptr);
// the fast (not bit-exact) compressor (k_deflate_fast.hip): 8 KiB tiles, one block each
#define FT_TILE_BYTES 8192u
#define FT_TILE_OUT 8256u                 // a tile's output slot (<= tile + 10 bytes)
void launch_fast_tiles(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len, const uint32_t* tile_stream,
                       const uint32_t* tile_idx, uint32_t ntiles, uint8_t* tile_out, uint32_t* tile_len, hipStream_t s);
void launch_fast_concat(const DeflateArgs& a, const uint32_t* tile0, const uint8_t* tile_out, const uint32_t* tile_len,
                        const int32_t* cks, hipStream_t s);
// incremental Deflater (k_deflate_stream): fresh state; one append (finish 0) / finish (1)
void launch_deflate_reset(uint8_t* state, uint32_t n, hipStream_t s);
void launch_deflate_stream(const DeflateArgs& a, uint32_t finish, hipStream_t s);
constexpr uint64_t kDeflateRecMax = 1ull << 30;    // longest input on the record path
constexpr uint32_t kRecUnitShift = 16;              // work units: k << 16 | unit (k, unit < 65536)
uint64_t deflate_rec_blocks(uint64_t len);          // block slots a record-path stream needs
uint32_t deflate_chain_units(uint64_t len);         // its k_dfl_chain units
uint32_t deflate_match_segs(uint64_t len, uint32_t seg = 16384);   // its k_dfl_match segments of `seg` positions
// max of n device-resident u64 values (blocking; for scratch sizing); d_slot: 8 device bytes
int device_max_u64(const uint64_t* v, uint32_t n, unsigned long long* d_slot, uint64_t* out, hipStream_t s);
int device_sum_u64(const uint64_t* v, uint32_t n, unsigned long long* d_slot, uint64_t* out, hipStream_t s);

void launch_checksum(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                     const int32_t* seed, int32_t* result, uint32_t n, int kind, hipStream_t s);
// one buffer, arguments by value (asynchronous: the DICTID of a dictionary)
void launch_checksum_one(const uint8_t* in, uint64_t len, int kind, int32_t seed, int32_t* result, hipStream_t s);
// batched span copy (k_gather.hip)
void launch_gather(uint8_t* dst, const uint64_t* dst_off, const uint8_t* src, const uint64_t* src_off,
                   const uint64_t* len, uint32_t n, hipStream_t s);
// a few pinned host words of this thread (sdz_runtime.cpp) for a round driver's counter read-back
uint32_t* rt_pinned_words();
// a small host call's [outputs | records] region back into mapped pinned memory (k_gather.hip)
void launch_copy_back(uint8_t* dst, const uint8_t* src, const uint64_t* out_off, const uint64_t* out_cap,
                      uint64_t rec_off, uint32_t rsz, uint32_t len_off, uint32_t m, hipStream_t s);
// the DICTID a kernel compares / writes
__device__ __forceinline__ int32_t dict_id_of(int32_t v, const int32_t* dev) { return dev ? *dev : v; }

}  // namespace sdz
