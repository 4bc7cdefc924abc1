// split.h -- block-parallel decode of long streams: shared between the runtime (planning,
// sdz_runtime.cpp), the finder/chain/feed kernels (k_split.hip) and the segment mode of the
// decoder (k_inflate.hip).
#pragma once
#include <stdint.h>

namespace sdz {

#define SP_CAND_MAX 4096              // candidate block starts kept per stream
#define SPLIT_FILTER_BLOCKS 8192u    // k_split_filter's grid (one survivor region each)
#define SEG_HANDOVER 3                // DSave.stall of a segment that reached a candidate block start
#define SEG_FINAL 4                   // ... that reached the end of the last block (the trailer)
// split_state per stream: 0 serial decode; 1 fed from its segments; 2 planned (segments still
// decoding: skipped by the first round-0 decode); 3 planned, chain broken: decoded serially,
// starting in a second round-0 decode pass
#define SPS_FED 1u
#define SPS_PENDING 2u
#define SPS_FALLBACK 3u

struct SplitInfo {                    // one per split stream
    uint32_t sid;                     // stream index in the batch
    uint32_t ncand;                   // candidates found (atomic; may exceed SP_CAND_MAX: then no split)
    uint64_t nbits;
    uint64_t lane0;                   // first finder lane of this stream (32 bit positions per lane)
    uint32_t seg0, nseg;              // its segments: seg0 starts at bit 0, then one per candidate
    uint32_t skip0;                   // 1 when candidate 0 is bit 0 (covered by seg0, no own segment)
    uint32_t chain0;                  // offset of its chain arrays (nseg entries)
    uint32_t chain_len;
    uint32_t cand0;                   // offset of its candidates in the packed list (host copy)
    uint64_t ntok;                    // tokens of the chained stream
};

struct SegInfo {                      // one per segment
    uint64_t bit;                     // start bit
    uint64_t tok;                     // token buffer offset (tokens) in the segment token pool
    uint32_t cap;                     // token capacity
    uint32_t split;                   // index of its split stream (candidate list)
    uint32_t stream;                  // stream index in the batch
    uint32_t pad;
};

struct SplitPlan {                    // device pointers of one inflate call's split pre-pass
    uint32_t nsplit, nseg;
    SplitInfo* sp;
    SegInfo* seg;
    uint64_t* cand;
    uint32_t* chain;
    uint64_t* chain_tok;
    uint32_t* segtok;
    const void* segD;                 // the segments' decode states (their own DSave array)
    void* ready;                      // hipEvent_t: the segment decode (side stream) is done
};

}  // namespace sdz
