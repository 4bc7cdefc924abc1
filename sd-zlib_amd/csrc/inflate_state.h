// inflate_state.h -- per-stream state shared by the two inflate phases
// (k_inflate.hip: Huffman decode -> tokens; k_resolve.hip: tokens -> bytes).
#pragma once
#include "sdz_internal.h"

namespace sdz {

enum : int { LM_INIT = 0, LM_TYPE = 1, LM_CODES = 2, LM_STORED = 3, LM_TRAILER = 4, LM_DONE = 5 };

#define IL_REGION 324                 // LDS symbol-table bytes per stream (81 dwords: odd stride)
#define IL_DSYM 288                   // u8 distance symbols follow the 288 u8 lit/len entries

// One canonical Huffman tree, decoded table-free.
//   lim[k]  left-justified 15-bit limit of the codes of length <= k
//   pk[k]   (rank offset + 32768) << 16 | literal threshold << 4 | (15 - k)
//           rank = (pk >> 16) - 32768 + (rc >> (15 - k)) for a code of length k;
//           ranks below the threshold are literals (lit/len tree only)
//   pk[16]  what codes at or past lim[15] select (incomplete trees): rank 300
//   c[]     code counts per length (3 x 10 bits per word) for huft_build replay
struct HTree {                        // what the hot loop keeps in registers
    uint32_t lim[16];
    uint32_t pk[17];
};
struct Tree : HTree {
    uint32_t c[5];
    int32_t l, kmin, g, left;         // huft_build root bits, min/max length, Kraft remainder
};

// per-stream decode state in HBM: between rounds, and the hand-off between the
// decoder's register-resident hot loop and its cold (block-level) code
struct DSave {
    uint8_t region[IL_REGION];
    uint64_t bitpos, pos;
    int32_t mode, last, container, status, zmsg, fixed, nl, nd;
    int32_t stored_ck, stored_size, mtime;
    uint32_t name_off, name_len, stored_left;
    int32_t dict_used, full;
    uint32_t ntok, litw, nlit;
    int32_t stall;                    // incremental mode: 1 out of input, 2 out of output room
    Tree LL, DD;
};

// per-stream resolve state (phase 2)
struct RSave {
    uint64_t pos;                     // this call: output bytes resolved so far
    uint32_t s1, s2;                  // this call: sum b, sum i b (mod 65521) of its output
    int32_t ck;                       // sticky watchdog flag
    uint32_t hist;                    // incremental: window[] holds the 32 KiB before this call
    // incremental mode: kept across calls
    uint64_t total;                   // output bytes of the earlier calls
    uint64_t in_base;                 // stream offset of this call's staged input byte 0
    uint32_t a1, a2;                  // Inflater.checksum (adler32.ts state) after earlier calls
    uint32_t crc;                     // Inflater.checksum (crc32, gzip) after earlier calls
    uint32_t carry_len;               // input bytes carried into the next call
    uint64_t abase;                   // output position where the current append() began
    uint32_t a1s, a2s;                // the (exact) adler32 state there
};

}  // namespace sdz
