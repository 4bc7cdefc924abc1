/*
 * sdz_oracle.h -- CPU restatement of @stardazed/zlib's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / the reported CPU baseline.  The product path (libsdz.so) never
 * links, loads or calls anything in oracle/.
 *
 * Parity pin: the reference is TypeScript and the environment denied running it
 * (SURVEY.md §8c).  This restatement is pinned by the reference's own fixtures
 * (tests/golden/, copied from /root/reference/test/) and by the survey's
 * pre-denial observations (deflate L6 == paradiselost.deflate byte-exact; L1..L9
 * output sizes), see tests/test_oracle.py.
 */
#ifndef SDZ_ORACLE_H
#define SDZ_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* adler32.ts:34-105 (including its sum2 += BASE quirk); returns signed int32 */
int32_t oracle_adler32(const uint8_t* buf, size_t len, int32_t seed);
/* crc32.ts:48-106; returns signed int32 */
int32_t oracle_crc32(const uint8_t* buf, size_t len, int32_t seed);

/* What the facade would throw, or ORA_OK.  Messages: oracle_error_message(). */
enum {
    ORA_OK = 0,
    ORA_E_INFLATE_MSG = 1,          /* "inflate error: " + z.msg      sd-inflate.ts:128 */
    ORA_E_BAD_INPUT_DATA = 2,       /* "inflate error: bad input data" sd-inflate.ts:131 */
    ORA_E_DICT_INVALID = 3,         /* sd-inflate.ts:120 */
    ORA_E_DICT_REQUIRED = 4,        /* sd-inflate.ts:124 */
    ORA_E_UNEXPECTED_EOF = 5,       /* sd-inflate.ts:216 */
    ORA_E_INTEGRITY = 6,            /* sd-inflate.ts:219 */
    ORA_E_SIZE = 7,                 /* sd-inflate.ts:222 */
    ORA_E_DECOMPRESSION = 8,        /* sd-inflate.ts:224 */
    ORA_E_TOO_SMALL = 9,            /* sd-inflate.ts:195 */
    ORA_E_HANG = 10,                /* reference loops forever */
    ORA_E_OUT_CAP = 11,             /* caller's output buffer too small (oracle limit) */
    ORA_E_FINISH_BEFORE_APPEND = 12,/* sd-deflate.ts:233 */
    ORA_E_PENDING_OVERFLOW = 13,    /* reference would index past pending_buf (undefined) */
    ORA_E_BAD_ARG = 14,
};

typedef struct {
    int32_t error;            /* ORA_* */
    int32_t zmsg;             /* index into oracle_zmsg() when error == ORA_E_INFLATE_MSG */
    int32_t success;
    int32_t complete;
    int32_t checksum_verdict; /* 0 unchecked, 1 match, 2 mismatch */
    int32_t size_verdict;     /* 0 unchecked, 1 match, 2 mismatch */
    int32_t stored_checksum;
    int32_t running_checksum; /* Inflater.checksum (chunk-wise, quirks included) */
    int32_t stored_size;
    int32_t container;        /* 0 raw, 1 deflate(zlib), 2 gzip */
    int32_t mtime;
    int32_t name_len;
    uint64_t total_out;
    char name[256];
} oracle_inflate_result;

/* new Inflater({raw, dictionary}); append(part) for each part; finish().
 * raw: 0/1.  dict may be NULL.  Output (all chunks concatenated) goes to out. */
int32_t oracle_inflater_run(const uint8_t* const* parts, const size_t* part_lens, int32_t nparts,
                            int32_t raw, const uint8_t* dict, size_t dict_len,
                            uint8_t* out, size_t out_cap, oracle_inflate_result* res);

/* The same, also reporting each append()'s output length (part_out[nparts], may be
 * NULL) and the index of the append that threw (*err_part, -1 if none; may be NULL). */
int32_t oracle_inflater_run_parts(const uint8_t* const* parts, const size_t* part_lens, int32_t nparts,
                                  int32_t raw, const uint8_t* dict, size_t dict_len,
                                  uint8_t* out, size_t out_cap, oracle_inflate_result* res,
                                  size_t* part_out, int32_t* err_part);

/* The same, also reporting the arrays append() returns: the length of each Uint8Array the
 * reference pushes (sd-inflate.ts:101-150, one per 16 KiB ZStream pass that produced output)
 * and the append it belongs to; *nchunks counts them all (entries past chunk_cap dropped). */
int32_t oracle_inflater_run_chunks(const uint8_t* const* parts, const size_t* part_lens, int32_t nparts,
                                   int32_t raw, const uint8_t* dict, size_t dict_len,
                                   uint8_t* out, size_t out_cap, oracle_inflate_result* res,
                                   size_t* part_out, int32_t* err_part,
                                   size_t* chunk_sz, int32_t* chunk_part, size_t chunk_cap, size_t* nchunks);

/* inflate(data, dictionary) one-shot: auto-detect + throw mapping (sd-inflate.ts:189-228). */
int32_t oracle_inflate(const uint8_t* in, size_t in_len, const uint8_t* dict, size_t dict_len,
                       uint8_t* out, size_t out_cap, oracle_inflate_result* res);

const char* oracle_error_message(int32_t err);
const char* oracle_zmsg(int32_t idx);

/* new Deflater({level, format, dictionary, fileName}); append(part)...; finish();
 * format: 0 raw, 1 deflate, 2 gzip.  fname: Latin-1 bytes already mapped
 * (sd-deflate.ts:125-130), fname_len 0 => no FNAME.  mtime: gzip MTIME field
 * (the reference uses Math.floor(Date.now()/1000); pinned here for parity). */
int32_t oracle_deflater_run(const uint8_t* const* parts, const size_t* part_lens, int32_t nparts,
                            int32_t level, int32_t format, const uint8_t* dict, size_t dict_len,
                            int32_t has_dict, const uint8_t* fname, size_t fname_len,
                            uint32_t mtime, uint8_t* out, size_t out_cap, size_t* out_len);
/* the same; part_end (nparts + 1 entries): output length after each append() and after
 * finish(), i.e. where the reference's per-call outputs end (sd-deflate.ts:173-253) */
int32_t oracle_deflater_run_parts(const uint8_t* const* parts, const size_t* part_lens, int32_t nparts,
                                  int32_t level, int32_t format, const uint8_t* dict, size_t dict_len,
                                  int32_t has_dict, const uint8_t* fname, size_t fname_len,
                                  uint32_t mtime, uint8_t* out, size_t out_cap, size_t* out_len,
                                  size_t* part_end);

#ifdef __cplusplus
}
#endif
#endif
