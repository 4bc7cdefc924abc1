/*
 * sdz.h -- C ABI of libsdz.so, the MI355X-native batched DEFLATE engine that
 * replaces the inflate/deflate hot path of @stardazed/zlib 1.0.1.
 *
 * The reference has no FFI: its boundary is the ES-module API
 * (src/sd-zlib.ts:39-43, typed in dist/sd-zlib.d.ts:11-149) over the engine seams
 * Inflate.inflate(z) (src/inflate.ts:132) and Deflate.deflate(flush)
 * (src/deflate.ts:1218).  Each entry point below names the reference interface it
 * replaces.  The N-API addon (sd-zlib_amd/js/sdz_napi.cpp) and the pytest ctypes
 * binding (sd-zlib_amd/python/sdz.py) are its two callers; see INTEGRATION.md.
 *
 * Conventions
 *  - plain pointers and sizes; no C++ exceptions cross this boundary;
 *  - functions return SDZ_API_OK (0) or a negative SDZ_API_* code, with the
 *    message in sdz_last_error();
 *  - per-stream outcomes are reported in records, never as API errors;
 *  - *_device entry points take device pointers and a hipStream_t (as void*),
 *    are asynchronous, and are the timed hot path;
 *  - the host entry points copy in, run the same kernels, and copy out.
 *  - there is no CPU implementation of any codec in this library: every path
 *    runs on the GPU and fails (SDZ_API_NO_DEVICE) when none is present.
 */
#ifndef SDZ_H
#define SDZ_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDZ_ABI_VERSION 4

/* API return codes */
enum {
    SDZ_API_OK = 0,
    SDZ_API_BAD_ARG = -1,
    SDZ_API_NO_DEVICE = -2,
    SDZ_API_HIP_ERROR = -3,
    SDZ_API_OOM = -4,
};

/* Container handling for inflate.
 *  AUTO:      inflate() detection rule, sd-inflate.ts:203-207
 *             (78 + FCHECK -> zlib, 1F 8B -> gzip, else raw);
 *  RAW:       Inflater({raw: true})  -> Inflate(blocksOnly) inflate.ts:100;
 *  CONTAINER: Inflater({raw: false}) -> DETECT mode, inflate.ts:142-175.      */
enum { SDZ_FMT_AUTO = 0, SDZ_FMT_RAW = 1, SDZ_FMT_CONTAINER = 2 };

/* Deflate container, sd-deflate.ts:17-30 ("raw" | "deflate" | "gzip") */
enum { SDZ_DEFLATE_RAW = 0, SDZ_DEFLATE_ZLIB = 1, SDZ_DEFLATE_GZIP = 2 };

/* Per-stream inflate status (maps 1:1 onto the reference's outcomes) */
enum {
    SDZ_OK = 0,            /* decoded; see verdict fields (finish(), sd-inflate.ts:159-179) */
    SDZ_DATA_ERROR = 1,    /* "inflate error: " + sdz_zmsg(zmsg)        sd-inflate.ts:128 */
    SDZ_NEED_DICT = 2,     /* "Custom dictionary required for this data" sd-inflate.ts:124 */
    SDZ_DICT_MISMATCH = 3, /* "Custom dictionary is not valid for this data" :120 */
    SDZ_TRUNCATED = 4,     /* incomplete: "Unexpected EOF during decompression" :216 */
    SDZ_OUT_OVERFLOW = 5,  /* out_cap too small: retry with a larger capacity */
    SDZ_TRAILING = 6,      /* bytes after the end of the stream: the reference's append()
                              loops forever here; reported instead */
    SDZ_TOO_SMALL = 7,     /* AUTO and < 2 bytes: "data buffer is too small" :195 */
    SDZ_BAD_RECORD = 8,    /* misaligned output offset (must be a multiple of 8) */
    SDZ_INTERNAL = 9,      /* engine watchdog: a resolve wait did not complete (never expected) */
    SDZ_CARRY_OVERFLOW = 10, /* incremental mode: one header or block header needed more than
                              SDZ_INFLATE_CARRY bytes of buffered input (a gzip FNAME/FCOMMENT
                              longer than that); the stream cannot continue */
};

/* Checksum / size verdicts ("unchecked" | "match" | "mismatch") */
enum { SDZ_UNCHECKED = 0, SDZ_MATCH = 1, SDZ_MISMATCH = 2 };
/* container actually seen (Inflate.containerFormat, inflate.ts:128-130) */
enum { SDZ_CONTAINER_RAW = 0, SDZ_CONTAINER_ZLIB = 1, SDZ_CONTAINER_GZIP = 2 };

/* One record per stream, written by the device (64 bytes). */
typedef struct sdz_inflate_record {
    int32_t  status;            /* SDZ_OK ... */
    int32_t  zmsg;              /* reason, sdz_zmsg(); 0 = none */
    uint64_t out_len;           /* bytes written to the stream's output slot */
    uint64_t in_used;           /* input bytes consumed */
    int32_t  stored_checksum;   /* Inflate.checksum (signed, 0 = absent) */
    int32_t  running_checksum;  /* Inflater.checksum over the output, reference quirks included */
    int32_t  stored_size;       /* gzip ISIZE as the reference reads it (signed int32) */
    int32_t  mtime;             /* gzip MTIME (signed int32); 0 => modDate undefined */
    uint32_t name_off;          /* gzip FNAME: byte offset within the input stream */
    uint32_t name_len;          /*            and length (Latin-1, no terminator) */
    uint8_t  container;         /* SDZ_CONTAINER_* */
    uint8_t  complete;          /* Inflate.isComplete, inflate.ts:103-107 */
    uint8_t  checksum_verdict;  /* SDZ_UNCHECKED / SDZ_MATCH / SDZ_MISMATCH */
    uint8_t  size_verdict;
    uint8_t  success;           /* complete && no mismatch */
    uint8_t  out_full;          /* incremental mode: stopped at out_cap; pass the input from
                                   in_used on again (sdz_inflate_append_batch_device) */
    uint8_t  reserved[10];
} sdz_inflate_record;

typedef struct sdz_deflate_record {
    int32_t  status;            /* 0 ok; SDZ_OUT_OVERFLOW; SDZ_DATA_ERROR (pending_buf overflow
                                   in the reference's overlay, undefined output there) */
    int32_t  checksum;          /* adler32 / crc32 of the input as written in the trailer */
    uint64_t out_len;
    uint64_t reserved;
} sdz_deflate_record;

/* ---------------------------------------------------------------- inflate */

/* Replaces Inflater.append(whole stream) + finish() / inflate()
 * (sd-inflate.ts:87-179, 189-228; engine inflate.ts:132 + infblocks/infcodes/inftree).
 * Device pointers.  Stream i reads in[in_off[i] .. +in_len[i]) and writes
 * out[out_off[i] .. +out_cap[i]).  out_off must be a multiple of 8; the input
 * allocation must have >= 64 readable bytes after the last stream (reads are
 * 16-byte vectors).  dict (may be NULL) is the preset dictionary offered to
 * every stream that sets FDICT.  stream = hipStream_t (NULL = default). */
int sdz_inflate_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                             uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap,
                             sdz_inflate_record* rec, uint32_t n, int32_t format,
                             const uint8_t* dict, uint32_t dict_len, void* stream);

/* Host convenience wrapper around sdz_inflate_batch_device (copies both ways). */
int sdz_inflate_batch(const uint8_t* const* in, const size_t* in_len, uint8_t* const* out,
                      const size_t* out_cap, sdz_inflate_record* rec, uint32_t n,
                      int32_t format, const uint8_t* dict, size_t dict_len);

/* ------------------------------------------------- incremental inflate */

/* Inflater.append(chunk) across calls, as many Inflaters at once (sd-inflate.ts:54-179;
 * engine state inflate.ts:79-95, infblocks.ts:45-50, infcodes.ts:35-55).  A state slab
 * holds n independent streams' decoder state in device memory between calls: the bit
 * position, block mode and Huffman tables, the last 32 KiB of output (the LZ77 window),
 * the input bytes of a unit (header, block header, symbol) not yet complete, and the
 * running checksum exactly as the reference's Inflater keeps it (adler32 per 16 KiB
 * output chunk with the adler32.ts:67 NMAX quirk; crc32 for gzip).
 *
 * Each sdz_inflate_append_batch_device call hands every stream its next input chunk
 * (in_len[i] may be 0) and an output slot; the stream decodes as far as its input allows
 * -- output ends where the reference's append() output would end -- and writes a record:
 *  - out_len: bytes written by this call (out[out_off[i] ..]);
 *  - status SDZ_TRUNCATED with complete = 0: more input is needed (not an error);
 *  - in_used: the stream offset up to which input is consumed or held on the device;
 *  - out_full = 1: out_cap was reached before the chunk was used up; the chunk's bytes
 *    from stream offset in_used on were not taken: pass them again (before any new
 *    bytes) in the next call, which continues the output;
 *  - name_off: gzip FNAME offset from the stream's first input byte;
 *  - checksum/size verdicts and success as finish() would report them now.
 * A stream that already finished reports SDZ_TRAILING if it is given more bytes.
 * Divergences from the reference are its defects: a stored block or a dynamic block
 * header split across calls decodes correctly here. */
#define SDZ_INFLATE_CARRY 16384u
uint64_t sdz_inflate_state_bytes(uint32_t n);
/* fresh Inflaters: format SDZ_FMT_RAW (options.raw) or SDZ_FMT_CONTAINER */
int sdz_inflate_state_reset_device(void* state, uint32_t n, void* stream);
int sdz_inflate_append_batch_device(void* state, const uint8_t* in, const uint64_t* in_off,
                                    const uint64_t* in_len, uint8_t* out, const uint64_t* out_off,
                                    const uint64_t* out_cap, sdz_inflate_record* rec, uint32_t n,
                                    int32_t format, const uint8_t* dict, uint32_t dict_len,
                                    void* stream);

/* One Inflater on host buffers (what the N-API and ctypes facades call): create, then
 * append(chunk) -> *out / *out_len (valid until the next call on this handle) and the
 * record of the stream so far; the loop over out_full is done inside. */
typedef struct sdz_inflater sdz_inflater;
sdz_inflater* sdz_inflater_create(int32_t format, const uint8_t* dict, size_t dict_len);
int sdz_inflater_append(sdz_inflater* z, const uint8_t* data, size_t len, const uint8_t** out,
                        size_t* out_len, sdz_inflate_record* rec);
void sdz_inflater_destroy(sdz_inflater* z);

/* ---------------------------------------------------------------- deflate */

/* Replaces Deflater(opts).append(whole input) + finish() / deflate()
 * (sd-deflate.ts:51-274; engine deflate.ts:196-1327 + deftree.ts).  Output is
 * bit-exact with the reference for the same input, level, format, file name and
 * MTIME (the reference stamps Math.floor(Date.now()/1000), sd-deflate.ts:140;
 * the caller passes it here).  fname: Latin-1 bytes already mapped as
 * sd-deflate.ts:125-130 does (NULL/0 = no FNAME).  dict (may be NULL; format
 * SDZ_DEFLATE_ZLIB only, as sd-deflate.ts:80-90 requires) is the preset dictionary of
 * every stream: deflateSetDictionary (deflate.ts:1184-1216) and the 78 20 + DICTID
 * header.  Device pointers (dict too). */
int sdz_deflate_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                             uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap,
                             sdz_deflate_record* rec, uint32_t n, int32_t level, int32_t format,
                             const uint8_t* fname, uint32_t fname_len, uint32_t mtime,
                             const uint8_t* dict, uint32_t dict_len, void* stream);

int sdz_deflate_batch(const uint8_t* const* in, const size_t* in_len, uint8_t* const* out,
                      const size_t* out_cap, sdz_deflate_record* rec, uint32_t n, int32_t level,
                      int32_t format, const uint8_t* fname, size_t fname_len, uint32_t mtime,
                      const uint8_t* dict, size_t dict_len);

/* ------------------------------------------------- incremental deflate */

/* Deflater.append(chunk) / finish() across calls, as many Deflaters at once
 * (sd-deflate.ts:51-254 over deflate.ts:1218-1327 with NO_FLUSH / FINISH).  A state slab
 * (sdz_deflate_state_bytes) holds each stream's compressor between calls: window, hash
 * chains, the block being built, the bit buffer, the running input checksum.  Each call
 * hands every stream its next chunk (in_len[i] may be 0) with finish = 0, or ends every
 * stream with finish = 1 (a chunk given with finish is compressed first).  A stream's output
 * for the call -- what the reference's append()/finish() returns, concatenated: the header
 * on the first non-empty append, the blocks flushed meanwhile, the trailer at finish -- goes
 * to out[out_off[i] ..]; out_cap[i] >= sdz_deflate_append_bound(in_len[i], ...) always
 * suffices.  rec: status (SDZ_DATA_ERROR for finish before any append and for an append
 * after finish, which the reference throws on), out_len of this call, the running checksum.
 * level, format, fname, mtime and dict must be the same on every call of a stream.  The
 * concatenated output equals sdz_deflate_batch_device's on the concatenated input. */
uint64_t sdz_deflate_state_bytes(uint32_t n);
uint64_t sdz_deflate_append_bound(uint64_t in_len, int32_t format, uint32_t fname_len);
int sdz_deflate_state_reset_device(void* state, uint32_t n, void* stream);
int sdz_deflate_append_batch_device(void* state, const uint8_t* in, const uint64_t* in_off,
                                    const uint64_t* in_len, uint8_t* out, const uint64_t* out_off,
                                    const uint64_t* out_cap, sdz_deflate_record* rec, uint32_t n,
                                    int32_t level, int32_t format, const uint8_t* fname,
                                    uint32_t fname_len, uint32_t mtime, const uint8_t* dict,
                                    uint32_t dict_len, int32_t finish, void* stream);

/* One Deflater on host buffers: create, then append(chunk, finish 0) / append(chunk or
 * NULL, finish 1) -> *out / *out_len (valid until the next call on this handle). */
typedef struct sdz_deflater sdz_deflater;
sdz_deflater* sdz_deflater_create(int32_t level, int32_t format, const uint8_t* fname, size_t fname_len,
                                  uint32_t mtime, const uint8_t* dict, size_t dict_len);
int sdz_deflater_append(sdz_deflater* z, const uint8_t* data, size_t len, int32_t finish,
                        const uint8_t** out, size_t* out_len, sdz_deflate_record* rec);
void sdz_deflater_destroy(sdz_deflater* z);

/* ------------------------------------------- fast deflate (NOT bit-exact) */

/* The opt-in fast compressor: valid raw / zlib / gzip streams -- the
 * container as sd-deflate.ts:98-165 writes it, any inflater reads them, adler32 / crc32 of
 * the input in the trailer -- but not the reference's bytes: each 8 KiB tile of a stream
 * is compressed on its own (greedy parse, one dynamic-Huffman or stored block per tile,
 * byte-aligned by an empty stored block).  Not a drop-in for deflate(); for callers that
 * only need a valid stream fast.  out_cap[i] >= sdz_deflate_fast_bound(in_len[i], ...). */
uint64_t sdz_deflate_fast_bound(uint64_t in_len, int32_t format, uint32_t fname_len);
int sdz_deflate_fast_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                                  uint8_t* out, const uint64_t* out_off, const uint64_t* out_cap,
                                  sdz_deflate_record* rec, uint32_t n, int32_t format,
                                  const uint8_t* fname, uint32_t fname_len, uint32_t mtime, void* stream);

/* Worst-case compressed size for one stream (header + blocks + trailer). */
uint64_t sdz_deflate_bound(uint64_t in_len, int32_t format, uint32_t fname_len);

/* -------------------------------------------------------------- checksums */

/* adler32(src, seed = 1) / crc32(src, seed = 0): adler32.ts:17-24 (including the
 * adler32.ts:67 NMAX quirk) and crc32.ts:17-23.  Signed int32 results.  Run on
 * the GPU (host buffer copied in).  The *_checked forms return SDZ_API_OK or an
 * error code (message in sdz_last_error()) and write the checksum to *result; the
 * plain forms return 0 on failure (0 is also a valid checksum: bindings use the
 * checked forms and throw). */
int sdz_adler32_checked(const uint8_t* buf, size_t len, int32_t seed, int32_t* result);
int sdz_crc32_checked(const uint8_t* buf, size_t len, int32_t seed, int32_t* result);
int32_t sdz_adler32(const uint8_t* buf, size_t len, int32_t seed);
int32_t sdz_crc32(const uint8_t* buf, size_t len, int32_t seed);

/* Batched device versions: result[i] = checksum(in[in_off[i] .. +in_len[i]), seed[i]) */
int sdz_adler32_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                             const int32_t* seed, int32_t* result, uint32_t n, void* stream);
int sdz_crc32_batch_device(const uint8_t* in, const uint64_t* in_off, const uint64_t* in_len,
                           const int32_t* seed, int32_t* result, uint32_t n, void* stream);

/* ------------------------------------------------------ multi-GPU */

/* The reference is single-threaded and has no batch API; these entry points run the batched
 * engine over several GPUs of one node.  Streams are independent, so a batch is cut into
 * shards by LPT (largest stream first, onto the shard with the fewest bytes so far), one
 * shard per entry of `devices`; one host thread per shard runs the single-device path on its
 * GPU (hipSetDevice), and the fixed-size per-stream records are all-gathered over RCCL
 * (ncclAllGather over xGMI) -- the only collective, after the codec kernels.  A device listed
 * twice (N logical shards on one GPU, for tests) uses a loopback gather instead (RCCL allows
 * one rank per device).  Outputs return to the caller's host buffers from each shard's GPU.
 * Records come back in the caller's stream order. */
#define SDZ_MAX_SHARDS 16

/* owner[i] = shard of stream i (LPT over sizes; ties by index: deterministic) */
int sdz_lpt_shard(const uint64_t* sizes, uint32_t n, uint32_t nshards, uint32_t* owner);

typedef struct sdz_multi_stats {
    double wall_ms;                        /* the whole call (host clock) */
    double compute_ms;                     /* slowest shard: staging + kernels + outputs back */
    double gather_ms;                      /* record all-gather (RCCL or loopback) + records to host */
    float kernel_ms[SDZ_MAX_SHARDS];       /* per shard: codec kernels (HIP events) */
    uint64_t bytes_in[SDZ_MAX_SHARDS];     /* per shard: input and output bytes */
    uint64_t bytes_out[SDZ_MAX_SHARDS];
    uint32_t streams[SDZ_MAX_SHARDS];
    int32_t nshards;
    int32_t collective;                    /* 1: RCCL ncclAllGather, 0: loopback gather */
} sdz_multi_stats;

/* sdz_inflate_batch / sdz_deflate_batch over ndev shards (devices[k] = HIP device of shard k,
 * ndev <= SDZ_MAX_SHARDS).  stats may be NULL. */
int sdz_inflate_batch_multi(const uint8_t* const* in, const size_t* in_len, uint8_t* const* out,
                            const size_t* out_cap, sdz_inflate_record* rec, uint32_t n, int32_t format,
                            const uint8_t* dict, size_t dict_len, const int32_t* devices, int32_t ndev,
                            sdz_multi_stats* stats);
int sdz_deflate_batch_multi(const uint8_t* const* in, const size_t* in_len, uint8_t* const* out,
                            const size_t* out_cap, sdz_deflate_record* rec, uint32_t n, int32_t level,
                            int32_t format, const uint8_t* fname, size_t fname_len, uint32_t mtime,
                            const uint8_t* dict, size_t dict_len, const int32_t* devices, int32_t ndev,
                            sdz_multi_stats* stats);

/* One process per GPU (torchrun-style launchers): a communicator over RCCL for the record
 * gather and the step barrier.  Rank 0 makes the id (sdz_comm_unique_id), every rank gets it
 * by the caller's own means, then each calls sdz_comm_init_rank on its current device. */
#define SDZ_COMM_ID_BYTES 128
typedef struct sdz_comm sdz_comm;
int sdz_comm_unique_id(uint8_t* id /* SDZ_COMM_ID_BYTES */);
sdz_comm* sdz_comm_init_rank(const uint8_t* id, int32_t nranks, int32_t rank);
/* recv (device) <- every rank's `bytes` of send (device), rank order; blocking */
int sdz_comm_allgather_device(sdz_comm* c, const void* send, void* recv, uint64_t bytes);
/* *v <- max over ranks (host value; a barrier for step timing) */
int sdz_comm_allreduce_max(sdz_comm* c, double* v);
int sdz_comm_destroy(sdz_comm* c);

/* ----------------------------------------------------------------- misc */

const char* sdz_zmsg(int32_t code);       /* z.msg text for a record's zmsg */
const char* sdz_last_error(void);
int sdz_version(void);                    /* SDZ_ABI_VERSION */
int sdz_device_count(void);
int sdz_set_device(int device);

/* Device memory plumbing for callers without their own HIP runtime (node, ctypes). */
void* sdz_device_alloc(uint64_t bytes);
void sdz_device_free(void* ptr);
int sdz_copy_to_device(void* dst, const void* src, uint64_t bytes);
int sdz_copy_to_host(void* dst, const void* src, uint64_t bytes);
int sdz_memset_device(void* dst, int value, uint64_t bytes);
int sdz_copy_device_to_device(void* dst, const void* src, uint64_t bytes);
/* n spans in one launch: dst[dst_off[i] ..] <- src[src_off[i] .. + len[i]) (device pointers,
 * asynchronous on stream; spans must not overlap).  Stages batches for the *_device calls. */
int sdz_gather_device(uint8_t* dst, const uint64_t* dst_off, const uint8_t* src, const uint64_t* src_off,
                      const uint64_t* len, uint32_t n, void* stream);
int sdz_sync(void* stream);
/* a non-blocking hipStream_t (as void*) for the *_device calls; NULL on failure */
void* sdz_stream_create(void);
int sdz_stream_destroy(void* stream);

/* Kernel timing: when enabled, *_device calls record HIP events on their launch
 * stream around the codec kernel(s); sdz_last_kernel_ms() waits for the stop
 * event of the most recent call on this thread and returns the elapsed ms. */
int sdz_set_timing(int enabled);
float sdz_last_kernel_ms(void);
/* per-kernel split of the last inflate call with timing on: [0] k_inflate_decode,
 * [1] k_inflate_resolve (both summed over rounds), [2] k_inflate_finalize, in ms */
int sdz_last_kernel_breakdown(float* ms3);

#ifdef __cplusplus
}
#endif
#endif
