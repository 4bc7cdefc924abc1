/*
 * sdz_oracle.c -- CPU restatement of @stardazed/zlib 1.0.1 (stardazed/sd-zlib).
 *
 * TEST INFRASTRUCTURE ONLY (see sdz_oracle.h).  Restates, function by function,
 * the reference TypeScript in /root/reference/src; each function cites the
 * file:line it follows.  JS semantics are kept where they matter for bytes:
 * signed int32 results, Uint8Array/Uint16Array truncating stores, the 32 KiB
 * inflate ring window, the 16 KiB ZStream output chunks (they decide the
 * Inflater's chunk-wise running checksum), and the deflate pending_buf overlay.
 *
 * Pinned by tests/test_oracle.py against the reference's fixtures.
 */
#define _POSIX_C_SOURCE 200809L
#include "sdz_oracle.h"
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* checksums                                                                  */
/* ------------------------------------------------------------------------- */

/* adler32.ts:34-105.  NB adler32.ts:67 adds BASE to sum2 after every NMAX block
 * instead of reducing it; the final reduction happens only when a remainder of
 * the buffer is left (adler32.ts:72,101), so a length that is a non-zero multiple
 * of 5552 returns the low 16 bits of the unreduced sum2 (JS ToInt32 then <<16). */
int32_t oracle_adler32(const uint8_t* buf, size_t len, int32_t seed) {
    uint32_t a = (uint32_t)seed;
    uint64_t s2 = (a >> 16) & 0xffffu;
    uint64_t s1 = a & 0xffffu;
    size_t off = 0;
    while (len >= 5552) {
        len -= 5552;
        for (int i = 0; i < 5552; i++) { s1 += buf[off++]; s2 += s1; }
        s1 %= 65521u;
        s2 += 65521u;
    }
    if (len) {
        while (len--) { s1 += buf[off++]; s2 += s1; }
        s1 %= 65521u;
        s2 %= 65521u;
    }
    return (int32_t)((uint32_t)s1 | ((uint32_t)s2 << 16));
}

static uint32_t crc_table0[256];
/* crc32.ts:179-214 (only table 0 is needed: slicing-by-4 is a pure speed-up).  The tables
 * are built once (pthread_once): the CPU baseline calls the oracle from many threads. */
static void crc_init_once(void) {
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
        crc_table0[n] = c;
    }
}
static pthread_once_t crc_once = PTHREAD_ONCE_INIT;
static void crc_init(void) { pthread_once(&crc_once, crc_init_once); }

/* crc32.ts:48-106: c = ~seed; reflected byte loop; return ~c as int32 */
int32_t oracle_crc32(const uint8_t* buf, size_t len, int32_t seed) {
    crc_init();
    uint32_t c = ~(uint32_t)seed;
    for (size_t i = 0; i < len; i++) c = crc_table0[(c ^ buf[i]) & 0xff] ^ (c >> 8);
    return (int32_t)~c;
}

/* ------------------------------------------------------------------------- */
/* common.ts:15-58                                                            */
/* ------------------------------------------------------------------------- */
enum { Z_OK = 0, Z_STREAM_END = 1, Z_NEED_DICT = 2, Z_STREAM_ERROR = -2, Z_DATA_ERROR = -3,
       Z_MEM_ERROR = -4, Z_BUF_ERROR = -5 };
static const uint32_t inflate_mask[17] = {
    0x0, 0x1, 0x3, 0x7, 0xf, 0x1f, 0x3f, 0x7f, 0xff, 0x1ff, 0x3ff, 0x7ff, 0xfff,
    0x1fff, 0x3fff, 0x7fff, 0xffff };

/* z.msg strings (Appendix B of SURVEY.md; sources cited per entry) */
enum {
    ZM_NONE = 0, ZM_INVALID_GZIP_ID, ZM_UNKNOWN_METHOD, ZM_INVALID_WINDOW, ZM_HEADER_CHECK,
    ZM_NEED_DICT, ZM_BLOCK_TYPE, ZM_STORED_LENS, ZM_TOO_MANY_SYMS, ZM_BL_REPEAT,
    ZM_BL_OVERSUB, ZM_BL_INCOMPLETE, ZM_LL_OVERSUB, ZM_LL_INCOMPLETE, ZM_D_OVERSUB,
    ZM_D_INCOMPLETE, ZM_D_EMPTY, ZM_INVALID_DIST, ZM_INVALID_LITLEN, ZM_COUNT
};
static const char* const zmsg_text[ZM_COUNT] = {
    "",
    "invalid gzip id",                          /* inflate.ts:169 */
    "unknown compression method",               /* inflate.ts:187 */
    "invalid window size",                      /* inflate.ts:192 */
    "incorrect header check",                   /* inflate.ts:216 */
    "need dictionary",                          /* inflate.ts:274 */
    "invalid block type",                       /* infblocks.ts:231 */
    "invalid stored block lengths",             /* infblocks.ts:263 */
    "too many length or distance symbols",      /* infblocks.ts:357 */
    "invalid bit length repeat",                /* infblocks.ts:505 */
    "oversubscribed dynamic bit lengths tree",  /* inftree.ts:325 */
    "incomplete dynamic bit lengths tree",      /* inftree.ts:327 */
    "oversubscribed literal/length tree",       /* inftree.ts:350 */
    "incomplete literal/length tree",           /* inftree.ts:353 */
    "oversubscribed distance tree",             /* inftree.ts:365 */
    "incomplete distance tree",                 /* inftree.ts:368 */
    "empty distance tree with lengths",         /* inftree.ts:372 */
    "invalid distance code",                    /* infcodes.ts:215,500 */
    "invalid literal/length code",              /* infcodes.ts:266,417 */
};
const char* oracle_zmsg(int32_t idx) {
    return (idx >= 0 && idx < ZM_COUNT) ? zmsg_text[idx] : "";
}

const char* oracle_error_message(int32_t err) {
    switch (err) {
    case ORA_OK: return "";
    case ORA_E_INFLATE_MSG: return "inflate error: ";
    case ORA_E_BAD_INPUT_DATA: return "inflate error: bad input data";
    case ORA_E_DICT_INVALID: return "Custom dictionary is not valid for this data";
    case ORA_E_DICT_REQUIRED: return "Custom dictionary required for this data";
    case ORA_E_UNEXPECTED_EOF: return "Unexpected EOF during decompression";
    case ORA_E_INTEGRITY: return "Data integrity check failed";
    case ORA_E_SIZE: return "Data size check failed";
    case ORA_E_DECOMPRESSION: return "Decompression error";
    case ORA_E_TOO_SMALL: return "data buffer is too small";
    case ORA_E_HANG: return "(reference loops forever: trailing input after end of stream)";
    case ORA_E_OUT_CAP: return "(oracle output capacity exceeded)";
    case ORA_E_FINISH_BEFORE_APPEND: return "Cannot call finish before at least 1 call to append";
    case ORA_E_PENDING_OVERFLOW: return "(reference indexes past pending_buf: undefined output)";
    default: return "(bad argument)";
    }
}

/* ------------------------------------------------------------------------- */
/* zstream.ts:19-95 (input side + a 16 KiB next_out)                          */
/* ------------------------------------------------------------------------- */
#define OUTPUT_BUFSIZE 16384
typedef struct {
    const uint8_t* next_in;
    int64_t avail_in;
    int64_t next_in_index;
    uint64_t total_in;
    uint8_t next_out[OUTPUT_BUFSIZE];
    int64_t avail_out;
    int64_t next_out_index;
    uint64_t total_out;
    int msg;
} zstream;

/* ------------------------------------------------------------------------- */
/* inftree.ts                                                                 */
/* ------------------------------------------------------------------------- */
#define BMAX 15
#define MANY 1400
static const int cplens[31] = { 3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35,
    43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258, 0, 0 };
static const int cplext[31] = { 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4,
    4, 4, 4, 5, 5, 5, 5, 0, 112, 112 };
static const int cpdist[30] = { 1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
    257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577 };
static const int cpdext[30] = { 0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9,
    9, 10, 10, 11, 11, 12, 12, 13, 13 };

/* module-level work area of inftree.ts:87-93 (the module is single-threaded) */
typedef struct {
    int32_t v[288];
    int32_t c[BMAX + 1];
    int32_t r[3];
    int32_t u[BMAX];
    int32_t x[BMAX + 1];
    int32_t hn;
} huft_work;

/* inftree.ts:301-311 */
static void init_work(huft_work* w) {
    memset(w->v, 0, sizeof w->v);
    memset(w->c, 0, sizeof w->c);
    memset(w->u, 0, sizeof w->u);
    memset(w->x, 0, sizeof w->x);
    memset(w->r, 0, sizeof w->r);
}

static void put3(int32_t* hp, int idx, const int32_t* r) {
    hp[idx * 3 + 0] = r[0];
    hp[idx * 3 + 1] = r[1];
    hp[idx * 3 + 2] = r[2];
}

/* inftree.ts:95-299 huft_build (zlib 1.1.3 multi-level tables of [op,bits,val]) */
static int huft_build(const uint8_t* b, int bindex, int n, int s, const int* d, const int* e,
                      int* t, int* m, int32_t* hp, huft_work* W) {
    int32_t* c = W->c; int32_t* r = W->r; int32_t* u = W->u; int32_t* x = W->x;
    int32_t* v = W->v;
    int a, f, g, h, i, j, k, l, mask, p, q, w, xp, y, z;

    p = 0; i = n;
    do { c[b[bindex + p]]++; p++; i--; } while (i != 0);
    if (c[0] == n) { *t = -1; *m = 0; return Z_OK; }

    l = *m;
    for (j = 1; j <= BMAX; j++) if (c[j] != 0) break;
    k = j;
    if (l < j) l = j;
    for (i = BMAX; i != 0; i--) if (c[i] != 0) break;
    g = i;
    if (l > i) l = i;
    *m = l;

    for (y = 1 << j; j < i; j++, y <<= 1) {
        y -= c[j];
        if (y < 0) return Z_DATA_ERROR;
    }
    y -= c[i];
    if (y < 0) return Z_DATA_ERROR;
    c[i] += y;

    x[1] = j = 0; p = 1; xp = 2;
    while (--i != 0) { x[xp] = (j += c[p]); xp++; p++; }

    i = 0; p = 0;
    do {
        j = b[bindex + p];
        if (j != 0) v[x[j]++] = i;
        p++;
    } while (++i < n);
    n = x[g];

    x[0] = i = 0; p = 0; h = -1; w = -l; u[0] = 0; q = 0; z = 0;
    for (; k <= g; k++) {
        a = c[k];
        while (a-- != 0) {
            while (k > w + l) {
                h++;
                w += l;
                z = g - w;
                z = (z > l) ? l : z;
                f = 1 << (j = k - w);
                if (f > a + 1) {
                    f -= a + 1;
                    xp = k;
                    if (j < z) {
                        while (++j < z) {
                            f <<= 1;
                            if (f <= c[++xp]) break;
                            f -= c[xp];
                        }
                    }
                }
                z = 1 << j;
                if (W->hn + z > MANY) return Z_DATA_ERROR;
                u[h] = q = W->hn;
                W->hn += z;
                if (h != 0) {
                    x[h] = i;
                    r[0] = j;
                    r[1] = l;
                    j = (int)((uint32_t)i >> (w - l));
                    r[2] = q - u[h - 1] - j;
                    put3(hp, u[h - 1] + j, r);
                } else {
                    *t = q;
                }
            }
            r[1] = k - w;
            if (p >= n) {
                r[0] = 128 + 64;
            } else if (v[p] < s) {
                r[0] = (v[p] < 256 ? 0 : 32 + 64);
                r[2] = v[p++];
            } else {
                r[0] = e[v[p] - s] + 16 + 64;
                r[2] = d[v[p++] - s];
            }
            f = 1 << (k - w);
            for (j = (int)((uint32_t)i >> w); j < z; j += f) put3(hp, q + j, r);
            for (j = 1 << (k - 1); (i & j) != 0; j = (int)((uint32_t)j >> 1)) i ^= j;
            i ^= j;
            mask = (1 << w) - 1;
            while ((i & mask) != x[h]) {
                h--;
                w -= l;
                mask = (1 << w) - 1;
            }
        }
    }
    return (y != 0 && g != 1) ? Z_BUF_ERROR : Z_OK;
}

/* inftree.ts:313-331 */
static int inflate_trees_bits(const uint8_t* cl, int* bb, int* tb, int32_t* hp, zstream* zs,
                              huft_work* W) {
    init_work(W);
    W->hn = 0;
    int result = huft_build(cl, 0, 19, 19, NULL, NULL, tb, bb, hp, W);
    if (result == Z_DATA_ERROR) {
        zs->msg = ZM_BL_OVERSUB;
    } else if (result == Z_BUF_ERROR || *bb == 0) {
        zs->msg = ZM_BL_INCOMPLETE;
        result = Z_DATA_ERROR;
    }
    return result;
}

/* inftree.ts:333-379 */
static int inflate_trees_dynamic(int nl, int nd, const uint8_t* cl, int* bl, int* bd, int* tl,
                                 int* td, int32_t* hp, zstream* zs, huft_work* W) {
    init_work(W);
    W->hn = 0;
    int result = huft_build(cl, 0, nl, 257, cplens, cplext, tl, bl, hp, W);
    if (result != Z_OK || *bl == 0) {
        if (result == Z_DATA_ERROR) zs->msg = ZM_LL_OVERSUB;
        else { zs->msg = ZM_LL_INCOMPLETE; result = Z_DATA_ERROR; }
        return result;
    }
    init_work(W);
    result = huft_build(cl, nl, nd, 0, cpdist, cpdext, td, bd, hp, W);
    if (result != Z_OK || (*bd == 0 && nl > 257)) {
        if (result == Z_DATA_ERROR) zs->msg = ZM_D_OVERSUB;
        else if (result == Z_BUF_ERROR) { zs->msg = ZM_D_INCOMPLETE; result = Z_DATA_ERROR; }
        else { zs->msg = ZM_D_EMPTY; result = Z_DATA_ERROR; }
        return result;
    }
    return Z_OK;
}

/* inftree.ts:16-63 + 381-392: the fixed tables are the huft_build output for the
 * fixed code (zlib 1.1.3 inffixed.h); regenerated here, spot-checked in tests. */
static int32_t fixed_tl[512 * 3];
static int32_t fixed_td[32 * 3];
static void fixed_init_once(void) {
    uint8_t lens[288];
    huft_work W;
    int t, m;
    for (int i = 0; i < 144; i++) lens[i] = 8;
    for (int i = 144; i < 256; i++) lens[i] = 9;
    for (int i = 256; i < 280; i++) lens[i] = 7;
    for (int i = 280; i < 288; i++) lens[i] = 8;
    init_work(&W); W.hn = 0; m = 9;
    huft_build(lens, 0, 288, 257, cplens, cplext, &t, &m, fixed_tl, &W);
    for (int i = 0; i < 30; i++) lens[i] = 5;
    init_work(&W); W.hn = 0; m = 5;
    huft_build(lens, 0, 30, 0, cpdist, cpdext, &t, &m, fixed_td, &W);
}
static pthread_once_t fixed_once = PTHREAD_ONCE_INIT;
static void fixed_init(void) { pthread_once(&fixed_once, fixed_init_once); }

/* exported for the fixed-table spot check in tests */
int32_t oracle_fixed_table_entry(int which, int idx) {
    fixed_init();
    return which == 0 ? fixed_tl[idx] : fixed_td[idx];
}

/* ------------------------------------------------------------------------- */
/* infcodes.ts                                                                */
/* ------------------------------------------------------------------------- */
enum { C_START = 0, C_LEN, C_LENEXT, C_DIST, C_DISTEXT, C_COPY, C_LIT, C_WASH, C_END, C_BADCODE };

typedef struct {
    int mode;
    int len;
    const int32_t* tree; int tree_index;
    int need;
    int lit;
    int get;
    int dist;
    int lbits, dbits;
    const int32_t* ltree; int ltree_index;
    const int32_t* dtree; int dtree_index;
} infcodes;

#define WIN_END 32768
typedef struct {
    int mode;
    uint32_t bitb; int bitk;
    uint8_t window[WIN_END];
    int end;
    int read, write;
    int last;
    int32_t hufts[MANY * 3];
    infcodes codes;
    huft_work work;
} infblocks;

/* infblocks.ts:61-121 */
static int inflate_flush(infblocks* s, zstream* z, int r) {
    int64_t p = z->next_out_index;
    int q = s->read;
    int64_t n = (q <= s->write ? s->write : s->end) - q;
    if (n > z->avail_out) n = z->avail_out;
    if (n != 0 && r == Z_BUF_ERROR) r = Z_OK;
    z->avail_out -= n;
    z->total_out += (uint64_t)n;
    memcpy(z->next_out + p, s->window + q, (size_t)n);
    p += n; q += (int)n;
    if (q == s->end) {
        q = 0;
        if (s->write == s->end) s->write = 0;
        n = s->write - q;
        if (n > z->avail_out) n = z->avail_out;
        if (n != 0 && r == Z_BUF_ERROR) r = Z_OK;
        z->avail_out -= n;
        z->total_out += (uint64_t)n;
        memcpy(z->next_out + p, s->window + q, (size_t)n);
        p += n; q += (int)n;
    }
    z->next_out_index = p;
    s->read = q;
    return r;
}

#define WMAX(s, q) ((q) < (s)->read ? (s)->read - (q) - 1 : (s)->end - (q))
#define INB(z, p) ((uint32_t)((p) < (int64_t)0 ? 0 : (z)->next_in[(p)]))

/* infcodes.ts:62-301 inflate_fast (entered with m >= 258 && n >= 10) */
static int inflate_fast(int bl, int bd, const int32_t* tl, int tl_index, const int32_t* td,
                        int td_index, infblocks* s, zstream* z) {
    int t, e, k, q, m, c, d, r, tpi3, tp_index;
    const int32_t* tp;
    uint32_t b, ml, md;
    int64_t p, n;

    p = z->next_in_index; n = z->avail_in;
    b = s->bitb; k = s->bitk;
    q = s->write; m = WMAX(s, q);
    ml = inflate_mask[bl]; md = inflate_mask[bd];

    do {
        while (k < 20) { n--; b |= INB(z, p) << k; p++; k += 8; }
        t = (int)(b & ml);
        tp = tl; tp_index = tl_index;
        tpi3 = (tp_index + t) * 3;
        e = tp[tpi3];
        if (e == 0) {
            b >>= tp[tpi3 + 1]; k -= tp[tpi3 + 1];
            s->window[q++] = (uint8_t)tp[tpi3 + 2];
            m--;
            continue;
        }
        for (;;) {
            b >>= tp[tpi3 + 1]; k -= tp[tpi3 + 1];
            if ((e & 16) != 0) {
                e &= 15;
                c = tp[tpi3 + 2] + (int)(b & inflate_mask[e]);
                b >>= e; k -= e;
                while (k < 15) { n--; b |= INB(z, p) << k; p++; k += 8; }
                t = (int)(b & md);
                tp = td; tp_index = td_index;
                tpi3 = (tp_index + t) * 3;
                e = tp[tpi3];
                for (;;) {
                    b >>= tp[tpi3 + 1]; k -= tp[tpi3 + 1];
                    if ((e & 16) != 0) {
                        e &= 15;
                        while (k < e) { n--; b |= INB(z, p) << k; p++; k += 8; }
                        d = tp[tpi3 + 2] + (int)(b & inflate_mask[e]);
                        b >>= e; k -= e;
                        m -= c;
                        if (q >= d) {
                            r = q - d;
                            s->window[q++] = s->window[r++];
                            s->window[q++] = s->window[r++];
                            c -= 2;
                        } else {
                            r = q - d;
                            do { r += s->end; } while (r < 0);
                            e = s->end - r;
                            if (c > e) {
                                c -= e;
                                do { s->window[q++] = s->window[r++]; } while (--e != 0);
                                r = 0;
                            }
                        }
                        do { s->window[q++] = s->window[r++]; } while (--c != 0);
                        break;
                    } else if ((e & 64) == 0) {
                        t += tp[tpi3 + 2];
                        t += (int)(b & inflate_mask[e]);
                        tpi3 = (tp_index + t) * 3;
                        e = tp[tpi3];
                    } else {
                        z->msg = ZM_INVALID_DIST;
                        c = (int)(z->avail_in - n);
                        c = (k >> 3) < c ? k >> 3 : c;
                        n += c; p -= c; k -= c << 3;
                        s->bitb = b; s->bitk = k;
                        z->avail_in = n; z->total_in += (uint64_t)(p - z->next_in_index);
                        z->next_in_index = p; s->write = q;
                        return Z_DATA_ERROR;
                    }
                }
                break;
            }
            if ((e & 64) == 0) {
                t += tp[tpi3 + 2];
                t += (int)(b & inflate_mask[e]);
                tpi3 = (tp_index + t) * 3;
                e = tp[tpi3];
                if (e == 0) {
                    b >>= tp[tpi3 + 1]; k -= tp[tpi3 + 1];
                    s->window[q++] = (uint8_t)tp[tpi3 + 2];
                    m--;
                    break;
                }
            } else if ((e & 32) != 0) {
                c = (int)(z->avail_in - n);
                c = (k >> 3) < c ? k >> 3 : c;
                n += c; p -= c; k -= c << 3;
                s->bitb = b; s->bitk = k;
                z->avail_in = n; z->total_in += (uint64_t)(p - z->next_in_index);
                z->next_in_index = p; s->write = q;
                return Z_STREAM_END;
            } else {
                z->msg = ZM_INVALID_LITLEN;
                c = (int)(z->avail_in - n);
                c = (k >> 3) < c ? k >> 3 : c;
                n += c; p -= c; k -= c << 3;
                s->bitb = b; s->bitk = k;
                z->avail_in = n; z->total_in += (uint64_t)(p - z->next_in_index);
                z->next_in_index = p; s->write = q;
                return Z_DATA_ERROR;
            }
        }
    } while (m >= 258 && n >= 10);

    c = (int)(z->avail_in - n);
    c = (k >> 3) < c ? k >> 3 : c;
    n += c; p -= c; k -= c << 3;
    s->bitb = b; s->bitk = k;
    z->avail_in = n; z->total_in += (uint64_t)(p - z->next_in_index);
    z->next_in_index = p; s->write = q;
    return Z_OK;
}

/* infcodes.ts:303-312 */
static void codes_init(infcodes* C, int bl, int bd, const int32_t* tl, int tl_index,
                       const int32_t* td, int td_index) {
    C->mode = C_START;
    C->lbits = bl; C->dbits = bd;
    C->ltree = tl; C->ltree_index = tl_index;
    C->dtree = td; C->dtree_index = td_index;
}

/* save the UPDATE locals back and flush (the recurring exit of infcodes/infblocks) */
#define SAVE_STATE()                                                        \
    do {                                                                    \
        s->bitb = b; s->bitk = k; z->avail_in = n;                          \
        z->total_in += (uint64_t)(p - z->next_in_index);                    \
        z->next_in_index = p; s->write = q;                                 \
    } while (0)
#define LEAVE() do { SAVE_STATE(); return inflate_flush(s, z, r); } while (0)
#define NEEDBYTE_OR_LEAVE()                                                 \
    do { if (n != 0) r = Z_OK; else LEAVE(); } while (0)
#define NEXTBYTE() do { n--; b |= (uint32_t)z->next_in[p++] << k; k += 8; } while (0)

/* infcodes.ts:314-676 */
static int codes_proc(infcodes* C, infblocks* s, zstream* z, int r) {
    int j, tindex, e, q, m, f;
    uint32_t b; int k;
    int64_t p, n;

    p = z->next_in_index; n = z->avail_in;
    b = s->bitb; k = s->bitk;
    q = s->write; m = WMAX(s, q);

    for (;;) {
        switch (C->mode) {
        case C_START:
            if (m >= 258 && n >= 10) {
                SAVE_STATE();
                r = inflate_fast(C->lbits, C->dbits, C->ltree, C->ltree_index, C->dtree,
                                 C->dtree_index, s, z);
                p = z->next_in_index; n = z->avail_in;
                b = s->bitb; k = s->bitk;
                q = s->write; m = WMAX(s, q);
                if (r != Z_OK) {
                    C->mode = (r == Z_STREAM_END) ? C_WASH : C_BADCODE;
                    break;
                }
            }
            C->need = C->lbits;
            C->tree = C->ltree; C->tree_index = C->ltree_index;
            C->mode = C_LEN;
            /* fall through */
        case C_LEN:
            j = C->need;
            while (k < j) { NEEDBYTE_OR_LEAVE(); NEXTBYTE(); }
            tindex = (C->tree_index + (int)(b & inflate_mask[j])) * 3;
            b >>= C->tree[tindex + 1]; k -= C->tree[tindex + 1];
            e = C->tree[tindex];
            if (e == 0) { C->lit = C->tree[tindex + 2]; C->mode = C_LIT; break; }
            if ((e & 16) != 0) { C->get = e & 15; C->len = C->tree[tindex + 2]; C->mode = C_LENEXT; break; }
            if ((e & 64) == 0) { C->need = e; C->tree_index = tindex / 3 + C->tree[tindex + 2]; break; }
            if ((e & 32) != 0) { C->mode = C_WASH; break; }
            C->mode = C_BADCODE;
            z->msg = ZM_INVALID_LITLEN;
            r = Z_DATA_ERROR;
            LEAVE();
        case C_LENEXT:
            j = C->get;
            while (k < j) { NEEDBYTE_OR_LEAVE(); NEXTBYTE(); }
            C->len += (int)(b & inflate_mask[j]);
            b >>= j; k -= j;
            C->need = C->dbits;
            C->tree = C->dtree; C->tree_index = C->dtree_index;
            C->mode = C_DIST;
            /* fall through */
        case C_DIST:
            j = C->need;
            while (k < j) { NEEDBYTE_OR_LEAVE(); NEXTBYTE(); }
            tindex = (C->tree_index + (int)(b & inflate_mask[j])) * 3;
            b >>= C->tree[tindex + 1]; k -= C->tree[tindex + 1];
            e = C->tree[tindex];
            if ((e & 16) != 0) { C->get = e & 15; C->dist = C->tree[tindex + 2]; C->mode = C_DISTEXT; break; }
            if ((e & 64) == 0) { C->need = e; C->tree_index = tindex / 3 + C->tree[tindex + 2]; break; }
            C->mode = C_BADCODE;
            z->msg = ZM_INVALID_DIST;
            r = Z_DATA_ERROR;
            LEAVE();
        case C_DISTEXT:
            j = C->get;
            while (k < j) { NEEDBYTE_OR_LEAVE(); NEXTBYTE(); }
            C->dist += (int)(b & inflate_mask[j]);
            b >>= j; k -= j;
            C->mode = C_COPY;
            /* fall through */
        case C_COPY:
            f = q - C->dist;
            while (f < 0) f += s->end;
            while (C->len != 0) {
                if (m == 0) {
                    if (q == s->end && s->read != 0) { q = 0; m = WMAX(s, q); }
                    if (m == 0) {
                        s->write = q;
                        r = inflate_flush(s, z, r);
                        q = s->write; m = WMAX(s, q);
                        if (q == s->end && s->read != 0) { q = 0; m = WMAX(s, q); }
                        if (m == 0) LEAVE();
                    }
                }
                s->window[q++] = s->window[f++];
                m--;
                if (f == s->end) f = 0;
                C->len--;
            }
            C->mode = C_START;
            break;
        case C_LIT:
            if (m == 0) {
                if (q == s->end && s->read != 0) { q = 0; m = WMAX(s, q); }
                if (m == 0) {
                    s->write = q;
                    r = inflate_flush(s, z, r);
                    q = s->write; m = WMAX(s, q);
                    if (q == s->end && s->read != 0) { q = 0; m = WMAX(s, q); }
                    if (m == 0) LEAVE();
                }
            }
            r = Z_OK;
            s->window[q++] = (uint8_t)C->lit;
            m--;
            C->mode = C_START;
            break;
        case C_WASH:
            if (k > 7) { k -= 8; n++; p--; }
            s->write = q;
            r = inflate_flush(s, z, r);
            q = s->write; m = WMAX(s, q);
            if (s->read != s->write) LEAVE();
            C->mode = C_END;
            /* fall through */
        case C_END:
            r = Z_STREAM_END;
            LEAVE();
        case C_BADCODE:
            r = Z_DATA_ERROR;
            LEAVE();
        default:
            r = Z_STREAM_ERROR;
            LEAVE();
        }
    }
}

/* ------------------------------------------------------------------------- */
/* infblocks.ts                                                               */
/* ------------------------------------------------------------------------- */
enum { B_TYPE = 0, B_LENS, B_STORED, B_TABLE, B_BTREE, B_DTREE, B_CODES, B_DRY, B_DONELOCKS,
       B_BADBLOCKS };
static const int border[19] = { 16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15 };

/* infblocks.ts:52-58 */
static void blocks_reset(infblocks* s) {
    s->bitk = 0; s->bitb = 0; s->read = 0; s->write = 0; s->last = 0;
}

/* infblocks.ts:123-628.  left/table/index/blens/bb/tb are proc-locals exactly as
 * in the reference (they do not survive a return). */
static int blocks_proc(infblocks* s, zstream* z, int r) {
    int t, i, q, m;
    uint32_t b; int k;
    int64_t p, n;
    int left = 0, table = 0, index = 0;
    uint8_t blens[320];
    int bb = 0, tb = 0;
    infcodes* codes = &s->codes;
    int32_t* hufts = s->hufts;
    memset(blens, 0, sizeof blens);

    p = z->next_in_index; n = z->avail_in;
    b = s->bitb; k = s->bitk;
    q = s->write; m = WMAX(s, q);

    for (;;) {
        switch (s->mode) {
        case B_TYPE:
            if (s->last) return Z_STREAM_END;
            while (k < 3) { NEEDBYTE_OR_LEAVE(); NEXTBYTE(); }
            t = (int)(b & 7);
            s->last = t & 1;
            switch (t >> 1) {
            case 0:
                b >>= 3; k -= 3;
                t = k & 7;
                b >>= t; k -= t;
                s->mode = B_LENS;
                break;
            case 1:
                fixed_init();
                codes_init(codes, 9, 5, fixed_tl, 0, fixed_td, 0);
                b >>= 3; k -= 3;
                s->mode = B_CODES;
                break;
            case 2:
                b >>= 3; k -= 3;
                s->mode = B_TABLE;
                break;
            case 3:
                b >>= 3; k -= 3;
                s->mode = B_BADBLOCKS;
                z->msg = ZM_BLOCK_TYPE;
                r = Z_DATA_ERROR;
                LEAVE();
            }
            break;
        case B_LENS:
            while (k < 32) { NEEDBYTE_OR_LEAVE(); NEXTBYTE(); }
            if ((((~b) >> 16) & 0xffff) != (b & 0xffff)) {
                s->mode = B_BADBLOCKS;
                z->msg = ZM_STORED_LENS;
                r = Z_DATA_ERROR;
                LEAVE();
            }
            left = (int)(b & 0xffff);
            b = 0; k = 0;
            s->mode = left != 0 ? B_STORED : (s->last != 0 ? B_DRY : B_TYPE);
            break;
        case B_STORED:
            if (n == 0) LEAVE();
            if (m == 0) {
                if (q == s->end && s->read != 0) { q = 0; m = WMAX(s, q); }
                if (m == 0) {
                    s->write = q;
                    r = inflate_flush(s, z, r);
                    q = s->write; m = WMAX(s, q);
                    if (q == s->end && s->read != 0) { q = 0; m = WMAX(s, q); }
                    if (m == 0) LEAVE();
                }
            }
            r = Z_OK;
            t = left;
            if (t > n) t = (int)n;
            if (t > m) t = m;
            memcpy(s->window + q, z->next_in + p, (size_t)t);
            p += t; n -= t; q += t; m -= t; left -= t;
            if (left != 0) break;
            s->mode = s->last != 0 ? B_DRY : B_TYPE;
            break;
        case B_TABLE:
            while (k < 14) { NEEDBYTE_OR_LEAVE(); NEXTBYTE(); }
            table = t = (int)(b & 0x3fff);
            if ((t & 0x1f) > 29 || ((t >> 5) & 0x1f) > 29) {
                s->mode = B_BADBLOCKS;
                z->msg = ZM_TOO_MANY_SYMS;
                r = Z_DATA_ERROR;
                LEAVE();
            }
            t = 258 + (t & 0x1f) + ((t >> 5) & 0x1f);
            for (i = 0; i < t; i++) blens[i] = 0;
            b >>= 14; k -= 14;
            index = 0;
            s->mode = B_BTREE;
            /* infblocks.ts:380: falls through into the BTREE body (no case label) */
            while (index < 4 + (table >> 10)) {
                while (k < 3) { NEEDBYTE_OR_LEAVE(); NEXTBYTE(); }
                blens[border[index++]] = (uint8_t)(b & 7);
                b >>= 3; k -= 3;
            }
            while (index < 19) blens[border[index++]] = 0;
            bb = 7;
            t = inflate_trees_bits(blens, &bb, &tb, hufts, z, &s->work);
            if (t != Z_OK) {
                r = t;
                if (r == Z_DATA_ERROR) s->mode = B_BADBLOCKS;
                LEAVE();
            }
            index = 0;
            s->mode = B_DTREE;
            /* DTREE body (no case label) */
            for (;;) {
                int j, c;
                t = table;
                if (index >= 258 + (t & 0x1f) + ((t >> 5) & 0x1f)) break;
                t = bb;
                while (k < t) { NEEDBYTE_OR_LEAVE(); NEXTBYTE(); }
                {
                    int ti = (tb + (int)(b & inflate_mask[t])) * 3;
                    t = hufts[ti + 1];
                    c = hufts[ti + 2];
                }
                if (c < 16) {
                    b >>= t; k -= t;
                    blens[index++] = (uint8_t)c;
                } else {
                    i = c == 18 ? 7 : c - 14;
                    j = c == 18 ? 11 : 3;
                    while (k < t + i) { NEEDBYTE_OR_LEAVE(); NEXTBYTE(); }
                    b >>= t; k -= t;
                    j += (int)(b & inflate_mask[i]);
                    b >>= i; k -= i;
                    i = index;
                    t = table;
                    if (i + j > 258 + (t & 0x1f) + ((t >> 5) & 0x1f) || (c == 16 && i < 1)) {
                        s->mode = B_BADBLOCKS;
                        z->msg = ZM_BL_REPEAT;
                        r = Z_DATA_ERROR;
                        LEAVE();
                    }
                    c = c == 16 ? blens[i - 1] : 0;
                    do { blens[i++] = (uint8_t)c; } while (--j != 0);
                    index = i;
                }
            }
            tb = -1;
            {
                int bl_ = 9, bd_ = 6, tl_ = 0, td_ = 0;
                t = inflate_trees_dynamic(257 + (t & 0x1f), 1 + ((t >> 5) & 0x1f), blens, &bl_,
                                          &bd_, &tl_, &td_, hufts, z, &s->work);
                if (t != Z_OK) {
                    if (t == Z_DATA_ERROR) s->mode = B_BADBLOCKS;
                    r = t;
                    LEAVE();
                }
                codes_init(codes, bl_, bd_, hufts, tl_, hufts, td_);
            }
            s->mode = B_CODES;
            /* fall through */
        case B_CODES:
            SAVE_STATE();
            r = codes_proc(codes, s, z, r);
            if (r != Z_STREAM_END) return inflate_flush(s, z, r);
            r = Z_OK;
            p = z->next_in_index; n = z->avail_in;
            b = s->bitb; k = s->bitk;
            q = s->write; m = WMAX(s, q);
            if (s->last == 0) { s->mode = B_TYPE; break; }
            s->mode = B_DRY;
            /* fall through */
        case B_DRY:
            s->write = q;
            r = inflate_flush(s, z, r);
            q = s->write; m = WMAX(s, q);
            if (s->read != s->write) LEAVE();
            s->mode = B_DONELOCKS;
            /* fall through */
        case B_DONELOCKS:
            r = Z_STREAM_END;
            LEAVE();
        case B_BADBLOCKS:
            r = Z_DATA_ERROR;
            LEAVE();
        default:  /* includes BTREE / DTREE: no case label */
            r = Z_STREAM_ERROR;
            LEAVE();
        }
    }
}

/* infblocks.ts:630-633 */
static void blocks_set_dictionary(infblocks* s, const uint8_t* d, size_t start, size_t n) {
    memcpy(s->window, d + start, n);
    s->read = s->write = (int)n;
}

/* ------------------------------------------------------------------------- */
/* inflate.ts                                                                 */
/* ------------------------------------------------------------------------- */
enum { M_DETECT = 0, M_ID2, M_METHOD, M_FLAG, M_DICT4, M_DICT3, M_DICT2, M_DICT1, M_DICT0,
       M_MTIME0, M_MTIME1, M_MTIME2, M_MTIME3, M_XFLAGS, M_OS, M_EXTRA0, M_EXTRA1, M_EXTRA,
       M_NAME, M_COMMENT, M_HCRC0, M_HCRC1, M_BLOCKS, M_CHKSUM0, M_CHKSUM1, M_CHKSUM2,
       M_CHKSUM3, M_ISIZE0, M_ISIZE1, M_ISIZE2, M_ISIZE3, M_DONE, M_BAD };
enum { G_FTEXT = 1, G_FHCRC = 2, G_FEXTRA = 4, G_FNAME = 8, G_FCOMMENT = 16 };

typedef struct {
    int mode;
    int is_gzip;
    int method;
    int gflags;
    char name[256]; int name_len;
    int32_t mtime;
    uint32_t xlen;
    int32_t dict_checksum;
    int32_t full_checksum;
    int32_t inflated_size;
    int wbits;
    infblocks blocks;
} inflate_state;

/* inflate.ts:97-101 */
static void inflate_ctor(inflate_state* st, int blocks_only) {
    memset(st, 0, sizeof *st);
    st->wbits = 15;
    st->blocks.end = 1 << st->wbits;
    st->blocks.mode = B_TYPE;
    st->mode = blocks_only ? M_BLOCKS : M_DETECT;
}

/* inflate.ts:103-107 */
static int inflate_is_complete(const inflate_state* st) {
    const infblocks* bl = &st->blocks;
    int blocks_complete = (bl->mode == B_TYPE || bl->mode == B_DONELOCKS) && bl->bitb == 0 &&
                          bl->bitk == 0;
    return st->mode == M_DONE && blocks_complete;
}

/* inflate.ts:128-130: 0 raw, 1 deflate, 2 gzip */
static int inflate_container(const inflate_state* st) {
    return st->is_gzip ? 2 : (st->method == 0 ? 0 : 1);
}

#define ZIN_BYTE() (z->avail_in--, z->total_in++, z->next_in[z->next_in_index++])

/* inflate.ts:132-473 */
static int inflate_run(inflate_state* st, zstream* z) {
    uint32_t bt;
    const int f = Z_OK;
    int r = Z_BUF_ERROR;
    if (!z->next_in) return Z_STREAM_ERROR;
    for (;;) {
        switch (st->mode) {
        case M_DETECT:
            if (z->avail_in == 0) return r;
            bt = z->next_in[z->next_in_index];
            if (bt != 0x1f) { st->mode = M_METHOD; break; }
            st->mode = M_ID2;
            r = f;
            z->avail_in--; z->total_in++; z->next_in_index++;
            /* fall through */
        case M_ID2:
            if (z->avail_in == 0) return r;
            r = f;
            bt = ZIN_BYTE();
            if (bt != 0x8b) { st->mode = M_BAD; z->msg = ZM_INVALID_GZIP_ID; break; }
            st->is_gzip = 1;
            st->mode = M_METHOD;
            /* fall through */
        case M_METHOD:
            if (z->avail_in == 0) return r;
            r = f;
            st->method = ZIN_BYTE();
            if ((st->method & 0xf) != 8) { st->mode = M_BAD; z->msg = ZM_UNKNOWN_METHOD; break; }
            if ((st->method >> 4) + 8 > st->wbits) { st->mode = M_BAD; z->msg = ZM_INVALID_WINDOW; break; }
            st->mode = M_FLAG;
            /* fall through */
        case M_FLAG:
            if (z->avail_in == 0) return r;
            r = f;
            bt = ZIN_BYTE() & 0xff;
            if (st->is_gzip) { st->gflags = (int)bt; st->mode = M_MTIME0; break; }
            if ((((st->method << 8) + (int)bt) % 31) != 0) {
                st->mode = M_BAD; z->msg = ZM_HEADER_CHECK; break;
            }
            if ((bt & 0x20) == 0) { st->mode = M_BLOCKS; break; }
            st->mode = M_DICT4;
            /* fall through */
        case M_DICT4:
            if (z->avail_in == 0) return r;
            r = f;
            st->dict_checksum = (int32_t)(((uint32_t)ZIN_BYTE() << 24) & 0xff000000u);
            st->mode = M_DICT3;
            /* fall through */
        case M_DICT3:
            if (z->avail_in == 0) return r;
            r = f;
            st->dict_checksum |= (int32_t)(((uint32_t)ZIN_BYTE() << 16) & 0xff0000u);
            st->mode = M_DICT2;
            /* fall through */
        case M_DICT2:
            if (z->avail_in == 0) return r;
            r = f;
            st->dict_checksum |= (int32_t)(((uint32_t)ZIN_BYTE() << 8) & 0xff00u);
            st->mode = M_DICT1;
            /* fall through */
        case M_DICT1:
            if (z->avail_in == 0) return r;
            r = f;
            st->dict_checksum |= (int32_t)ZIN_BYTE();
            st->mode = M_DICT0;
            return Z_NEED_DICT;
        case M_DICT0:
            st->mode = M_BAD;
            z->msg = ZM_NEED_DICT;
            return Z_STREAM_ERROR;
        case M_MTIME0: case M_MTIME1: case M_MTIME2: case M_MTIME3:
            if (z->avail_in == 0) return r;
            r = f;
            bt = ZIN_BYTE() & 0xff;
            st->mtime = (int32_t)(((uint32_t)st->mtime >> 8) | (bt << 24));
            if (st->mode != M_MTIME3) { st->mode++; break; }
            st->mode = M_XFLAGS;
            /* fall through */
        case M_XFLAGS: case M_OS: case M_HCRC0: case M_HCRC1:
            if (z->avail_in == 0) return r;
            r = f;
            z->avail_in--; z->total_in++; z->next_in_index++;
            if (st->mode == M_OS) {
                if (st->gflags & G_FEXTRA) st->mode = M_EXTRA0;
                else if (st->gflags & G_FNAME) st->mode = M_NAME;
                else if (st->gflags & G_FCOMMENT) st->mode = M_COMMENT;
                else if (st->gflags & G_FHCRC) st->mode = M_HCRC0;
                else st->mode = M_BLOCKS;
            } else {
                st->mode++;
            }
            break;
        case M_EXTRA0: case M_EXTRA1:
            if (z->avail_in == 0) return r;
            r = f;
            bt = ZIN_BYTE() & 0xff;
            st->xlen = (st->xlen >> 8) | (bt << 24);
            /* inflate.ts:343-345 breaks out of EXTRA0 without advancing the mode, so
             * an FEXTRA header swallows the rest of the input (reference defect). */
            if (st->mode == M_EXTRA0) break;
            st->xlen = st->xlen >> 16;
            st->mode = M_EXTRA;
            /* fall through */
        case M_EXTRA:
            if (z->avail_in == 0) return r;
            r = f;
            z->avail_in--; z->total_in++; z->next_in_index++;
            st->xlen--;
            if (st->xlen == 0) {
                if (st->gflags & G_FNAME) st->mode = M_NAME;
                else if (st->gflags & G_FCOMMENT) st->mode = M_COMMENT;
                else if (st->gflags & G_FHCRC) st->mode = M_HCRC0;
                else st->mode = M_BLOCKS;
            }
            break;
        case M_NAME: case M_COMMENT:
            if (z->avail_in == 0) return r;
            r = f;
            bt = ZIN_BYTE() & 0xff;
            if (bt != 0) {
                if (st->mode == M_NAME && st->name_len < 255) st->name[st->name_len++] = (char)bt;
            } else {
                if (st->mode != M_COMMENT && (st->gflags & G_FCOMMENT)) st->mode = M_COMMENT;
                else if (st->gflags & G_FHCRC) st->mode = M_HCRC0;
                else st->mode = M_BLOCKS;
            }
            break;
        case M_BLOCKS:
            r = blocks_proc(&st->blocks, z, r);
            if (r == Z_DATA_ERROR) { st->mode = M_BAD; break; }
            if (r != Z_STREAM_END) return r;
            r = f;
            blocks_reset(&st->blocks);
            if (st->method == 0) { st->mode = M_DONE; break; }
            st->mode = M_CHKSUM0;
            /* fall through */
        case M_CHKSUM0: case M_CHKSUM1: case M_CHKSUM2: case M_CHKSUM3:
            if (z->avail_in == 0) return r;
            r = f;
            bt = ZIN_BYTE() & 0xff;
            if (st->is_gzip) st->full_checksum = (int32_t)(((uint32_t)st->full_checksum >> 8) | (bt << 24));
            else st->full_checksum = (int32_t)(((uint32_t)st->full_checksum << 8) | bt);
            st->mode++;
            if (st->mode == M_ISIZE0 && !st->is_gzip) st->mode = M_DONE;
            break;
        case M_ISIZE0: case M_ISIZE1: case M_ISIZE2: case M_ISIZE3:
            if (z->avail_in == 0) return r;
            r = f;
            bt = ZIN_BYTE() & 0xff;
            st->inflated_size = (int32_t)(((uint32_t)st->inflated_size >> 8) | (bt << 24));
            st->mode++;
            break;
        case M_DONE:
            return Z_STREAM_END;
        case M_BAD:
            return Z_DATA_ERROR;
        default:
            return Z_STREAM_ERROR;
        }
    }
}

/* inflate.ts:475-503 (dictionary checksum via adler32.ts) */
static int inflate_set_dictionary(inflate_state* st, const uint8_t* dict, size_t dict_len) {
    if (st->mode != M_DICT0) return Z_STREAM_ERROR;
    size_t index = 0, length = dict_len;
    if (length >= ((size_t)1 << st->wbits)) {
        length = ((size_t)1 << st->wbits) - 1;
        index = dict_len - length;
    }
    int32_t cs = oracle_adler32(dict, dict_len, 1);
    if (cs != st->dict_checksum) return Z_DATA_ERROR;
    blocks_set_dictionary(&st->blocks, dict, index, length);
    st->mode = M_BLOCKS;
    return Z_OK;
}

/* ------------------------------------------------------------------------- */
/* sd-inflate.ts: Inflater (54-180) and inflate() (189-228)                   */
/* ------------------------------------------------------------------------- */
typedef struct {
    inflate_state inf;
    zstream z;
    const uint8_t* dict; size_t dict_len; int has_dict;
    int have_checksum;
    int32_t checksum;
} inflater;

int32_t oracle_inflater_run(const uint8_t* const* parts, const size_t* part_lens, int32_t nparts,
                            int32_t raw, const uint8_t* dict, size_t dict_len,
                            uint8_t* out, size_t out_cap, oracle_inflate_result* res) {
    return oracle_inflater_run_parts(parts, part_lens, nparts, raw, dict, dict_len, out, out_cap, res,
                                     NULL, NULL);
}

int32_t oracle_inflater_run_parts(const uint8_t* const* parts, const size_t* part_lens, int32_t nparts,
                                  int32_t raw, const uint8_t* dict, size_t dict_len,
                                  uint8_t* out, size_t out_cap, oracle_inflate_result* res,
                                  size_t* part_out, int32_t* err_part) {
    return oracle_inflater_run_chunks(parts, part_lens, nparts, raw, dict, dict_len, out, out_cap, res,
                                      part_out, err_part, NULL, NULL, 0, NULL);
}

int32_t oracle_inflater_run_chunks(const uint8_t* const* parts, const size_t* part_lens, int32_t nparts,
                                   int32_t raw, const uint8_t* dict, size_t dict_len,
                                   uint8_t* out, size_t out_cap, oracle_inflate_result* res,
                                   size_t* part_out, int32_t* err_part,
                                   size_t* chunk_sz, int32_t* chunk_part, size_t chunk_cap, size_t* nchunks) {
    memset(res, 0, sizeof *res);
    if (nchunks) *nchunks = 0;
    if (err_part) *err_part = -1;
    if (part_out) for (int32_t k = 0; k < nparts; k++) part_out[k] = 0;
    if (raw && dict) { res->error = ORA_E_BAD_ARG; return res->error; }
    inflater* I = (inflater*)calloc(1, sizeof(inflater));
    if (!I) { res->error = ORA_E_BAD_ARG; return res->error; }
    inflate_ctor(&I->inf, raw ? 1 : 0);
    I->dict = dict; I->dict_len = dict_len; I->has_dict = dict != NULL;
    zstream* z = &I->z;
    size_t out_len = 0;
    int32_t err_code = ORA_OK;

    int pi = 0;
    for (; pi < nparts && err_code == ORA_OK; pi++) {
        size_t out_before = out_len;
        const uint8_t* chunk = parts[pi];
        int64_t chunk_len = (int64_t)part_lens[pi];
        if (chunk_len == 0) continue;                           /* sd-inflate.ts:92-94 */
        int nomoreinput = 0;
        z->next_in = chunk; z->avail_in = chunk_len; z->next_in_index = 0;
        int64_t guard_last_avail = -1; int guard_spins = 0;
        do {
            z->next_out_index = 0;
            z->avail_out = OUTPUT_BUFSIZE;
            if (z->avail_in == 0 && !nomoreinput) { z->next_in_index = 0; nomoreinput = 1; }
            z->msg = ZM_NONE;
            int zerr = inflate_run(&I->inf, z);
            if (nomoreinput && zerr == Z_BUF_ERROR) {
                if (z->avail_in != 0) { err_code = ORA_E_INFLATE_MSG; res->zmsg = ZM_NONE; break; }
            } else if (zerr == Z_NEED_DICT) {
                if (I->has_dict) {
                    if (inflate_set_dictionary(&I->inf, I->dict, I->dict_len) != Z_OK) {
                        err_code = ORA_E_DICT_INVALID; break;
                    }
                } else { err_code = ORA_E_DICT_REQUIRED; break; }
            } else if (zerr != Z_OK && zerr != Z_STREAM_END) {
                err_code = ORA_E_INFLATE_MSG; res->zmsg = z->msg; break;
            }
            if ((nomoreinput || zerr == Z_STREAM_END) && z->avail_in == chunk_len) {
                err_code = ORA_E_BAD_INPUT_DATA; break;
            }
            if (z->next_out_index) {
                size_t cl = (size_t)z->next_out_index;
                int useCRC = inflate_container(&I->inf) == 2;
                if (!I->have_checksum) { I->checksum = useCRC ? 0 : 1; I->have_checksum = 1; }
                if (useCRC) I->checksum = oracle_crc32(z->next_out, cl, I->checksum);
                else I->checksum = oracle_adler32(z->next_out, cl, I->checksum);
                if (out_len + cl > out_cap) { err_code = ORA_E_OUT_CAP; break; }
                memcpy(out + out_len, z->next_out, cl);
                out_len += cl;
                /* the Uint8Array this iteration pushes (sd-inflate.ts:134) */
                if (nchunks && *nchunks < chunk_cap) { chunk_sz[*nchunks] = cl; chunk_part[*nchunks] = pi; }
                if (nchunks) (*nchunks)++;
            }
            /* DONE keeps returning STREAM_END without consuming input */
            if (zerr == Z_STREAM_END && z->next_out_index == 0 && z->avail_in > 0) {
                if (z->avail_in == guard_last_avail && ++guard_spins > 2) { err_code = ORA_E_HANG; break; }
                guard_last_avail = z->avail_in;
            }
        } while (z->avail_in > 0 || z->avail_out == 0);
        if (part_out) part_out[pi] = out_len - out_before;
        if (err_code != ORA_OK && err_part) *err_part = pi;
    }

    /* finish(): sd-inflate.ts:159-179 */
    int32_t stored_cs = I->inf.full_checksum;
    int32_t stored_size = I->inf.inflated_size;
    int complete = inflate_is_complete(&I->inf);
    int cs_verdict, size_verdict;
    if (stored_cs == 0) cs_verdict = 0;
    else cs_verdict = (I->have_checksum && stored_cs == I->checksum) ? 1 : 2;
    if (stored_size == 0) size_verdict = 0;
    else size_verdict = ((int64_t)stored_size == (int64_t)z->total_out) ? 1 : 2;
    res->error = err_code;
    res->complete = complete;
    res->checksum_verdict = cs_verdict;
    res->size_verdict = size_verdict;
    res->success = complete && cs_verdict != 2 && size_verdict != 2;
    res->stored_checksum = stored_cs;
    res->running_checksum = I->have_checksum ? I->checksum : 0;
    res->stored_size = stored_size;
    res->container = inflate_container(&I->inf);
    res->mtime = I->inf.mtime;
    res->name_len = I->inf.name_len;
    memcpy(res->name, I->inf.name, (size_t)I->inf.name_len);
    res->total_out = out_len;
    free(I);
    return err_code;
}

int32_t oracle_inflate(const uint8_t* in, size_t in_len, const uint8_t* dict, size_t dict_len,
                       uint8_t* out, size_t out_cap, oracle_inflate_result* res) {
    memset(res, 0, sizeof *res);
    if (in_len < 2) { res->error = ORA_E_TOO_SMALL; return res->error; }
    uint8_t method = in[0], flag = in[1];
    int starts = (method == 0x78 && ((((int)method << 8) + flag) % 31) == 0) ||
                 (method == 0x1f && flag == 0x8b);
    const uint8_t* parts[1] = { in };
    size_t lens[1] = { in_len };
    int32_t e = oracle_inflater_run(parts, lens, 1, starts ? 0 : 1, dict, dict_len, out, out_cap, res);
    if (e != ORA_OK) return e;
    if (!res->success) {
        if (!res->complete) res->error = ORA_E_UNEXPECTED_EOF;
        else if (res->checksum_verdict == 2) res->error = ORA_E_INTEGRITY;
        else if (res->size_verdict == 2) res->error = ORA_E_SIZE;
        else res->error = ORA_E_DECOMPRESSION;
    }
    return res->error;
}

/* ------------------------------------------------------------------------- */
/* deftree.ts                                                                 */
/* ------------------------------------------------------------------------- */
#define D_CODES 30
#define BL_CODES 19
#define LENGTH_CODES 29
#define LITERALS 256
#define L_CODES (LITERALS + 1 + LENGTH_CODES)
#define HEAP_SIZE (2 * L_CODES + 1)
#define MAX_BITS 15
#define MAX_BL_BITS 7

static uint8_t dist_code_tab[512];
static uint8_t length_code_tab[256];
static int base_length[LENGTH_CODES];
static int base_dist[D_CODES];
static const int extra_lbits[LENGTH_CODES] = { 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2,
    3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0 };
static const int extra_dbits[D_CODES] = { 0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7,
    8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13 };
static const int extra_blbits[BL_CODES] = { 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7 };
static const int bl_order[BL_CODES] = { 16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15 };
static uint16_t static_ltree[(L_CODES + 2) * 2];
static uint16_t static_dtree[D_CODES * 2];

static int bi_reverse(int code, int len);

/* deftree.ts:25-38, 269-298, 319-337: the code tables are zlib's trees.h; they are
 * derived here from extra_lbits/extra_dbits exactly as zlib's tr_static_init does,
 * and spot-checked against the reference's literals in tests. */
static void trees_init_once(void) {
    int length = 0, code, n, dist;
    for (code = 0; code < LENGTH_CODES - 1; code++) {
        base_length[code] = length;
        for (n = 0; n < (1 << extra_lbits[code]); n++) length_code_tab[length++] = (uint8_t)code;
    }
    length_code_tab[length - 1] = (uint8_t)code;   /* 255 -> code 28 (length 258) */
    base_length[LENGTH_CODES - 1] = 0;              /* deftree.ts:277 last entry is 0 */
    dist = 0;
    for (code = 0; code < 16; code++) {
        base_dist[code] = dist;
        for (n = 0; n < (1 << extra_dbits[code]); n++) dist_code_tab[dist++] = (uint8_t)code;
    }
    dist >>= 7;
    for (; code < D_CODES; code++) {
        base_dist[code] = dist << 7;
        for (n = 0; n < (1 << (extra_dbits[code] - 7)); n++) dist_code_tab[256 + dist++] = (uint8_t)code;
    }
    /* static trees: fixed code lengths with canonical codes */
    int bl_count[MAX_BITS + 1] = { 0 };
    for (n = 0; n <= 143; n++) { static_ltree[n * 2 + 1] = 8; bl_count[8]++; }
    for (; n <= 255; n++) { static_ltree[n * 2 + 1] = 9; bl_count[9]++; }
    for (; n <= 279; n++) { static_ltree[n * 2 + 1] = 7; bl_count[7]++; }
    for (; n <= 287; n++) { static_ltree[n * 2 + 1] = 8; bl_count[8]++; }
    {
        int next_code[MAX_BITS + 1]; int c = 0;
        for (int bits = 1; bits <= MAX_BITS; bits++) next_code[bits] = c = (c + bl_count[bits - 1]) << 1;
        for (n = 0; n <= L_CODES + 1; n++) {
            int len = static_ltree[n * 2 + 1];
            static_ltree[n * 2] = (uint16_t)bi_reverse(next_code[len]++, len);
        }
    }
    for (n = 0; n < D_CODES; n++) {
        static_dtree[n * 2 + 1] = 5;
        static_dtree[n * 2] = (uint16_t)bi_reverse(n, 5);
    }
}
static pthread_once_t trees_once = PTHREAD_ONCE_INIT;
static void trees_init(void) { pthread_once(&trees_once, trees_init_once); }

/* exported for the table spot checks in tests */
int32_t oracle_tree_table(int which, int idx) {
    trees_init();
    switch (which) {
    case 0: return static_ltree[idx];
    case 1: return static_dtree[idx];
    case 2: return dist_code_tab[idx];
    case 3: return length_code_tab[idx];
    case 4: return base_length[idx];
    default: return base_dist[idx];
    }
}

/* deftree.ts:285-287 */
static int d_code(int dist) { return dist < 256 ? dist_code_tab[dist] : dist_code_tab[256 + (dist >> 7)]; }

/* deftree.ts:137-147 */
static int bi_reverse(int code, int len) {
    int res = 0;
    do { res |= code & 1; code = (int)((unsigned)code >> 1); res <<= 1; } while (--len > 0);
    return (int)((unsigned)res >> 1);
}

typedef struct {
    const uint16_t* static_tree;
    const int* extra_bits;
    int extra_base;
    int elems;
    int max_length;
} static_desc;

typedef struct {
    uint16_t* dyn_tree;
    const static_desc* stat_desc;
    int max_code;
} tree_desc;

/* ------------------------------------------------------------------------- */
/* deflate.ts                                                                 */
/* ------------------------------------------------------------------------- */
#define W_BITS 15
#define W_SIZE (1 << W_BITS)
#define W_MASK (W_SIZE - 1)
#define HASH_BITS 15
#define HASH_SIZE (1 << HASH_BITS)
#define HASH_MASK (HASH_SIZE - 1)
#define HASH_SHIFT 5
#define LIT_BUFSIZE (1 << 14)
#define PENDING_BUF_SIZE (LIT_BUFSIZE * 4)
#define D_BUF (LIT_BUFSIZE / 2)
#define L_BUF (3 * LIT_BUFSIZE)
#define WINDOW_SIZE (2 * W_SIZE)
#define MIN_MATCH 3
#define MAX_MATCH 258
#define MIN_LOOKAHEAD (MAX_MATCH + MIN_MATCH + 1)
#define END_BLOCK 256
#define REP_3_6 16
#define REPZ_3_10 17
#define REPZ_11_138 18
#define STORED_BLOCK 0
#define STATIC_TREES 1
#define DYN_TREES 2

enum { NeedMore = 0, BlockDone = 1, FinishStarted = 2, FinishDone = 3 };
enum { NO_FLUSH = 0, FINISH = 4 };
enum { DS_INIT = 1, DS_BUSY = 2, DS_FINISH = 3 };

typedef struct { int good_length, max_lazy, nice_length, max_chain, func; } config;
/* defconfig.ts:33-44 (func: 0 stored, 1 fast, 2 slow) */
static const config config_table[10] = {
    { 0, 0, 0, 0, 0 }, { 4, 4, 8, 4, 1 }, { 4, 5, 16, 8, 1 }, { 4, 6, 32, 32, 1 },
    { 4, 4, 16, 16, 2 }, { 8, 16, 32, 32, 2 }, { 8, 16, 128, 128, 2 }, { 8, 32, 128, 256, 2 },
    { 32, 128, 258, 1024, 2 }, { 32, 258, 258, 4096, 2 } };

typedef struct {
    /* ZStream input side + unbounded output (output chunking does not change the
     * bitstream: deflate() only pauses when next_out is full) */
    const uint8_t* next_in; int64_t avail_in; int64_t next_in_index;
    uint8_t* out; size_t out_cap; size_t out_len;
    int status;
    uint8_t pending_buf[PENDING_BUF_SIZE];
    int pending, pending_out;
    int last_flush;
    uint8_t window[WINDOW_SIZE];
    uint16_t prev[W_SIZE];
    uint16_t head[HASH_SIZE];
    int ins_h;
    int block_start;
    int match_length, match_available, strstart, match_start, lookahead, prev_length;
    int level;
    int good_match, nice_match, max_chain_length, max_lazy_match;
    uint16_t dyn_ltree[HEAP_SIZE * 2];
    uint16_t dyn_dtree[(2 * D_CODES + 1) * 2];
    uint16_t bl_tree[(2 * BL_CODES + 1) * 2];
    tree_desc l_desc, d_desc, bl_desc;
    uint16_t depth[2 * L_CODES + 1];
    int last_lit, matches;
    int64_t opt_len, static_len;
    int last_eob_len;
    uint32_t bi_buf; int bi_valid;
    uint16_t bl_count[MAX_BITS + 1];
    uint16_t heap[2 * L_CODES + 1];
    int heap_len, heap_max;
    int overflow;   /* reference would write/read past pending_buf */
} deflate_state;

static const static_desc static_l_desc = { static_ltree, extra_lbits, LITERALS + 1, L_CODES, MAX_BITS };
static const static_desc static_d_desc = { static_dtree, extra_dbits, 0, D_CODES, MAX_BITS };
static const static_desc static_bl_desc = { NULL, extra_blbits, 0, BL_CODES, MAX_BL_BITS };

/* Uint8Array store semantics: out-of-range writes are dropped by JS; the oracle
 * flags them instead (the reference output would be undefined). */
static inline void pbuf_put(deflate_state* s, int idx, uint32_t v) {
    if (idx < 0 || idx >= PENDING_BUF_SIZE) { s->overflow = 1; return; }
    s->pending_buf[idx] = (uint8_t)v;
}

/* deflate.ts:16-20 */
static int smaller(const uint16_t* tree, int n, int m, const uint16_t* depth) {
    int tn2 = tree[n * 2], tm2 = tree[m * 2];
    return tn2 < tm2 || (tn2 == tm2 && depth[n] <= depth[m]);
}

/* deflate.ts:222-234 */
static void init_block(deflate_state* s) {
    for (int i = 0; i < L_CODES; i++) s->dyn_ltree[i * 2] = 0;
    for (int i = 0; i < D_CODES; i++) s->dyn_dtree[i * 2] = 0;
    for (int i = 0; i < BL_CODES; i++) s->bl_tree[i * 2] = 0;
    s->dyn_ltree[END_BLOCK * 2] = 1;
    s->opt_len = s->static_len = 0;
    s->last_lit = s->matches = 0;
}

/* deflate.ts:241-263 */
static void pqdownheap(deflate_state* s, const uint16_t* tree, int k) {
    uint16_t* heap = s->heap;
    int v = heap[k];
    int j = k << 1;
    while (j <= s->heap_len) {
        if (j < s->heap_len && smaller(tree, heap[j + 1], heap[j], s->depth)) j++;
        if (smaller(tree, v, heap[j], s->depth)) break;
        heap[k] = heap[j];
        k = j;
        j <<= 1;
    }
    heap[k] = (uint16_t)v;
}

/* deftree.ts:60-132 */
static void gen_bitlen(deflate_state* s, tree_desc* desc) {
    uint16_t* tree = desc->dyn_tree;
    const uint16_t* stree = desc->stat_desc->static_tree;
    const int* extra = desc->stat_desc->extra_bits;
    int base = desc->stat_desc->extra_base;
    int max_length = desc->stat_desc->max_length;
    int h, n, m, bits, xbits, f, overflow = 0;

    for (bits = 0; bits <= MAX_BITS; bits++) s->bl_count[bits] = 0;
    tree[s->heap[s->heap_max] * 2 + 1] = 0;
    for (h = s->heap_max + 1; h < HEAP_SIZE; h++) {
        n = s->heap[h];
        bits = tree[tree[n * 2 + 1] * 2 + 1] + 1;
        if (bits > max_length) { bits = max_length; overflow++; }
        tree[n * 2 + 1] = (uint16_t)bits;
        if (n > desc->max_code) continue;
        s->bl_count[bits]++;
        xbits = 0;
        if (n >= base) xbits = extra[n - base];
        f = tree[n * 2];
        s->opt_len += (int64_t)f * (bits + xbits);
        if (stree) s->static_len += (int64_t)f * (stree[n * 2 + 1] + xbits);
    }
    if (overflow == 0) return;
    do {
        bits = max_length - 1;
        while (s->bl_count[bits] == 0) bits--;
        s->bl_count[bits]--;
        s->bl_count[bits + 1] += 2;
        s->bl_count[max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    for (bits = max_length; bits != 0; bits--) {
        n = s->bl_count[bits];
        while (n != 0) {
            m = s->heap[--h];
            if (m > desc->max_code) continue;
            if (tree[m * 2 + 1] != bits) {
                s->opt_len += (int64_t)(bits - tree[m * 2 + 1]) * tree[m * 2];
                tree[m * 2 + 1] = (uint16_t)bits;
            }
            n--;
        }
    }
}

/* deftree.ts:155-182 */
static void gen_codes(uint16_t* tree, int max_code, const uint16_t* bl_count) {
    uint16_t next_code[MAX_BITS + 1];
    int code = 0;
    for (int bits = 1; bits <= MAX_BITS; bits++) {
        code = (code + bl_count[bits - 1]) << 1;
        next_code[bits] = (uint16_t)code;
    }
    for (int n = 0; n <= max_code; n++) {
        int len = tree[n * 2 + 1];
        if (len == 0) continue;
        tree[n * 2] = (uint16_t)bi_reverse(next_code[len]++, len);
    }
}

/* deftree.ts:190-267 */
static void build_tree(deflate_state* s, tree_desc* desc) {
    uint16_t* tree = desc->dyn_tree;
    const uint16_t* stree = desc->stat_desc->static_tree;
    int elems = desc->stat_desc->elems;
    int n, m, max_code = -1, node;

    s->heap_len = 0;
    s->heap_max = HEAP_SIZE;
    for (n = 0; n < elems; n++) {
        if (tree[n * 2] != 0) {
            s->heap[++s->heap_len] = (uint16_t)(max_code = n);
            s->depth[n] = 0;
        } else {
            tree[n * 2 + 1] = 0;
        }
    }
    while (s->heap_len < 2) {
        node = s->heap[++s->heap_len] = (uint16_t)(max_code < 2 ? ++max_code : 0);
        tree[node * 2] = 1;
        s->depth[node] = 0;
        s->opt_len--;
        if (stree) s->static_len -= stree[node * 2 + 1];
    }
    desc->max_code = max_code;
    for (n = s->heap_len / 2; n >= 1; n--) pqdownheap(s, tree, n);
    node = elems;
    do {
        n = s->heap[1];
        s->heap[1] = s->heap[s->heap_len--];
        pqdownheap(s, tree, 1);
        m = s->heap[1];
        s->heap[--s->heap_max] = (uint16_t)n;
        s->heap[--s->heap_max] = (uint16_t)m;
        tree[node * 2] = (uint16_t)(tree[n * 2] + tree[m * 2]);
        s->depth[node] = (uint16_t)((s->depth[n] > s->depth[m] ? s->depth[n] : s->depth[m]) + 1);
        tree[n * 2 + 1] = tree[m * 2 + 1] = (uint16_t)node;
        s->heap[1] = (uint16_t)(node++);
        pqdownheap(s, tree, 1);
    } while (s->heap_len >= 2);
    s->heap[--s->heap_max] = s->heap[1];
    gen_bitlen(s, desc);
    gen_codes(tree, desc->max_code, s->bl_count);
}

/* deflate.ts:267-312 */
static void scan_tree(deflate_state* s, uint16_t* tree, int max_code) {
    int prevlen = -1, curlen, nextlen = tree[0 * 2 + 1], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    tree[(max_code + 1) * 2 + 1] = 0xffff;
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = tree[(n + 1) * 2 + 1];
        if (++count < max_count && curlen == nextlen) continue;
        else if (count < min_count) s->bl_tree[curlen * 2] = (uint16_t)(s->bl_tree[curlen * 2] + count);
        else if (curlen != 0) {
            if (curlen != prevlen) s->bl_tree[curlen * 2]++;
            s->bl_tree[REP_3_6 * 2]++;
        } else if (count <= 10) s->bl_tree[REPZ_3_10 * 2]++;
        else s->bl_tree[REPZ_11_138 * 2]++;
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

/* deflate.ts:316-339 */
static int build_bl_tree(deflate_state* s) {
    int max_blindex;
    scan_tree(s, s->dyn_ltree, s->l_desc.max_code);
    scan_tree(s, s->dyn_dtree, s->d_desc.max_code);
    build_tree(s, &s->bl_desc);
    for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
        if (s->bl_tree[bl_order[max_blindex] * 2 + 1] != 0) break;
    s->opt_len += 3 * (max_blindex + 1) + 5 + 5 + 4;
    return max_blindex;
}

/* deflate.ts:347-350 */
static void put_short(deflate_state* s, uint32_t w) {
    pbuf_put(s, s->pending++, w & 0xff);
    pbuf_put(s, s->pending++, (w >> 8) & 0xff);
}

/* deflate.ts:352-369 */
static void send_bits(deflate_state* s, int value, int length) {
    uint32_t v = (uint32_t)value;
    if (s->bi_valid > 16 - length) {
        s->bi_buf |= (v << s->bi_valid) & 0xffff;
        pbuf_put(s, s->pending, s->bi_buf);
        pbuf_put(s, s->pending + 1, s->bi_buf >> 8);
        s->pending += 2;
        s->bi_buf = v >> (16 - s->bi_valid);
        s->bi_valid += length - 16;
    } else {
        s->bi_buf |= (v << s->bi_valid) & 0xffff;
        s->bi_valid += length;
    }
}

/* deflate.ts:371-374 */
static void send_code(deflate_state* s, int c, const uint16_t* tree) {
    send_bits(s, tree[c * 2] & 0xffff, tree[c * 2 + 1] & 0xffff);
}

/* deflate.ts:378-429 */
static void send_tree(deflate_state* s, const uint16_t* tree, int max_code) {
    int prevlen = -1, curlen, nextlen = tree[0 * 2 + 1], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    for (int n = 0; n <= max_code; n++) {
        curlen = nextlen;
        nextlen = tree[(n + 1) * 2 + 1];
        if (++count < max_count && curlen == nextlen) continue;
        else if (count < min_count) {
            do { send_code(s, curlen, s->bl_tree); } while (--count != 0);
        } else if (curlen != 0) {
            if (curlen != prevlen) { send_code(s, curlen, s->bl_tree); count--; }
            send_code(s, REP_3_6, s->bl_tree);
            send_bits(s, count - 3, 2);
        } else if (count <= 10) {
            send_code(s, REPZ_3_10, s->bl_tree);
            send_bits(s, count - 3, 3);
        } else {
            send_code(s, REPZ_11_138, s->bl_tree);
            send_bits(s, count - 11, 7);
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

/* deflate.ts:434-443 */
static void send_all_trees(deflate_state* s, int lcodes, int dcodes, int blcodes) {
    send_bits(s, lcodes - 257, 5);
    send_bits(s, dcodes - 1, 5);
    send_bits(s, blcodes - 4, 4);
    for (int rank = 0; rank < blcodes; rank++) send_bits(s, s->bl_tree[bl_order[rank] * 2 + 1], 3);
    send_tree(s, s->dyn_ltree, lcodes - 1);
    send_tree(s, s->dyn_dtree, dcodes - 1);
}

static int pbuf_get(deflate_state* s, int idx) {
    if (idx < 0 || idx >= PENDING_BUF_SIZE) { s->overflow = 1; return 0; }
    return s->pending_buf[idx];
}

/* deflate.ts:488-524 (TRUNCATE_BLOCK heuristic at 508-518 kept) */
static int tr_tally(deflate_state* s, int dist, int lc) {
    pbuf_put(s, D_BUF + s->last_lit * 2, ((uint32_t)dist >> 8) & 0xff);
    pbuf_put(s, D_BUF + s->last_lit * 2 + 1, (uint32_t)dist & 0xff);
    pbuf_put(s, L_BUF + s->last_lit, (uint32_t)lc & 0xff);
    s->last_lit++;
    if (dist == 0) {
        s->dyn_ltree[lc * 2]++;
    } else {
        s->matches++;
        dist--;
        s->dyn_ltree[(length_code_tab[lc] + LITERALS + 1) * 2]++;
        s->dyn_dtree[d_code(dist) * 2]++;
    }
    if ((s->last_lit & 0x1fff) == 0 && s->level > 2) {
        int64_t out_length = (int64_t)s->last_lit * 8;
        int64_t in_length = s->strstart - s->block_start;
        for (int dcode = 0; dcode < D_CODES; dcode++)
            out_length += (int64_t)s->dyn_dtree[dcode * 2] * (5 + extra_dbits[dcode]);
        out_length = (int64_t)((uint32_t)out_length >> 3);
        if (s->matches < s->last_lit / 2 && out_length < in_length / 2) return 1;
    }
    return s->last_lit == LIT_BUFSIZE - 1;
}

/* deflate.ts:527-571 (reads d_buf/l_buf out of the same pending_buf it writes) */
static void compress_block(deflate_state* s, const uint16_t* ltree, const uint16_t* dtree) {
    int lx = 0;
    if (s->last_lit != 0) {
        do {
            int dist = ((pbuf_get(s, D_BUF + lx * 2) << 8) & 0xff00) | (pbuf_get(s, D_BUF + lx * 2 + 1) & 0xff);
            int lc = pbuf_get(s, L_BUF + lx) & 0xff;
            lx++;
            if (dist == 0) {
                send_code(s, lc, ltree);
            } else {
                int code = length_code_tab[lc];
                send_code(s, code + LITERALS + 1, ltree);
                int extra = extra_lbits[code];
                if (extra != 0) { lc -= base_length[code]; send_bits(s, lc, extra); }
                dist--;
                code = d_code(dist);
                send_code(s, code, dtree);
                extra = extra_dbits[code];
                if (extra != 0) { dist -= base_dist[code]; send_bits(s, dist, extra); }
            }
        } while (lx < s->last_lit);
    }
    send_code(s, END_BLOCK, ltree);
    s->last_eob_len = ltree[END_BLOCK * 2 + 1];
}

/* deflate.ts:574-583 */
static void bi_windup(deflate_state* s) {
    if (s->bi_valid > 8) put_short(s, s->bi_buf);
    else if (s->bi_valid > 0) pbuf_put(s, s->pending++, s->bi_buf);
    s->bi_buf = 0;
    s->bi_valid = 0;
}

/* deflate.ts:587-601 */
static void copy_block(deflate_state* s, int buf, int len, int header) {
    bi_windup(s);
    s->last_eob_len = 8;
    if (header) { put_short(s, (uint32_t)len); put_short(s, ~(uint32_t)len); }
    if (s->pending + len > PENDING_BUF_SIZE) { s->overflow = 1; return; }  /* TypedArray.set throws */
    memcpy(s->pending_buf + s->pending, s->window + buf, (size_t)len);
    s->pending += len;
}

/* deflate.ts:604-610 */
static void tr_stored_block(deflate_state* s, int buf, int stored_len, int eof) {
    send_bits(s, (STORED_BLOCK << 1) + (eof ? 1 : 0), 3);
    copy_block(s, buf, stored_len, 1);
}

/* deflate.ts:614-674 */
static void tr_flush_block(deflate_state* s, int buf, int stored_len, int eof) {
    int64_t opt_lenb, static_lenb;
    int max_blindex = 0;
    if (s->level > 0) {
        build_tree(s, &s->l_desc);
        build_tree(s, &s->d_desc);
        max_blindex = build_bl_tree(s);
        opt_lenb = (int64_t)((uint32_t)(s->opt_len + 3 + 7) >> 3);
        static_lenb = (int64_t)((uint32_t)(s->static_len + 3 + 7) >> 3);
        if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    } else {
        opt_lenb = static_lenb = stored_len + 5;
    }
    if ((stored_len + 4 <= opt_lenb) && buf != -1) {
        tr_stored_block(s, buf, stored_len, eof);
    } else if (static_lenb == opt_lenb) {
        send_bits(s, (STATIC_TREES << 1) + (eof ? 1 : 0), 3);
        compress_block(s, static_ltree, static_dtree);
    } else {
        send_bits(s, (DYN_TREES << 1) + (eof ? 1 : 0), 3);
        send_all_trees(s, s->l_desc.max_code + 1, s->d_desc.max_code + 1, max_blindex + 1);
        compress_block(s, s->dyn_ltree, s->dyn_dtree);
    }
    init_block(s);
    if (eof) bi_windup(s);
}

/* zstream.ts:76-94 with an unbounded next_out */
static void flush_pending(deflate_state* s) {
    int len = s->pending;
    if (len == 0) return;
    if (s->out_len + (size_t)len > s->out_cap) { s->overflow = 2; len = 0; }
    else {
        if (s->pending_out + len > PENDING_BUF_SIZE) { s->overflow = 1; len = 0; }
        else memcpy(s->out + s->out_len, s->pending_buf + s->pending_out, (size_t)len);
    }
    s->out_len += (size_t)len;
    s->pending_out += len;
    s->pending -= len;
    if (s->pending == 0) s->pending_out = 0;
    s->pending = 0; s->pending_out = 0;
}

/* deflate.ts:676-680 */
static void flush_block_only(deflate_state* s, int eof) {
    tr_flush_block(s, s->block_start >= 0 ? s->block_start : -1, s->strstart - s->block_start, eof);
    s->block_start = s->strstart;
    flush_pending(s);
}

/* zstream.ts:56-70 */
static int read_into_buf(deflate_state* s, int start, int size) {
    int64_t len = s->avail_in;
    if (len > size) len = size;
    if (len == 0) return 0;
    memcpy(s->window + start, s->next_in + s->next_in_index, (size_t)len);
    s->avail_in -= len;
    s->next_in_index += len;
    return (int)len;
}

/* deflate.ts:690-766 */
static void fill_window(deflate_state* s) {
    do {
        int more = WINDOW_SIZE - s->lookahead - s->strstart;
        if (more == 0 && s->strstart == 0 && s->lookahead == 0) {
            more = W_SIZE;
        } else if (more == -1) {
            more--;
        } else if (s->strstart >= W_SIZE + W_SIZE - MIN_LOOKAHEAD) {
            memcpy(s->window, s->window + W_SIZE, W_SIZE);
            s->match_start -= W_SIZE;
            s->strstart -= W_SIZE;
            s->block_start -= W_SIZE;
            int n = HASH_SIZE, p = n, m;
            do { m = s->head[--p]; s->head[p] = (uint16_t)(m >= W_SIZE ? m - W_SIZE : 0); } while (--n != 0);
            n = W_SIZE; p = n;
            do { m = s->prev[--p]; s->prev[p] = (uint16_t)(m >= W_SIZE ? m - W_SIZE : 0); } while (--n != 0);
            more += W_SIZE;
        }
        if (s->avail_in == 0) return;
        int n = read_into_buf(s, s->strstart + s->lookahead, more);
        s->lookahead += n;
        if (s->lookahead >= MIN_MATCH) {
            s->ins_h = s->window[s->strstart] & 0xff;
            s->ins_h = ((s->ins_h << HASH_SHIFT) ^ (s->window[s->strstart + 1] & 0xff)) & HASH_MASK;
        }
    } while (s->lookahead < MIN_LOOKAHEAD && s->avail_in != 0);
}

/* deflate.ts:827-946 */
static int longest_match(deflate_state* s, int cur_match) {
    int chain_length = s->max_chain_length;
    int scan = s->strstart;
    int best_len = s->prev_length;
    int limit = s->strstart > (W_SIZE - MIN_LOOKAHEAD) ? s->strstart - (W_SIZE - MIN_LOOKAHEAD) : 0;
    int nice = s->nice_match;
    const uint8_t* win = s->window;
    int strend = s->strstart + MAX_MATCH;
    int scan_end1 = win[scan + best_len - 1];
    int scan_end = win[scan + best_len];
    int scan_start = win[scan];
    int scan_start1 = win[scan + 1];

    if (s->prev_length >= s->good_match) chain_length >>= 2;
    if (nice > s->lookahead) nice = s->lookahead;

    do {
        int match = cur_match;
        int cont = 1;
        for (;;) {
            match = cur_match;
            if (win[match + best_len] != scan_end || win[match + best_len - 1] != scan_end1) {
                if ((cur_match = s->prev[cur_match & W_MASK]) > limit && --chain_length != 0) continue;
                else cont = 0;
            }
            break;
        }
        if (!cont) break;
        if (win[match] != scan_start || win[match + 1] != scan_start1) continue;
        scan += 2;
        match += 2;
        do {
            uint32_t sv = ((uint32_t)win[scan] << 24) | ((uint32_t)win[scan + 1] << 16) |
                          ((uint32_t)win[scan + 2] << 8) | win[scan + 3];
            uint32_t mv = ((uint32_t)win[match] << 24) | ((uint32_t)win[match + 1] << 16) |
                          ((uint32_t)win[match + 2] << 8) | win[match + 3];
            uint32_t sxm = sv ^ mv;
            if (sxm) {
                int mb = __builtin_clz(sxm) >> 3;
                scan += mb; match += mb;
                break;
            } else {
                scan += 4; match += 4;
            }
        } while (scan < strend);
        if (scan > strend) scan = strend;
        int len = MAX_MATCH - (strend - scan);
        scan = strend - MAX_MATCH;
        if (len > best_len) {
            s->match_start = cur_match;
            best_len = len;
            if (len >= nice) break;
            scan_end1 = win[scan + best_len - 1];
            scan_end = win[scan + best_len];
        }
    } while ((cur_match = s->prev[cur_match & W_MASK]) > limit && --chain_length != 0);

    if (best_len <= s->lookahead) return best_len;
    return s->lookahead;
}

#define INSERT_STRING(s, hh)                                                              \
    do {                                                                                  \
        (s)->ins_h = (((s)->ins_h << HASH_SHIFT) ^ ((s)->window[(s)->strstart + (MIN_MATCH - 1)] & 0xff)) & HASH_MASK; \
        hh = (s)->head[(s)->ins_h] & 0xffff;                                             \
        (s)->prev[(s)->strstart & W_MASK] = (s)->head[(s)->ins_h];                       \
        (s)->head[(s)->ins_h] = (uint16_t)(s)->strstart;                                 \
    } while (0)

/* deflate.ts:953-1049 */
static int deflate_fast(deflate_state* s, int flush) {
    int hash_head = 0, bflush;
    for (;;) {
        if (s->lookahead < MIN_LOOKAHEAD) {
            fill_window(s);
            if (s->lookahead < MIN_LOOKAHEAD && flush == NO_FLUSH) return NeedMore;
            if (s->lookahead == 0) break;
        }
        if (s->lookahead >= MIN_MATCH) INSERT_STRING(s, hash_head);
        if (hash_head != 0 && ((s->strstart - hash_head) & 0xffff) <= W_SIZE - MIN_LOOKAHEAD) {
            s->match_length = longest_match(s, hash_head);
        }
        if (s->match_length >= MIN_MATCH) {
            bflush = tr_tally(s, s->strstart - s->match_start, s->match_length - MIN_MATCH);
            s->lookahead -= s->match_length;
            if (s->match_length <= s->max_lazy_match && s->lookahead >= MIN_MATCH) {
                s->match_length--;
                do {
                    s->strstart++;
                    INSERT_STRING(s, hash_head);
                } while (--s->match_length != 0);
                s->strstart++;
            } else {
                s->strstart += s->match_length;
                s->match_length = 0;
                s->ins_h = s->window[s->strstart] & 0xff;
                s->ins_h = ((s->ins_h << HASH_SHIFT) ^ (s->window[s->strstart + 1] & 0xff)) & HASH_MASK;
            }
        } else {
            bflush = tr_tally(s, 0, s->window[s->strstart] & 0xff);
            s->lookahead--;
            s->strstart++;
        }
        if (bflush) flush_block_only(s, 0);
    }
    flush_block_only(s, flush == FINISH);
    return flush == FINISH ? FinishDone : BlockDone;
}

/* deflate.ts:1054-1182 */
static int deflate_slow(deflate_state* s, int flush) {
    int hash_head = 0, bflush, max_insert, prev_match;
    for (;;) {
        if (s->lookahead < MIN_LOOKAHEAD) {
            fill_window(s);
            if (s->lookahead < MIN_LOOKAHEAD && flush == NO_FLUSH) return NeedMore;
            if (s->lookahead == 0) break;
        }
        if (s->lookahead >= MIN_MATCH) INSERT_STRING(s, hash_head);
        s->prev_length = s->match_length;
        prev_match = s->match_start;
        s->match_length = MIN_MATCH - 1;
        if (hash_head != 0 && s->prev_length < s->max_lazy_match &&
            ((s->strstart - hash_head) & 0xffff) <= W_SIZE - MIN_LOOKAHEAD) {
            s->match_length = longest_match(s, hash_head);
            if (s->match_length <= 5 && (s->match_length == MIN_MATCH && s->strstart - s->match_start > 4096))
                s->match_length = MIN_MATCH - 1;
        }
        if (s->prev_length >= MIN_MATCH && s->match_length <= s->prev_length) {
            max_insert = s->strstart + s->lookahead - MIN_MATCH;
            bflush = tr_tally(s, s->strstart - 1 - prev_match, s->prev_length - MIN_MATCH);
            s->lookahead -= s->prev_length - 1;
            s->prev_length -= 2;
            do {
                if (++s->strstart <= max_insert) INSERT_STRING(s, hash_head);
            } while (--s->prev_length != 0);
            s->match_available = 0;
            s->match_length = MIN_MATCH - 1;
            s->strstart++;
            if (bflush) flush_block_only(s, 0);
        } else if (s->match_available) {
            bflush = tr_tally(s, 0, s->window[s->strstart - 1] & 0xff);
            if (bflush) flush_block_only(s, 0);
            s->strstart++;
            s->lookahead--;
        } else {
            s->match_available = 1;
            s->strstart++;
            s->lookahead--;
        }
    }
    if (s->match_available) {
        bflush = tr_tally(s, 0, s->window[s->strstart - 1] & 0xff);
        s->match_available = 0;
    }
    flush_block_only(s, flush == FINISH);
    return flush == FINISH ? FinishDone : BlockDone;
}

/* deflate.ts:1184-1216 */
static int deflate_set_dictionary(deflate_state* s, const uint8_t* dict, size_t dict_len) {
    size_t length = dict_len, index = 0;
    if (s->status != DS_INIT) return Z_STREAM_ERROR;
    if (length < MIN_MATCH) return Z_OK;
    if (length > W_SIZE - MIN_LOOKAHEAD) {
        length = W_SIZE - MIN_LOOKAHEAD;
        index = dict_len - length;
    }
    memcpy(s->window, dict + index, length);
    s->strstart = (int)length;
    s->block_start = (int)length;
    s->ins_h = s->window[0] & 0xff;
    s->ins_h = ((s->ins_h << HASH_SHIFT) ^ (s->window[1] & 0xff)) & HASH_MASK;
    for (int n = 0; n <= (int)length - MIN_MATCH; n++) {
        s->ins_h = ((s->ins_h << HASH_SHIFT) ^ (s->window[n + (MIN_MATCH - 1)] & 0xff)) & HASH_MASK;
        s->prev[n & W_MASK] = s->head[s->ins_h];
        s->head[s->ins_h] = (uint16_t)n;
    }
    return Z_OK;
}

/* deflate.ts:196-220 */
static void deflate_ctor(deflate_state* s, int level) {
    memset(s, 0, sizeof *s);
    trees_init();
    s->status = DS_INIT;
    s->l_desc.dyn_tree = s->dyn_ltree; s->l_desc.stat_desc = &static_l_desc;
    s->d_desc.dyn_tree = s->dyn_dtree; s->d_desc.stat_desc = &static_d_desc;
    s->bl_desc.dyn_tree = s->bl_tree; s->bl_desc.stat_desc = &static_bl_desc;
    s->match_length = MIN_MATCH - 1;
    s->prev_length = MIN_MATCH - 1;
    s->last_eob_len = 8;
    s->heap_max = HEAP_SIZE;
    s->level = level;
    init_block(s);
    s->max_lazy_match = config_table[level].max_lazy;
    s->good_match = config_table[level].good_length;
    s->nice_match = config_table[level].nice_length;
    s->max_chain_length = config_table[level].max_chain;
}

/* deflate.ts:1218-1327 restricted to NO_FLUSH/FINISH (the only values the API passes) */
static int deflate_call(deflate_state* s, int flush) {
    int old_flush = s->last_flush;
    s->last_flush = flush;
    if (s->status == DS_INIT) s->status = DS_BUSY;
    if (s->pending != 0) flush_pending(s);
    else if (s->avail_in == 0 && flush <= old_flush && flush != FINISH) return Z_BUF_ERROR;
    if (s->status == DS_FINISH && s->avail_in != 0) return Z_BUF_ERROR;
    if (s->avail_in != 0 || s->lookahead != 0 || (flush != NO_FLUSH && s->status != DS_FINISH)) {
        int bstate;
        if (config_table[s->level].func == 1) bstate = deflate_fast(s, flush);
        else bstate = deflate_slow(s, flush);
        if (bstate == FinishStarted || bstate == FinishDone) s->status = DS_FINISH;
        if (bstate == NeedMore || bstate == FinishStarted) return Z_OK;
    }
    if (flush != FINISH) return Z_OK;
    return Z_STREAM_END;
}

static void emit(deflate_state* s, const uint8_t* b, size_t n) {
    if (s->out_len + n > s->out_cap) { s->overflow = 2; return; }
    memcpy(s->out + s->out_len, b, n);
    s->out_len += n;
}

/* sd-deflate.ts:51-254 Deflater + 263-274 deflate().  part_end (may be NULL; nparts + 1
 * entries): the output length after each append() and after finish() -- where the
 * reference's per-call outputs end in the concatenation. */
int32_t oracle_deflater_run_parts(const uint8_t* const* parts, const size_t* part_lens, int32_t nparts,
                                  int32_t level, int32_t format, const uint8_t* dict, size_t dict_len,
                                  int32_t has_dict, const uint8_t* fname, size_t fname_len,
                                  uint32_t mtime, uint8_t* out, size_t out_cap, size_t* out_len,
                                  size_t* part_end) {
    *out_len = 0;
    if (level < 1 || level > 9 || format < 0 || format > 2) return ORA_E_BAD_ARG;
    if (has_dict && format != 1) return ORA_E_BAD_ARG;
    deflate_state* s = (deflate_state*)malloc(sizeof(deflate_state));
    if (!s) return ORA_E_BAD_ARG;
    deflate_ctor(s, level);
    s->out = out; s->out_cap = out_cap; s->out_len = 0;
    int32_t checksum = format == 2 ? 0 : 1;
    uint32_t orig_size = 0;
    int32_t dict_checksum = 0;
    if (has_dict) {
        dict_checksum = oracle_adler32(dict, dict_len, 1);
        deflate_set_dictionary(s, dict, dict_len);
    }
    for (int pi = 0; pi < nparts; pi++) {
        const uint8_t* chunk = parts[pi];
        size_t clen = part_lens[pi];
        if (clen == 0) { if (part_end) part_end[pi] = s->out_len; continue; }                                  /* sd-deflate.ts:180-182 */
        if (format != 2) checksum = oracle_adler32(chunk, clen, checksum);
        else checksum = oracle_crc32(chunk, clen, checksum);
        orig_size += (uint32_t)clen;
        s->next_in = chunk; s->avail_in = (int64_t)clen; s->next_in_index = 0;
        if (s->status == DS_INIT) {
            if (format == 1) {                                    /* sd-deflate.ts:98-115 */
                uint8_t h[6];
                uint32_t check = dict_checksum != 0 ? 0x20 : 1;
                h[0] = 0x78; h[1] = (uint8_t)check;
                if (dict_checksum != 0) {
                    uint32_t d = (uint32_t)dict_checksum;
                    h[2] = (uint8_t)(d >> 24); h[3] = (uint8_t)(d >> 16); h[4] = (uint8_t)(d >> 8); h[5] = (uint8_t)d;
                    emit(s, h, 6);
                } else emit(s, h, 2);
            } else if (format == 2) {                             /* sd-deflate.ts:117-152 */
                uint8_t h[10];
                h[0] = 0x1f; h[1] = 0x8b; h[2] = 8; h[3] = fname_len > 0 ? 0x08 : 0;
                h[4] = (uint8_t)mtime; h[5] = (uint8_t)(mtime >> 8); h[6] = (uint8_t)(mtime >> 16); h[7] = (uint8_t)(mtime >> 24);
                h[8] = 0; h[9] = 0xff;
                emit(s, h, 10);
                if (fname_len > 0) { uint8_t z0 = 0; emit(s, fname, fname_len); emit(s, &z0, 1); }
            }
        }
        do {
            deflate_call(s, NO_FLUSH);
        } while (s->avail_in > 0);
        if (part_end) part_end[pi] = s->out_len;
    }
    if (s->status == DS_INIT) { free(s); return ORA_E_FINISH_BEFORE_APPEND; }
    deflate_call(s, FINISH);
    if (format != 0) {                                            /* sd-deflate.ts:154-165 */
        uint32_t c = (uint32_t)checksum;
        if (format == 2) {
            uint8_t t[8] = { (uint8_t)c, (uint8_t)(c >> 8), (uint8_t)(c >> 16), (uint8_t)(c >> 24),
                             (uint8_t)orig_size, (uint8_t)(orig_size >> 8), (uint8_t)(orig_size >> 16), (uint8_t)(orig_size >> 24) };
            emit(s, t, 8);
        } else {
            uint8_t t[4] = { (uint8_t)(c >> 24), (uint8_t)(c >> 16), (uint8_t)(c >> 8), (uint8_t)c };
            emit(s, t, 4);
        }
    }
    int ovf = s->overflow;
    *out_len = s->out_len;
    if (part_end) part_end[nparts] = s->out_len;
    free(s);
    if (ovf == 2) return ORA_E_OUT_CAP;
    if (ovf) return ORA_E_PENDING_OVERFLOW;
    return ORA_OK;
}

int32_t oracle_deflater_run(const uint8_t* const* parts, const size_t* part_lens, int32_t nparts,
                            int32_t level, int32_t format, const uint8_t* dict, size_t dict_len,
                            int32_t has_dict, const uint8_t* fname, size_t fname_len,
                            uint32_t mtime, uint8_t* out, size_t out_cap, size_t* out_len) {
    return oracle_deflater_run_parts(parts, part_lens, nparts, level, format, dict, dict_len, has_dict, fname,
                                     fname_len, mtime, out, out_cap, out_len, NULL);
}
