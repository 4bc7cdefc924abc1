/*
 * sanitize_main.c -- drives the CPU restatement (sdz_oracle.c) under AddressSanitizer +
 * UndefinedBehaviorSanitizer (`make -C oracle asan`) or ThreadSanitizer (`make -C oracle
 * tsan`); SURVEY.md §5 "Race detection / sanitizers".  TEST INFRASTRUCTURE ONLY, run by
 * tests/test_oracle_sanitize.py.
 *
 * The restatement deliberately keeps the reference's quirks that read or write near buffer
 * edges -- stale window bytes past the input (deflate.ts:708-737, 943-945), the
 * pending_buf overlay (A7, deflate.ts:93-95, 536-537), the 32 KiB inflate ring wrap
 * (infcodes.ts:161-207) -- so the cases below aim at exactly those: the reference's
 * fixtures, every level and container, window-slide edge sizes, incompressible (stored)
 * inputs, dictionaries, split appends, and corrupted / truncated streams.  The threaded
 * part runs inflate and deflate from several threads at once, as bench.py's cpu_baseline
 * does through ctypes (the lazily built code tables were a data race before pthread_once).
 *
 * usage: oracle_san <tests/golden dir> [threads]
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sdz_oracle.h"

static int g_fail = 0;
#define CHECK(c, ...)                                         \
    do {                                                      \
        if (!(c)) {                                           \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                     \
            fprintf(stderr, "\n");                            \
            g_fail++;                                         \
        }                                                     \
    } while (0)

typedef struct { uint8_t* p; size_t n; } buf_t;

static buf_t load(const char* dir, const char* name) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE* f = fopen(path, "rb");
    buf_t b = { NULL, 0 };
    if (!f) { fprintf(stderr, "cannot open %s\n", path); exit(2); }
    fseek(f, 0, SEEK_END);
    b.n = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    b.p = (uint8_t*)malloc(b.n ? b.n : 1);   /* exact size: ASan sees any overread */
    if (b.n && fread(b.p, 1, b.n, f) != b.n) exit(2);
    fclose(f);
    return b;
}

static uint64_t g_rng = 0x5D5A1B1Eull;
static uint32_t rnd(void) {
    g_rng ^= g_rng << 13; g_rng ^= g_rng >> 7; g_rng ^= g_rng << 17;
    return (uint32_t)(g_rng >> 11);
}

/* one-shot deflate into an exactly sized heap buffer; returns length or (size_t)-1 */
static size_t deflate1(const uint8_t* in, size_t n, int level, int format, const uint8_t* dict, size_t dl,
                       uint8_t** out) {
    size_t cap = n + n / 8 + 4096, olen = 0;
    *out = (uint8_t*)malloc(cap);
    const uint8_t* parts[1] = { in };
    size_t lens[1] = { n };
    int32_t e = oracle_deflater_run(parts, lens, 1, level, format, dict, dl, dict != NULL, NULL, 0, 0,
                                    *out, cap, &olen);
    return e == ORA_OK ? olen : (size_t)-1;
}

/* inflate() auto-detects (sd-inflate.ts:203-207); a raw stream whose first two bytes pass
 * the zlib header check is read as zlib there, so raw streams go through
 * Inflater({raw: true}) */
static int inflate_fmt(const uint8_t* comp, size_t cn, const uint8_t* want, size_t wn, const uint8_t* dict,
                       size_t dl, int raw) {
    uint8_t* out = (uint8_t*)malloc(wn + 1);
    oracle_inflate_result r;
    const uint8_t* parts[1] = { comp };
    size_t lens[1] = { cn };
    int32_t e = raw ? oracle_inflater_run(parts, lens, 1, 1, NULL, 0, out, wn + 1, &r)
                    : oracle_inflate(comp, cn, dict, dl, out, wn + 1, &r);
    int ok = e == ORA_OK && r.total_out == wn && memcmp(out, want, wn) == 0;
    free(out);
    return ok;
}
static int inflate_eq(const uint8_t* comp, size_t cn, const uint8_t* want, size_t wn, const uint8_t* dict,
                      size_t dl) {
    return inflate_fmt(comp, cn, want, wn, dict, dl, 0);
}

static void fixtures(const char* dir) {
    buf_t txt = load(dir, "paradiselost.txt"), dfl = load(dir, "paradiselost.deflate");
    buf_t gz = load(dir, "paradiselost.gz"), p1 = load(dir, "paradiselost.part1.deflate");
    buf_t p2 = load(dir, "paradiselost.part2.deflate");
    buf_t st = load(dir, "simple.txt"), sd = load(dir, "simple.deflate"), sr = load(dir, "simple.raw");
    buf_t sg = load(dir, "simple.gz"), vx = load(dir, "vertices.deflate");
    CHECK(oracle_adler32(txt.p, txt.n, 1) == -1949153550, "adler32 paradiselost");
    CHECK(oracle_crc32(txt.p, txt.n, 0) == -499006831, "crc32 paradiselost");
    CHECK(oracle_adler32(st.p, st.n, 1) == -1612443532, "adler32 simple");
    CHECK(oracle_crc32(st.p, st.n, 0) == 1488305224, "crc32 simple");
    CHECK(inflate_eq(dfl.p, dfl.n, txt.p, txt.n, NULL, 0), "inflate paradiselost.deflate");
    CHECK(inflate_eq(gz.p, gz.n, txt.p, txt.n, NULL, 0), "inflate paradiselost.gz");
    CHECK(inflate_eq(sd.p, sd.n, st.p, st.n, NULL, 0), "inflate simple.deflate");
    CHECK(inflate_eq(sr.p, sr.n, st.p, st.n, NULL, 0), "inflate simple.raw");
    CHECK(inflate_eq(sg.p, sg.n, st.p, st.n, NULL, 0), "inflate simple.gz");
    {   /* vertices: judged by its trailer only (test/index.html:120-137) */
        uint8_t* out = (uint8_t*)malloc(43440);
        oracle_inflate_result r;
        CHECK(oracle_inflate(vx.p, vx.n, NULL, 0, out, 43440, &r) == ORA_OK && r.total_out == 43440 &&
              r.checksum_verdict == 1, "inflate vertices.deflate");
        free(out);
    }
    {   /* testInflateParts (test/index.html:29-53) */
        const uint8_t* parts[2] = { p1.p, p2.p };
        size_t lens[2] = { p1.n, p2.n };
        uint8_t* out = (uint8_t*)malloc(txt.n);
        oracle_inflate_result r;
        int32_t e = oracle_inflater_run(parts, lens, 2, 0, NULL, 0, out, txt.n, &r);
        CHECK(e == ORA_OK && r.success && r.total_out == txt.n && !memcmp(out, txt.p, txt.n), "inflate parts");
        free(out);
    }
    /* the perf.html:63-69 size table; L6 byte-exact with paradiselost.deflate */
    static const size_t sizes[10] = { 0, 226188, 216830, 207545, 203828, 197239, 193730, 193295, 193162, 193162 };
    for (int lv = 1; lv <= 9; ++lv) {
        uint8_t* o;
        size_t n = deflate1(txt.p, txt.n, lv, 1, NULL, 0, &o);
        CHECK(n == sizes[lv], "deflate L%d size %zu", lv, n);
        if (lv == 6) CHECK(n == dfl.n && !memcmp(o, dfl.p, n), "deflate L6 KAT");
        if (n != (size_t)-1) CHECK(inflate_eq(o, n, txt.p, txt.n, NULL, 0), "round trip L%d", lv);
        free(o);
    }
    /* corrupted and truncated streams: any outcome but a memory error is fine */
    for (int k = 0; k < 300; ++k) {
        uint8_t* c = (uint8_t*)malloc(dfl.n);
        memcpy(c, dfl.p, dfl.n);
        size_t cut = k < 100 ? dfl.n : 1 + rnd() % (dfl.n - 1);
        for (int f = 0; f < 1 + (int)(rnd() % 4); ++f) c[rnd() % cut] ^= (uint8_t)(1u << (rnd() % 8));
        uint8_t* out = (uint8_t*)malloc(txt.n + 1024);
        oracle_inflate_result r;
        (void)oracle_inflate(c, cut, NULL, 0, out, txt.n + 1024, &r);
        free(out);
        free(c);
    }
    free(txt.p); free(dfl.p); free(gz.p); free(p1.p); free(p2.p);
    free(st.p); free(sd.p); free(sr.p); free(sg.p); free(vx.p);
}

static void edges_and_dicts(const char* dir) {
    buf_t txt = load(dir, "paradiselost.txt"), terms = load(dir, "dict_terms.txt");
    /* window-slide edges (deflate.ts:690-766) and sizes around the 16 KiB output chunk */
    static const size_t ns[] = { 0, 1, 2, 3, 257, 258, 259, 5552, 11104, 16383, 16384, 16385, 32768,
                                 65273, 65274, 65275, 65536, 98304, 131072, 200000 };
    for (size_t i = 0; i < sizeof ns / sizeof ns[0]; ++i) {
        size_t n = ns[i];
        uint8_t* in = (uint8_t*)malloc(n ? n : 1);
        memcpy(in, txt.p + 1000, n);
        for (int lv = 1; lv <= 9; lv += (n > 70000 ? 4 : 1)) {
            for (int fmt = 0; fmt < 3; ++fmt) {
                uint8_t* o;
                size_t m = deflate1(in, n, lv, fmt, NULL, 0, &o);
                if (n == 0) CHECK(m == (size_t)-1, "deflate(empty) must throw");
                else CHECK(m != (size_t)-1 && inflate_fmt(o, m, in, n, NULL, 0, fmt == 0), "edge n=%zu L%d f%d", n, lv, fmt);
                free(o);
            }
        }
        free(in);
    }
    /* incompressible input: stored blocks, the pending_buf overlay at its limits */
    for (int k = 0; k < 3; ++k) {
        size_t n = 40000 + (size_t)k * 45000;
        uint8_t* in = (uint8_t*)malloc(n);
        for (size_t j = 0; j < n; ++j) in[j] = (uint8_t)rnd();
        for (int lv = 1; lv <= 9; lv += 2) {
            uint8_t* o;
            size_t m = deflate1(in, n, lv, 1, NULL, 0, &o);
            CHECK(m != (size_t)-1, "random n=%zu L%d", n, lv);
            free(o);
        }
        free(in);
    }
    /* preset dictionaries: the reference's own word list, and lengths around 32,506 */
    static const size_t dls[] = { 1, 300, 32506, 40000 };
    for (size_t i = 0; i < sizeof dls / sizeof dls[0]; ++i) {
        const uint8_t* dict = dls[i] == 300 ? terms.p : txt.p + 5000;
        size_t dl = dls[i] == 300 ? terms.n : dls[i];
        size_t n = 30000;
        for (int lv = 1; lv <= 9; lv += 4) {
            uint8_t* o;
            size_t m = deflate1(txt.p + 60000, n, lv, 1, dict, dl, &o);
            CHECK(m != (size_t)-1 && inflate_eq(o, m, txt.p + 60000, n, dict, dl), "dict %zu L%d", dl, lv);
            free(o);
        }
    }
    /* random appends, both ways (sd-inflate.ts:87-153, sd-deflate.ts:173-253) */
    for (int k = 0; k < 20; ++k) {
        size_t n = 1 + rnd() % 150000, off = rnd() % (txt.n - n);
        int np = 1 + (int)(rnd() % 6);
        const uint8_t* parts[8];
        size_t lens[8], at = 0;
        for (int p = 0; p < np; ++p) {
            size_t l = p + 1 == np ? n - at : rnd() % (n - at + 1);
            parts[p] = txt.p + off + at;
            lens[p] = l;
            at += l;
        }
        size_t cap = n + n / 8 + 4096, olen = 0;
        uint8_t* o = (uint8_t*)malloc(cap);
        size_t ends[9];
        int lv = 1 + (int)(rnd() % 9), fmt = (int)(rnd() % 3);
        int32_t e = oracle_deflater_run_parts(parts, lens, np, lv, fmt, NULL, 0, 0, NULL, 0, 0, o, cap, &olen, ends);
        CHECK(e == ORA_OK && inflate_fmt(o, olen, txt.p + off, n, NULL, 0, fmt == 0), "deflater parts %d", k);
        if (e == ORA_OK) {   /* inflate the result back in random appends */
            const uint8_t* ip[8];
            size_t il[8], ia = 0;
            for (int p = 0; p < np; ++p) {
                size_t l = p + 1 == np ? olen - ia : rnd() % (olen - ia + 1);
                ip[p] = o + ia;
                il[p] = l;
                ia += l;
            }
            uint8_t* back = (uint8_t*)malloc(n + 1);
            oracle_inflate_result r;
            size_t po[8];
            int32_t ep = -1;
            (void)oracle_inflater_run_parts(ip, il, np, fmt == 0, NULL, 0, back, n + 1, &r, po, &ep);
            free(back);
        }
        free(o);
    }
    free(txt.p);
    free(terms.p);
}

typedef struct { const char* dir; int id; int ok; } targ_t;
static void* worker(void* p) {
    targ_t* a = (targ_t*)p;
    buf_t txt = load(a->dir, "paradiselost.txt"), dfl = load(a->dir, "paradiselost.deflate");
    a->ok = 1;
    for (int k = 0; k < 3; ++k) {
        a->ok &= inflate_eq(dfl.p, dfl.n, txt.p, txt.n, NULL, 0);
        uint8_t* o;
        size_t n = 20000 + 1000 * (size_t)a->id;
        size_t m = deflate1(txt.p + 7 * (size_t)a->id, n, 1 + (a->id + k) % 9, (a->id + k) % 3, NULL, 0, &o);
        a->ok &= m != (size_t)-1 && inflate_fmt(o, m, txt.p + 7 * (size_t)a->id, n, NULL, 0, (a->id + k) % 3 == 0);
        free(o);
        a->ok &= oracle_crc32(txt.p, txt.n, 0) == -499006831;
    }
    free(txt.p);
    free(dfl.p);
    return NULL;
}

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s <golden dir> [threads]\n", argv[0]); return 2; }
    const int nth = argc > 2 ? atoi(argv[2]) : 0;
    if (nth > 0) {   /* threaded: first calls race on the lazily built tables */
        pthread_t th[64];
        targ_t a[64];
        const int n = nth > 64 ? 64 : nth;
        for (int i = 0; i < n; ++i) { a[i].dir = argv[1]; a[i].id = i; a[i].ok = 0; pthread_create(&th[i], NULL, worker, &a[i]); }
        for (int i = 0; i < n; ++i) { pthread_join(th[i], NULL); CHECK(a[i].ok, "thread %d", i); }
    } else {
        fixtures(argv[1]);
        edges_and_dicts(argv[1]);
    }
    printf("%s: %d failures\n", nth > 0 ? "threads" : "sanitized cases", g_fail);
    return g_fail ? 1 : 0;
}
