/* visit_pred.c -- CPU study for DESIGN.md §5 "Searching only where the parse steps": on 64 KiB
 * slices of a text (C3's shape, no window slide), the positions deflate_slow (deflate.ts:1054-1182)
 * searches, against the positions a parse over CHEAP records (the first K hash-chain candidates
 * only) steps on.  Reports how many exact step positions the cheap parse misses, how many it
 * visits, and the hash-chain candidates walked by: every position (today's k_dfl_match), the exact
 * step positions, and the scheme "K candidates everywhere + the rest of the walk where the cheap
 * parse steps".
 *   gcc -O2 -o /tmp/visit_pred tools/visit_pred.c && /tmp/visit_pred tests/golden/paradiselost.txt 6 8
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define WSEG 65536
#define MAX_DIST 32506
static uint8_t b[1 << 24];
static int head[32768], prv[1 << 24];
static int cfg[10][4] = { {0,0,0,0}, {4,4,8,4}, {4,5,16,8}, {4,6,32,32}, {4,4,16,16}, {8,16,32,32},
                          {8,16,128,128}, {8,32,128,256}, {32,128,258,1024}, {32,258,258,4096} };
static int H3(int p) { return ((b[p] << 10) ^ (b[p + 1] << 5) ^ b[p + 2]) & 32767; }
static int lcp(int p, int q, int mx) { int l = 0; while (l < mx && b[q + l] == b[p + l]) ++l; return l; }

/* longest_match from best_len 2 over at most `chain` candidates; returns len (0 if < 3), *dist;
 * *walked: candidates visited */
static int search(int p, int end, int chain, int nice, int* dist, long long* walked) {
    const int first = prv[p];
    if (first < 0 || p - first > MAX_DIST) return 0;
    int mx = end - p < 258 ? end - p : 258;
    if (nice > mx) nice = mx;
    const int limit = p - MAX_DIST;
    int best = 2, bpos = -1, cur = first;
    do {
        ++*walked;
        const int l = lcp(p, cur, mx);
        if (l > best) { best = l; bpos = cur; if (l >= nice) break; }
        cur = prv[cur];
    } while (cur > limit && cur >= 0 && --chain);
    if (best < 3) return 0;
    *dist = p - bpos;
    return best;
}

typedef struct { int fl, fd, ql, qd; } Rec;
static Rec rex[WSEG], rch[WSEG];
static uint8_t vis_x[WSEG], vis_c[WSEG], have[WSEG];
static Rec rmix[WSEG];
static long long it_hist[64], it_work[64];

/* deflate_slow's step positions over records r (lengths from best_len 2: the parse takes
 * max(prev_length, record)); vis[p] = 1 where it searches */
static void parse(const Rec* r, int n, int lvl, uint8_t* vis) {
    const int good = cfg[lvl][0], lazy = cfg[lvl][1];
    int s = 0, prev_len = 2, match_len = 2, avail = 0;
    memset(vis, 0, n);
    while (s < n - 300) {
        prev_len = match_len;
        match_len = 2;
        if (r[s].fl >= 0 && prev_len < lazy) {          /* fl < 0: no search (no head in range) */
            vis[s] = 1;
            const int L = prev_len >= good ? r[s].ql : r[s].fl;
            const int D = prev_len >= good ? r[s].qd : r[s].fd;
            match_len = L > prev_len ? L : 2;           /* a longer candidate, else none better */
            if (match_len == 3 && D > 4096) match_len = 2;   /* TOO_FAR */
        }
        if (prev_len >= 3 && match_len <= prev_len) {
            s += prev_len - 1;
            avail = 0;
            match_len = 2;
        } else {
            s += 1;
            avail = 1;
        }
    }
    (void)avail;
}

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: %s file level K\n", argv[0]); return 2; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    const int n = (int)fread(b, 1, sizeof b, f);
    fclose(f);
    const int lvl = atoi(argv[2]), K = atoi(argv[3]);
    const int nice = cfg[lvl][2], chain = cfg[lvl][3];
    long long w_all = 0, w_vis = 0, w_cheap = 0, w_rest = 0, nvx = 0, nvc = 0, miss = 0, npos = 0;
    for (int s0 = 0; s0 + WSEG <= n; s0 += WSEG / 2) {
        memset(head, -1, sizeof head);
        const int end = s0 + WSEG;
        for (int p = s0; p < end - 2; ++p) { const int h = H3(p); prv[p] = head[h] >= s0 ? head[h] : -1; head[h] = p; }
        for (int i = 0; i < WSEG - 300; ++i) {
            const int p = s0 + i;
            long long wf = 0, wq = 0, wk = 0;
            int d = 0;
            Rec x = { -1, 0, -1, 0 };
            if (prv[p] >= 0 && p - prv[p] <= MAX_DIST) {
                x.fl = search(p, end, chain, nice, &d, &wf); x.fd = d;
                x.ql = search(p, end, chain >> 2, nice, &d, &wq); x.qd = d;
            }
            rex[i] = x;
            Rec c = { -1, 0, -1, 0 };
            if (prv[p] >= 0 && p - prv[p] <= MAX_DIST) {
                c.fl = search(p, end, K, nice, &d, &wk); c.fd = d;
                c.ql = c.fl; c.qd = c.fd;
            }
            rch[i] = c;
            w_all += wf;
            w_cheap += wk;
            (void)wq;                                    /* (the quarter walk is the full walk's prefix) */
            npos++;
            /* per-position full-walk counts */
            static long long wcount[WSEG];
            wcount[i] = wf;
            if (i == WSEG - 301) {
                parse(rex, WSEG, lvl, vis_x);
                parse(rch, WSEG, lvl, vis_c);
                for (int j = 0; j < WSEG - 300; ++j) {
                    nvx += vis_x[j];
                    nvc += vis_c[j];
                    if (vis_x[j]) w_vis += wcount[j];
                    if (vis_x[j] && !vis_c[j]) ++miss;
                    if (vis_c[j]) w_rest += wcount[j] > K ? wcount[j] - K : 0;
                }
                /* rounds: full records where a parse stepped so far, cheap ones elsewhere; parse;
                 * full records for the new step positions; until no step lacks a full record */
                memset(have, 0, sizeof have);
                for (int it = 0; it < 64; ++it) {
                    for (int j = 0; j < WSEG - 300; ++j) rmix[j] = have[j] ? rex[j] : rch[j];
                    parse(rmix, WSEG, lvl, vis_c);
                    long long nn = 0;
                    for (int j = 0; j < WSEG - 300; ++j)
                        if (vis_c[j] && !have[j]) { have[j] = 1; ++nn; it_work[it] += wcount[j] > K ? wcount[j] - K : 0; }
                    it_hist[it] += nn;
                    if (!nn) break;
                }
            }
        }
    }
    printf("L%d K=%d: %lld positions; exact parse searches %.1f %%; cheap parse steps %.1f %%, misses %lld (%.2f %% of "
           "exact steps)\n", lvl, K, npos, 100.0 * nvx / npos, 100.0 * nvc / npos, miss, 100.0 * miss / (nvx ? nvx : 1));
    printf("candidates per position: every position %.2f; exact steps only %.2f; K everywhere + rest at cheap steps %.2f "
           "(%.2f + %.2f)\n", (double)w_all / npos, (double)w_vis / npos, (double)(w_cheap + w_rest) / npos,
           (double)w_cheap / npos, (double)w_rest / npos);
    long long tot = 0;
    for (int it = 0; it < 64 && it_hist[it]; ++it) {
        tot += it_work[it];
        printf("  round %d: %lld new full searches (%.2f %% of positions), +%.2f candidates per position\n", it,
               it_hist[it], 100.0 * it_hist[it] / npos, (double)it_work[it] / npos);
    }
    printf("  total K everywhere + rounds: %.2f candidates per position\n", (double)(w_cheap + tot) / npos);
    return 0;
}
