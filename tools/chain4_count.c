/* chain4_count.c -- CPU count behind DESIGN.md §5 "Searching 4-byte chains": per search position
 * of a text (64 KiB streams, as C3), the hash-chain entries longest_match visits (deflate.ts:827-946
 * from best_len 2: max_chain entries above limit, nice cut) against the entries sharing the first
 * 4 bytes within the same ranks (+ the rank-ordered walk to the first 3-byte entry when no 4-byte
 * one is found), and that both give the same (length, position).
 *   gcc -O2 -o /tmp/chain4_count tools/chain4_count.c && /tmp/chain4_count tests/golden/paradiselost.txt 128 128
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint8_t b[1 << 24];
static int head[32768], prv[1 << 24], idx[1 << 24], cnt[32768], h4[1 << 20], p4[1 << 24];
static int H3(int p) { return ((b[p] << 10) ^ (b[p + 1] << 5) ^ b[p + 2]) & 32767; }
static int lcp(int p, int q) { int l = 0; while (l < 258 && b[q + l] == b[p + l]) ++l; return l; }

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: %s file max_chain nice\n", argv[0]); return 2; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    const int n = (int)fread(b, 1, sizeof b, f);
    fclose(f);
    const int K = atoi(argv[2]), nice = atoi(argv[3]), seg = 65536;
    long long c3 = 0, c4 = 0, c3f = 0, np = 0, bad = 0;
    for (int s0 = 0; s0 + seg <= n; s0 += seg) {
        memset(head, -1, sizeof head); memset(cnt, 0, sizeof cnt); memset(h4, -1, sizeof h4);
        for (int p = s0; p < s0 + seg - 8; ++p) {
            const int h = H3(p);
            prv[p] = head[h]; head[h] = p; idx[p] = cnt[h]++;      /* idx: rank counter per hash */
            uint32_t k = b[p] | b[p + 1] << 8 | b[p + 2] << 16 | (uint32_t)b[p + 3] << 24;
            k = (k * 2654435761u) >> 12;
            p4[p] = h4[k]; h4[k] = p;
        }
        for (int p = s0; p < s0 + seg - 300; ++p) {
            const int limit = p - 32506, first = prv[p];
            if (first < 0 || p - first > 32506) continue;            /* no search (deflate.ts:1092) */
            ++np;
            int best = 2, bpos = -1, chain = K, cur = first;
            do { ++c3; const int l = lcp(p, cur); if (l > best) { best = l; bpos = cur; if (l >= nice) break; }
                 cur = prv[cur]; } while (cur > limit && cur >= 0 && --chain);
            int sb = 2, spos = -1;
            for (int q = p4[p]; q >= 0; q = p4[q]) {                  /* same 4-byte hash, exact check */
                if (q <= limit && q != first) break;
                if (memcmp(b + q, b + p, 4)) continue;
                if (idx[p] - idx[q] > K) break;                     /* past max_chain ranks */
                ++c4;
                const int l = lcp(p, q);
                if (l > sb) { sb = l; spos = q; if (l >= nice) break; }
            }
            if (sb < 4) {                                            /* the first 3-byte entry */
                int c = first, ch = K;
                do { ++c3f; if (lcp(p, c) >= 3) { sb = 3; spos = c; break; } c = prv[c]; } while (c > limit && c >= 0 && --ch);
            }
            const int r1 = best > 2 ? best : 0, r2 = sb > 2 ? sb : 0;
            if (!(r1 == r2 && (r1 == 0 || bpos == spos))) ++bad;
        }
    }
    printf("max_chain %d nice %d: %lld searches, hash-chain entries %.2f, 4-byte candidates %.2f, "
           "3-byte walk %.2f per search, mismatches %lld\n", K, nice, np, (double)c3 / np, (double)c4 / np,
           (double)c3f / np, bad);
    return 0;
}
