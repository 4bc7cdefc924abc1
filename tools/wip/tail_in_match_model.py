#!/usr/bin/env python3
"""CPU model (analysis aid, not product): the last-position searches as k_dfl_match now runs them
(absolute positions, the LDS-staged window with the larger window-offset group's bytes past the
input, limit P - MAX_DIST, window index 0 of that offset NIL) against tail_search's reference
coordinates (slide offset, win_byte, rebased links), for every position of the larger group.
  python3 tools/wip/tail_in_match_model.py     -> prints mismatches (expects none)"""
import random
import sys

W = 32768
WIN = 65536
MIN_LOOK = 262
MAX_MATCH = 258
MAX_DIST = W - MIN_LOOK
HMASK = 0x7fff


def links(d):
    n = len(d)
    head, pv = {}, [0] * n
    for p in range(n):
        if p + 2 >= n:
            continue
        h = ((d[p] << 10) ^ (d[p + 1] << 5) ^ d[p + 2]) & HMASK
        q = head.get(h)
        pv[p] = p - q if q is not None and p - q <= 32767 else 0
        head[h] = p
    return pv


def slide_off(n, P):
    off = 0
    if P >= WIN - MIN_LOOK + 1 and n >= WIN:
        e = (P - (WIN - MIN_LOOK + 1)) // W + 1
        emid = (n - WIN) // W + 1
        off = W * min(e, emid)
    while True:
        fe = min(n, off + WIN)
        if fe - P < MIN_LOOK and P - off >= WIN - MIN_LOOK:
            off += W
        else:
            return off


def win_byte(d, n, off, i):
    e = off // W
    while True:
        base = e * W
        F = min(n - base, WIN)
        if i < F:
            return d[base + i]
        if e == 0:
            return 0
        if i < W:
            i += W
        e -= 1


def ref_search(d, pv, n, P, chain, nice):
    off = slide_off(n, P)
    s = P - off

    def prev_of(q):
        dd = pv[q]
        r = q - dd
        return r - off if dd and r > off else 0

    wb = lambda i: win_byte(d, n, off, i)
    cur = prev_of(P)
    if cur == 0 or ((s - cur) & 0xffff) > MAX_DIST:
        return (0, 0)
    nice = min(nice, n - P)
    limit = s - MAX_DIST if s > MAX_DIST else 0
    qchain = chain >> 2
    best, bst, qb, qs, k = 2, 0, -1, 0, 0
    while True:
        m = cur
        nx = prev_of(m + off)
        if wb(m + best) == wb(s + best) and wb(m + best - 1) == wb(s + best - 1) and wb(m) == wb(s) and wb(m + 1) == wb(s + 1):
            ln = 3
            while ln < MAX_MATCH and wb(s + ln) == wb(m + ln):
                ln += 1
            if ln > best:
                bst, best = m, ln
                if ln >= nice:
                    break
        k += 1
        if k == qchain:
            qb, qs = best, bst
        cur = nx
        chain -= 1
        if not (cur > limit and chain != 0):
            break
    if qb < 0:
        qb, qs = best, bst
    full = (best, s - bst) if best > 2 else (0, 0)
    quarter = (qb, s - qs) if qb > 2 else (0, 0)
    return full, quarter


def new_search(d, pv, n, P, chain, nice, offM, ext):
    # absolute coordinates; bytes past n from the group's staged extension
    b = lambda q: d[q] if q < n else ext[q - n]
    r = P - pv[P] if pv[P] else -1
    if r < 0 or P - r > MAX_DIST or not r > offM:
        return (0, 0)
    nice = min(nice, n - P)
    limit = P - MAX_DIST
    qchain = chain >> 2
    best, bst, qb, qs, k = 2, 0, -1, 0, 0
    cur = r
    while True:
        c = cur
        nx = c - pv[c] if pv[c] else -1
        ln = 0
        while ln < MAX_MATCH and b(P + ln) == b(c + ln):
            ln += 1
        if b(c + best) == b(P + best) and ln > best:
            bst, best = c, ln
            if ln >= nice:
                break
        k += 1
        if k == qchain:
            qb, qs = best, bst
        cur = nx
        chain -= 1
        if not (cur > limit and chain != 0):
            break
    if qb < 0:
        qb, qs = best, bst
    full = (best, P - bst) if best > 2 else (0, 0)
    quarter = (qb, P - qs) if qb > 2 else (0, 0)
    return full, quarter


def groups(n, tail):
    offA, offB = slide_off(n, tail), slide_off(n, n - 1)
    ps = n
    if offA != offB:
        ps = next(P for P in range(tail + 1, n) if slide_off(n, P) == offB)
    if n - ps >= ps - tail:
        return (tail if ps == n else ps), n, offB
    return tail, ps, offA


def main():
    text = open("tests/golden/paradiselost.txt", "rb").read()
    rng = random.Random(5)
    cases = []
    for n in (65273, 65274, 65275, 65536, 65537, 65536 + 262, 98041, 98304, 98305, 131077):
        cases.append(text[:n])
    for n in (65536, 98304):
        unit = bytes(rng.getrandbits(8) for _ in range(300))
        cases.append((unit * (n // 300 + 1))[:n])
        t = bytearray(text[:n])
        t[n - 400:] = t[n - 400 - 32768:n - 32768]
        cases.append(bytes(t))
    bad = 0
    for d in cases:
        n = len(d)
        pv = links(d)
        tail = n - 262
        mlo, mhi, offM = groups(n, tail)
        ext = bytes(win_byte(d, n, offM, n + j - offM) for j in range(MAX_MATCH + 16))
        for level, (chain, nice) in {4: (16, 16), 6: (128, 128), 9: (4096, 258)}.items():
            for P in range(mlo, min(mhi, n - 2)):
                a = ref_search(d, pv, n, P, chain, nice)
                b = new_search(d, pv, n, P, chain, nice, offM, ext)
                if a != b:
                    bad += 1
                    if bad < 10:
                        print("n %d L%d P %d ref %s new %s" % (n, level, P, a, b))
        print("n %d group [%d, %d) off %d checked" % (n, mlo, mhi, offM), flush=True)
    print("mismatches:", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
