#!/usr/bin/env python3
"""Token statistics of a zlib/raw DEFLATE stream (pure Python; analysis aid)."""
import sys, collections, zlib

def tokens(data, raw=False):
    pos = 0 if raw else 2
    bitbuf = 0; bitcnt = 0
    def need(n):
        nonlocal bitbuf, bitcnt, pos
        while bitcnt < n:
            bitbuf |= data[pos] << bitcnt; pos += 1; bitcnt += 8
    def get(n):
        nonlocal bitbuf, bitcnt
        need(n); v = bitbuf & ((1 << n) - 1); bitbuf >>= n; bitcnt -= n; return v
    def build(lens):
        code = 0; tab = {}
        for L in range(1, 16):
            for s, l in enumerate(lens):
                if l == L:
                    tab[(L, code)] = s; code += 1
            code <<= 1
        return tab
    def dec(tab):
        code = 0
        for L in range(1, 16):
            code = (code << 1) | get(1)
            if (L, code) in tab: return tab[(L, code)]
        raise ValueError
    LB = [3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258]
    LE = [0]*8+[1]*4+[2]*4+[3]*4+[4]*4+[5]*4+[0]
    DB = [1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577]
    DE = [0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13]
    out = []; blocks = 0
    while True:
        last = get(1); bt = get(2); blocks += 1
        if bt == 2:
            hl, hd, hc = get(5) + 257, get(5) + 1, get(4) + 4
            order = [16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15]
            cl = [0]*19
            for i in range(hc): cl[order[i]] = get(3)
            ct = build(cl); lens = []
            while len(lens) < hl + hd:
                c = dec(ct)
                if c < 16: lens.append(c)
                elif c == 16: lens += [lens[-1]] * (3 + get(2))
                elif c == 17: lens += [0] * (3 + get(3))
                else: lens += [0] * (11 + get(7))
            lt, dt = build(lens[:hl]), build(lens[hl:])
        elif bt == 1:
            lt = build([8]*144 + [9]*112 + [7]*24 + [8]*8); dt = build([5]*30)
        else:
            raise SystemExit("stored block")
        while True:
            s = dec(lt)
            if s < 256: out.append(("L", 1, 0))
            elif s == 256: break
            else:
                i = s - 257; ln = LB[i] + get(LE[i]); d = dec(dt); dist = DB[d] + get(DE[d])
                out.append(("M", ln, dist))
        if last: break
    return out, blocks

def main():
    data = open(sys.argv[1], "rb").read()
    toks, blocks = tokens(data)
    lits = sum(1 for t in toks if t[0] == "L"); ms = [t for t in toks if t[0] == "M"]
    print("blocks", blocks, "tokens", len(toks), "literals", lits, "matches", len(ms))
    print("avg match len %.2f" % (sum(m[1] for m in ms) / len(ms)), "bytes from matches", sum(m[1] for m in ms))
    dists = sorted(m[2] for m in ms)
    for q in (0.1, 0.25, 0.5, 0.75, 0.9):
        print("dist q%.2f = %d" % (q, dists[int(q * len(dists))]))
    print("frac dist<8: %.3f" % (sum(1 for d in dists if d < 8) / len(dists)))
    lens = sorted(m[1] for m in ms)
    for q in (0.5, 0.9, 0.99):
        print("len q%.2f = %d" % (q, lens[int(q * len(lens))]))


if __name__ == "__main__":
    main()
