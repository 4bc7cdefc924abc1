"""Development aid: decode a raw DEFLATE stream into (block type, symbols) for diffing two
encoders' outputs symbol by symbol.  Pure Python, small inputs only."""
import sys

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115,
         131, 163, 195, 227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537,
         2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class Bits:
    def __init__(self, data):
        self.d, self.p = data, 0

    def get(self, n):
        v = 0
        for i in range(n):
            v |= ((self.d[self.p >> 3] >> (self.p & 7)) & 1) << i
            self.p += 1
        return v


def huff(lengths):
    codes, code, bl = {}, 0, [0] * 16
    for l in lengths:
        bl[l] += 1
    bl[0] = 0
    nxt, code = [0] * 16, 0
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    for s, l in enumerate(lengths):
        if l:
            codes[(l, nxt[l])] = s
            nxt[l] += 1
    return codes


def sym(b, t):
    code = l = 0
    while True:
        code = (code << 1) | b.get(1)
        l += 1
        if (l, code) in t:
            return t[(l, code)]


def blocks(data):
    b = Bits(data)
    out = []
    while True:
        final, typ = b.get(1), b.get(2)
        syms = []
        if typ == 0:
            b.p = (b.p + 7) & ~7
            ln = b.get(16); b.get(16)
            b.p += 8 * ln
            out.append(("stored", ln, b.p))
        else:
            if typ == 1:
                lt = huff([8] * 144 + [9] * 112 + [7] * 24 + [8] * 8); dt = huff([5] * 30)
                hdr = None
            else:
                hl, hd, hc = b.get(5) + 257, b.get(5) + 1, b.get(4) + 4
                cl = [0] * 19
                for i in range(hc):
                    cl[ORDER[i]] = b.get(3)
                ct = huff(cl)
                lens = []
                while len(lens) < hl + hd:
                    s = sym(b, ct)
                    if s < 16: lens.append(s)
                    elif s == 16: lens += [lens[-1]] * (3 + b.get(2))
                    elif s == 17: lens += [0] * (3 + b.get(3))
                    else: lens += [0] * (11 + b.get(7))
                lt, dt = huff(lens[:hl]), huff(lens[hl:])
                hdr = (hl, hd, hc, cl, lens)
            while True:
                s = sym(b, lt)
                if s < 256: syms.append(s)
                elif s == 256: break
                else:
                    c = s - 257
                    ln = LBASE[c] + b.get(LEXT[c])
                    dc = sym(b, dt)
                    syms.append((ln, DBASE[dc] + b.get(DEXT[dc])))
            out.append(("static" if typ == 1 else "dynamic", syms, hdr, b.p))
        if final:
            return out


def diff(a, b):
    A, B = blocks(a), blocks(b)
    print("blocks", len(A), len(B))
    for i, (x, y) in enumerate(zip(A, B)):
        print("block", i, x[0], y[0], "end bits", x[-1], y[-1])
        if x[0] != y[0]:
            return
        if x[0] == "stored":
            continue
        if x[2] != y[2]:
            print(" header differs", x[2] and x[2][:3], y[2] and y[2][:3])
        for k, (s, t) in enumerate(zip(x[1], y[1])):
            if s != t:
                print(" first symbol diff at", k, s, t, "context", x[1][max(0, k - 3):k + 3], y[1][max(0, k - 3):k + 3])
                return
        if len(x[1]) != len(y[1]):
            print(" symbol counts", len(x[1]), len(y[1]))
            return


if __name__ == "__main__":
    a, b = open(sys.argv[1], "rb").read(), open(sys.argv[2], "rb").read()
    sk = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    diff(a[sk:], b[sk:])
