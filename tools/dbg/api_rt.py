import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sd-zlib_amd", "python"), os.path.join(ROOT, "oracle")]
import sdz, oracle as O
t = open(os.path.join(ROOT, "tests/golden/paradiselost.txt"), "rb").read()
for n in (20000, 70000, len(t)):
    for fmt in ("deflate", "gzip"):
        c = sdz.deflate_batch([t[:n]], 6, fmt, b"paradiselost.orig" if fmt == "gzip" else b"", 0)[0]
        ref = O.deflate(t[:n], level=6, format=fmt, file_name="paradiselost.orig" if fmt == "gzip" else None, mtime=0)
        print(n, fmt, c["status"], len(c["data"]), len(ref), c["data"] == ref, c["data"][:16].hex(), flush=True)
        r = sdz.inflate_batch([ref], [n + 64])[0]
        print("  inflate_batch", r["status"], r["success"], r["data"] == t[:n], flush=True)
        inf = sdz.Inflater()
        try:
            out = b"".join(inf.append(ref))
            print("  Inflater", out == t[:n], inf.finish(), flush=True)
        except Exception as e:
            print("  Inflater EXC", e, flush=True)
