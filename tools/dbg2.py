import sys, os, random
sys.path.insert(0, "sd-zlib_amd/python")
import sdz, zlib
g = "tests/golden/"
n = sys.argv[1] if len(sys.argv) > 1 else "paradiselost.deflate"
comp = open(g + n, "rb").read()
r = sdz.inflate_batch([comp], [600000], sdz.FMT_AUTO)[0]
print(n, r["status"], r["zmsg"], len(r["data"]), flush=True)
