"""debug: one gzip stream through InflateStreams with small output slots; per call:
out_len, out_full, running crc vs zlib.crc32 of the output so far"""
import os, sys, zlib, random
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "sd-zlib_amd", "python")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import sdz
gz = open(os.path.join(ROOT, "tests", "golden", "paradiselost.gz"), "rb").read()
for cap, parts in ((1 << 20, [gz]), (5073, [gz]), (1 << 20, [gz[:50000], gz[50000:]]), (5073, [gz[:50000], gz[50000:]])):
    st = sdz.InflateStreams(1)
    acc = b""; last = None; k = 0
    plan = list(parts)
    while True:
        if last is not None and last["out_full"]:
            ch = last["unconsumed"]
        elif (last is None or last["status"] == "TRUNCATED") and plan:
            ch = plan.pop(0)
        else:
            break
        r = st.append([ch], cap)[0]
        acc += r["data"]
        last = r
        k += 1
        ok = (r["running_checksum"] & 0xffffffff) == zlib.crc32(acc)
        if not ok or k < 3:
            print("cap", cap, "call", k, "len", len(ch), "out", len(r["data"]), "full", r["out_full"], r["status"],
                  "crc ok", ok, "in_used", r["in_used"])
        if not ok:
            break
    print("cap", cap, "calls", k, "status", last["status"], "checksum", last["checksum"], "total", len(acc))
