"""debug: the batched incremental test, checking every gzip stream's running crc per call"""
import os, sys, zlib, random
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "sd-zlib_amd", "python")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import sdz
G = lambda n: open(os.path.join(ROOT, "tests", "golden", n), "rb").read()
comp, text, gz, v = G("paradiselost.deflate"), G("paradiselost.txt"), G("paradiselost.gz"), G("vertices.deflate")
srcs = [comp, gz, v, zlib.compress(text[:50000], 1), zlib.compress(text[7:90000], 9)]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
streams = [srcs[i % len(srcs)] for i in range(n)]
rng = random.Random(11)
plans = []
for s in streams:
    cuts = sorted(rng.sample(range(1, len(s)), rng.randint(1, 4)))
    c = [0] + cuts + [len(s)]
    plans.append([s[a:b] for a, b in zip(c, c[1:])])
print("plan 1:", [len(p) for p in plans[1]])
st = sdz.InflateStreams(n)
got = [b""] * n; last = [None] * n
cap = [4096 + 977 * i for i in range(n)]
k = 0
bad = set()
while True:
    chunks = []
    for i in range(n):
        if last[i] is not None and last[i]["out_full"]:
            chunks.append(last[i]["unconsumed"])
        elif (last[i] is None or last[i]["status"] == "TRUNCATED") and plans[i]:
            chunks.append(plans[i].pop(0))
        else:
            chunks.append(b"")
    if all(not c for c in chunks) and all(r is not None and not r["out_full"] for r in last):
        break
    res = st.append(chunks, cap)
    k += 1
    for i, r in enumerate(res):
        got[i] += r["data"]
        last[i] = r
        if r["container"] == "gzip" and i not in bad:
            ok = (r["running_checksum"] & 0xffffffff) == zlib.crc32(got[i])
            if not ok:
                bad.add(i)
                print("call", k, "stream", i, "chunk", len(chunks[i]), "out", len(r["data"]), "full", r["out_full"],
                      r["status"], "total", len(got[i]), "rc", r["running_checksum"] & 0xffffffff, "want", zlib.crc32(got[i]))
print("calls", k, [(l["status"], l["checksum"]) for l in last])
