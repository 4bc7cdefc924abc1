"""GPU parity of the incremental inflate path: Inflater.append() across calls
(sd-inflate.ts:87-179) with the decoder state, window, unfinished input and running
checksum kept on the device between calls.

The bar, per append(): the output bytes the reference's append() returns for the same
chunk (the oracle restates its 16 KiB chunk loop, oracle_inflater_run_parts), and at the
end the finish() verdicts -- including the running adler32's NMAX quirk, which depends on
where each append's output ends (adler32.ts:67).  Where the reference fails on its own
defects (a dynamic block header split across appends returns STREAM_ERROR)
the GPU output is checked against the original bytes instead.
"""
import random
import zlib

import pytest

import oracle as O
import sdz
from conftest import golden

pytestmark = pytest.mark.gpu


def split(data, cuts):
    cuts = [0] + sorted(cuts) + [len(data)]
    return [data[a:b] for a, b in zip(cuts, cuts[1:])]


def run_inflater(parts, raw=False, dictionary=None):
    """The Python mirror (sdz.Inflater): per-append outputs, finish(), the error if any."""
    opts = {"raw": raw}
    if dictionary is not None:
        opts["dictionary"] = dictionary
    inf = sdz.Inflater(opts)
    outs, err = [], None
    for p in parts:
        try:
            outs.append(b"".join(inf.append(p)))
        except sdz.SdzError as e:
            err = str(e)
            break
    return outs, inf.finish(), err


def a10_split(o):
    """The reference's append() threw STREAM_ERROR ("inflate error: " + empty z.msg):
    a dynamic block header split across appends."""
    return o["error"] == 1 and o["zmsg"] == 0


def check_parts(parts, truth, raw=False, dictionary=None):
    o = O.inflater_parts(parts, raw=raw, dictionary=dictionary)
    outs, fin, err = run_inflater(parts, raw, dictionary)
    if a10_split(o):
        assert err is None and b"".join(outs) == truth and fin["success"]
        return "a10"
    assert err is None, err
    assert o["error"] == 0, o["message"]
    nz = [p for p in parts if p]
    assert len(outs) == len(nz)
    assert outs == [x for p, x in zip(parts, o["parts_out"]) if p]
    assert b"".join(outs) == truth
    for k in ("success", "complete", "checksum", "fileSize", "fileName"):
        assert fin[k] == o[k], (k, fin[k], o[k])
    return "ok"


def test_inflate_parts_like_reference_test(paradise):
    """test/index.html:29-53: paradiselost.deflate in two appends (96,125 + 97,605 B)."""
    comp, text = golden("paradiselost.deflate"), paradise
    p1 = golden("paradiselost.part1.deflate")
    p2 = golden("paradiselost.part2.deflate")
    assert p1 + p2 == comp
    assert check_parts([p1, p2], text) == "ok"


@pytest.mark.parametrize("name", ["paradiselost.deflate", "paradiselost.gz", "vertices.deflate"])
def test_random_splits_match_oracle(name):
    comp = golden(name)
    truth = O.inflater_run([comp])["data"]
    rng = random.Random(len(comp))
    kinds = []
    for _ in range(6):
        k = rng.randint(1, 6)
        cuts = rng.sample(range(1, len(comp)), k)
        kinds.append(check_parts(split(comp, cuts), truth))
    assert kinds.count("ok") >= 3


def test_small_pieces_cross_every_unit():
    """simple.* and a small dynamic stream fed in 1..7-byte pieces: headers, block headers,
    symbols, stored lengths and trailers all span appends."""
    rng = random.Random(7)
    for name in ("simple.deflate", "simple.gz", "simple.raw"):
        comp = golden(name)
        truth = golden("simple.txt")
        cuts, p = [], 0
        while True:
            p += rng.randint(1, 7)
            if p >= len(comp):
                break
            cuts.append(p)
        check_parts(split(comp, cuts), truth, raw=name.endswith(".raw"))
    text = golden("paradiselost.txt")[:3000]
    comp = zlib.compress(text, 9)
    for step in (1, 3, 5):
        parts = [comp[i:i + step] for i in range(0, len(comp), step)]
        check_parts(parts, text)


def quirk_splits(count=3):
    """(text, compressed, cut) where the first append's output is 5552 or 11104 bytes mod
    16 KiB: the output length at a cut is found by bisection over prefixes (oracle)."""
    full = golden("paradiselost.txt")
    found = []
    for off in range(0, 400000, 20000):
        text = full[off:off + 60000]
        comp = zlib.compress(text, 6)

        def outlen(cut):
            return len(O.inflater_parts([comp[:cut]], out_cap=1 << 17)["data"])

        for T in (5552, 11104, 21936, 27488, 38320, 43872, 54704):
            lo, hi = 1, len(comp)
            while lo < hi:
                m = (lo + hi) // 2
                if outlen(m) >= T:
                    hi = m
                else:
                    lo = m + 1
            if outlen(lo) == T:
                found.append((text, comp, lo))
                break
        if len(found) >= count:
            break
    return found


def test_chunkwise_adler_quirk_across_appends():
    """An append whose output is 5552 or 11104 bytes (mod 16 KiB) makes the reference's
    running adler32 skip its mod (adler32.ts:67): its finish() then says "mismatch" on a
    valid stream.  The GPU's running checksum must say the same."""
    hits = quirk_splits()
    assert len(hits) >= 2
    for text, comp, cut in hits:
        parts = [comp[:cut], comp[cut:]]
        o = O.inflater_parts(parts)
        assert o["checksum"] == "mismatch" and not o["success"]
        outs, fin, err = run_inflater(parts)
        assert err is None and outs == o["parts_out"]
        assert fin["checksum"] == "mismatch" and not fin["success"] and fin["complete"]
        # and one call later the state carries on: a third append split still agrees
        parts3 = [comp[:cut], comp[cut:cut + 700], comp[cut + 700:]]
        assert check_parts(parts3, text) == "ok"


def test_dictionary_roundtrip_in_parts():
    """test/index.html:173-208: a preset dictionary, fed in parts."""
    words = b" ".join(golden("paradiselost.txt").split()[:400])
    text = golden("paradiselost.txt")[1000:9000]
    comp = O.deflate(text, level=6, dictionary=words)
    rng = random.Random(3)
    for _ in range(3):
        cuts = rng.sample(range(1, len(comp)), 3)
        check_parts(split(comp, cuts), text, dictionary=words)
    outs, fin, err = run_inflater([comp[:10], comp[10:]])
    assert err == "Custom dictionary required for this data"


def test_append_after_end_and_errors():
    comp = golden("paradiselost.deflate")
    inf = sdz.Inflater()
    inf.append(comp)
    with pytest.raises(sdz.SdzError, match="bad input data"):
        inf.append(b"\x00\x01")
    bad = bytearray(golden("simple.deflate"))
    bad[2] = (bad[2] & 0xF9) | 0x06                         # BTYPE 3
    o = O.inflater_parts([bytes(bad[:3]), bytes(bad[3:])])
    outs, fin, err = run_inflater([bytes(bad[:3]), bytes(bad[3:])])
    assert err == o["message"] == "inflate error: invalid block type"


def test_batched_streams_with_small_output_slots(paradise):
    """Many Inflaters in one device call, each with its own split points and an output slot
    smaller than its output (out_full: called again with no new input)."""
    comp, text = golden("paradiselost.deflate"), paradise
    gz = golden("paradiselost.gz")
    v = golden("vertices.deflate")
    srcs = [comp, gz, v, zlib.compress(text[:50000], 1), zlib.compress(text[7:90000], 9)]
    n = 12
    streams = [srcs[i % len(srcs)] for i in range(n)]
    truth = [O.inflater_run([s])["data"] for s in streams]
    rng = random.Random(11)
    plans, refs = [], []
    for s in streams:
        cuts = sorted(rng.sample(range(1, len(s)), rng.randint(1, 4)))
        plans.append(split(s, cuts))
        refs.append(O.inflater_parts(plans[-1]))
    st = sdz.InflateStreams(n)
    got = [b""] * n
    last = [None] * n
    k = 0
    cap = [4096 + 977 * i for i in range(n)]
    while True:
        chunks = []
        for i in range(n):
            if last[i] is not None and last[i]["out_full"]:
                chunks.append(last[i]["unconsumed"])      # bytes the stream held back
            elif (last[i] is None or last[i]["status"] == "TRUNCATED") and plans[i]:
                chunks.append(plans[i].pop(0))
            else:
                chunks.append(b"")
        if all(not c for c in chunks) and all(r is not None and not r["out_full"] for r in last):
            break
        res = st.append(chunks, cap)
        for i, r in enumerate(res):
            got[i] += r["data"]
            last[i] = r
        k += 1
        assert k < 5000
    for i in range(n):
        assert got[i] == truth[i], i
        assert last[i]["status"] == "OK" and last[i]["complete"]
        if not a10_split(refs[i]):                        # the reference's own verdict for these appends
            assert (last[i]["success"], last[i]["checksum"]) == (refs[i]["success"], refs[i]["checksum"]), i


def test_node_facade_smoke():
    """The drop-in ES module over the N-API addon (tests/node/smoke.mjs): the reference's
    test/index.html cases, incremental appends included."""
    import os
    import shutil
    import subprocess
    node = shutil.which("node")
    if node is None:
        pytest.skip("node not installed")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([node, os.path.join(root, "tests", "node", "smoke.mjs")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


def test_inflater_arrays_match_reference_chunks():
    """Inflater.append returns the reference's arrays, not only its bytes: one Uint8Array per
    16 KiB ZStream pass (sd-inflate.ts:101-150), as the oracle's restatement pushes them."""
    text = golden("paradiselost.txt")
    rng = random.Random(44)
    cases = [[golden("paradiselost.part1.deflate"), golden("paradiselost.part2.deflate")],
             [golden("paradiselost.gz")]]
    for _ in range(6):
        comp = zlib.compress(text[rng.randrange(200000):][:rng.randrange(1000, 250000)], rng.randint(1, 9))
        cases.append(split(comp, [rng.randrange(len(comp)) for _ in range(rng.randint(0, 4))]))
    for parts in cases:
        per, ref = O.inflater_chunks(parts)
        inf = sdz.Inflater()
        got = [[len(a) for a in inf.append(p)] for p in parts]
        assert got == [per[k] if parts[k] else [] for k in range(len(parts))]
        assert inf.finish()["success"] == ref["success"]


def test_deflater_arrays_header_passes_trailer():
    """Deflater.append/finish return the reference's arrays (sd-deflate.ts:199-250): the
    container header alone, 16 KiB passes, the trailer alone; and its error text."""
    text = golden("paradiselost.txt")
    for fmt, hlen, tlen in (("deflate", 2, 4), ("gzip", 10 + len("x.txt") + 1, 8), ("raw", 0, 0)):
        d = sdz.Deflater({"level": 6, "format": fmt, "fileName": "x.txt" if fmt == "gzip" else None})
        d.mtime = 0
        a = d.append(text[:100000])
        b = d.append(text[100000:])
        f = d.finish()
        if hlen:
            assert len(a[0]) == hlen
        body = a[1:] if hlen else a
        assert all(len(x) == 16384 for x in body[:-1]) and all(len(x) == 16384 for x in b[:-1])
        if tlen:
            assert len(f[-1]) == tlen
        merged = b"".join(a + b + f)
        assert merged == O.deflater_run([text[:100000], text[100000:]], 6, fmt,
                                        file_name="x.txt" if fmt == "gzip" else None, mtime=0)
    # the reference throws "deflating: " + z.msg, and deflate.ts never sets z.msg
    d = sdz.Deflater({"level": 1})
    d.append(b"abc")
    d.finish()
    with pytest.raises(sdz.SdzError) as e:
        d.append(b"more")                                 # append after finish: a stream error
    assert str(e.value) == "deflating: "


def test_gzip_long_file_name_kept():
    """a FNAME longer than 64 KiB comes back whole (the facade keeps the input
    until the header is past, not a fixed 64 KiB head)"""
    name = "n" * 70000 + ".txt"
    data = golden("simple.txt") * 50
    comp = O.deflate(data, level=6, format="gzip", file_name=name, mtime=0)
    inf = sdz.Inflater()
    out = b"".join(inf.append(comp))
    res = inf.finish()
    assert out == data and res["success"] and res["fileName"] == name


def test_inflater_one_pass_first_append(monkeypatch):
    """A first append of >= 32 KiB holding a whole stream takes the one-pass path (block-parallel
    decode): its bytes and record equal the incremental path's; a stream continuing past the
    append, or an error, falls back to the incremental path untouched."""
    comp = golden("paradiselost.gz")
    text = golden("paradiselost.txt")

    def one(parts):
        inf = sdz.Inflater()
        out = b"".join(b"".join(inf.append(p)) for p in parts)
        return out, inf.finish()
    a = one([comp])
    monkeypatch.setenv("SDZ_INFLATER_STREAM_ONLY", "1")
    b = one([comp])
    monkeypatch.delenv("SDZ_INFLATER_STREAM_ONLY")
    assert a == b and a[0] == text and a[1]["success"] and a[1]["fileName"] == "paradiselost.txt"
    # the stream continues past the first append: the incremental path, as before
    c = one([comp[:100000], comp[100000:]])
    assert c == a
    # a damaged stream: the same error either way
    bad = bytearray(golden("paradiselost.deflate"))
    bad[50000] ^= 0xFF
    errs = []
    for env in (None, "1"):
        if env:
            monkeypatch.setenv("SDZ_INFLATER_STREAM_ONLY", env)
        inf = sdz.Inflater()
        try:
            inf.append(bytes(bad))
            errs.append(("ok", inf.finish()["success"]))
        except sdz.SdzError as e:
            errs.append(("err", str(e)))
    assert errs[0] == errs[1]
