"""GPU parity of the incremental deflate path: Deflater.append() /
finish() across calls (sd-deflate.ts:173-253 over deflate.ts:1218-1327 with NO_FLUSH /
FINISH), the compressor's window, hash chains, pending block, bit buffer and running
checksum kept on the device between calls (k_deflate_stream).

The bar, per call: the bytes the reference's append()/finish() returns for the same chunk,
concatenated -- the oracle restates the reference's Deflater loop and records where each
call's output ends (oracle_deflater_run_parts) -- and so, at the end, the stream itself.
"""
import random

import pytest

import oracle as O
import sdz

pytestmark = pytest.mark.gpu


def split(data, cuts):
    cuts = [0] + sorted(cuts) + [len(data)]
    return [data[a:b] for a, b in zip(cuts, cuts[1:])]


def run_deflater(parts, level, fmt, file_name=None, dictionary=None):
    opts = {"level": level, "format": fmt}
    if file_name:
        opts["fileName"] = file_name
    if dictionary is not None:
        opts["dictionary"] = dictionary
    d = sdz.Deflater(opts)
    d.mtime = 1234567
    outs = [b"".join(d.append(p)) for p in parts]
    outs.append(b"".join(d.finish()))
    return outs


@pytest.mark.parametrize("level", range(1, 10))
def test_per_call_output_matches_reference(paradise, level):
    rng = random.Random(100 + level)
    src = paradise[:200000]              # (the serial compressor runs one lane per stream)
    for fmt in ("deflate", "gzip", "raw"):
        for ncut in (0, 1, 5, 17):
            cuts = rng.sample(range(1, len(src)), ncut)
            parts = split(src, cuts)
            if ncut > 1:
                parts.insert(1, b"")                    # an empty append returns nothing
            exp = O.deflater_parts(parts, level=level, format=fmt, file_name="p.txt" if fmt == "gzip" else None,
                                   mtime=1234567)
            got = run_deflater(parts, level, fmt, "p.txt" if fmt == "gzip" else None)
            assert got == exp, (level, fmt, ncut)


def test_small_and_ragged_appends(paradise):
    """Appends of 1-300 bytes: every call stops where deflate(NO_FLUSH) returns NeedMore
    (lookahead < MIN_LOOKAHEAD), the window slides between calls."""
    rng = random.Random(7)
    data = paradise[:150000]
    o, parts = 0, []
    while o < len(data):
        z = rng.choice([1, 2, 3, 7, 100, 261, 262, 263, 300, 4096])
        parts.append(data[o:o + z])
        o += z
    for level in (1, 4, 6, 9):
        exp = O.deflater_parts(parts, level=level, format="deflate")
        got = run_deflater(parts, level, "deflate")
        assert got == exp, level


def test_dictionary_in_parts(paradise):
    terms = paradise[1000:9000]
    parts = split(paradise[:120000], [5000, 20000, 65536, 70000])   # (no 5552-byte append: NMAX quirk)
    for level in (1, 6, 9):
        exp = O.deflater_parts(parts, level=level, format="deflate", dictionary=terms)
        got = run_deflater(parts, level, "deflate", dictionary=terms)
        assert got == exp, level
        assert sdz.inflate(b"".join(got), terms) == paradise[:120000]


def test_batched_deflaters(paradise):
    """Many Deflaters in one device call per step, each with its own chunk sizes (empty
    chunks included), ended together; a last chunk may come with the finish."""
    rng = random.Random(11)
    n = 24
    srcs, plans = [], []
    for i in range(n):
        a = rng.randrange(0, len(paradise) - 60000)
        src = paradise[a:a + rng.randint(1, 60000)]
        srcs.append(src)
        plans.append(split(src, rng.sample(range(1, len(src)), min(len(src) - 1, rng.randint(0, 6)))))
    steps = max(len(p) for p in plans)
    for level, fmt in ((6, "deflate"), (9, "gzip"), (2, "raw")):
        st = sdz.DeflateStreams(n, level=level, format=fmt, file_name_latin1=b"b.txt" if fmt == "gzip" else b"",
                                mtime=99)
        outs = [[] for _ in range(n)]
        for k in range(steps - 1):
            res = st.append([p[k] if k < len(p) else b"" for p in plans])
            for i, (status, out) in enumerate(res):
                assert status == "OK"
                outs[i].append(out)
        res = st.finish([p[-1] if len(p) == steps else b"" for p in plans])
        for i, (status, out) in enumerate(res):
            assert status == "OK"
            outs[i].append(out)
        for i in range(n):
            parts = [plans[i][k] if k < len(plans[i]) else b"" for k in range(steps - 1)]
            parts.append(plans[i][-1] if len(plans[i]) == steps else b"")
            # the oracle's finish() takes no chunk: its last "append" is the chunk given with finish
            exp = O.deflater_parts(parts, level=level, format=fmt, file_name="b.txt" if fmt == "gzip" else None,
                                   mtime=99)
            exp = exp[:-2] + [exp[-2] + exp[-1]]
            assert outs[i] == exp, (level, fmt, i)
            assert b"".join(outs[i]) == O.deflate(srcs[i], level=level, format=fmt,
                                                  file_name="b.txt" if fmt == "gzip" else None, mtime=99)


def test_errors_and_repeated_finish(paradise):
    d = sdz.Deflater()
    with pytest.raises(sdz.SdzError, match="Cannot call finish before at least 1 call to append"):
        d.finish()
    d = sdz.Deflater({"format": "gzip"})
    d.mtime = 5
    first = b"".join(d.append(paradise[:1000])) + b"".join(d.finish())
    assert first == O.deflate(paradise[:1000], format="gzip", mtime=5)
    # finish() again: the compressor has nothing left; the reference appends its trailer again
    assert b"".join(d.finish()) == first[-8:]
    with pytest.raises(sdz.SdzError, match="deflating"):
        d.append(b"more")
    assert d.append(b"") == []


def test_record_path_deflater_hands_over_to_serial(monkeypatch, paradise):
    """Deflater.append runs on the record path (NO_FLUSH re-runs over the input so far) and
    falls back to the serial kernel, replaying the earlier appends into its state, when a block
    is handed back (the pending_buf overlay overtaken) or a call stops at the window-slide
    corner; forced here after each of the first calls.  Per-call bytes equal the reference's
    either way."""
    import test_gpu_parity as P
    rng = random.Random(23)
    src = paradise[:180000]
    parts = split(src, rng.sample(range(1, len(src)), 6))
    for level in (1, 6):
        exp = O.deflater_parts(parts, level=level, format="gzip", file_name="p.txt", mtime=1234567)
        for at in (1, 2, 4):
            monkeypatch.setenv("SDZ_DEFLATER_SWITCH_AT", str(at))
            assert run_deflater(parts, level, "gzip", "p.txt") == exp, (level, at)
        monkeypatch.delenv("SDZ_DEFLATER_SWITCH_AT")
    # overlay-overtaken blocks: the record path hands the call back
    stress = P._overlay_stress(rng, 200000)
    parts = split(stress, [70000, 130000])
    exp = O.deflater_parts(parts, level=6, format="deflate", mtime=1234567)
    assert run_deflater(parts, 6, "deflate") == exp


def test_record_path_deflater_large_appends(paradise):
    """Few large appends (the drop-in's streaming use): per-call bytes as the reference's."""
    big = paradise * 4
    parts = split(big, [300000, 1000000, 1500000])
    for level in (1, 6, 9):
        exp = O.deflater_parts(parts, level=level, format="deflate", mtime=1234567)
        assert run_deflater(parts, level, "deflate") == exp, level


@pytest.mark.timeout(300)
def test_many_small_appends_stay_linear(monkeypatch, paradise):
    """A multi-MB stream appended in 8 KiB chunks: the record-mode Deflater redoes all the
    input so far per call, so past a bound on that redone work (kDeflaterRedo x input + a floor,
    here a 1 MiB floor) it goes serial.  Per-call bytes match the reference, the switch
    included, and the whole run stays within a linear budget."""
    import time
    monkeypatch.setenv("SDZ_DEFLATER_REDO_FLOOR", str(1 << 20))
    data = (paradise * 5)[:2 << 20]
    parts = [data[o:o + 8192] for o in range(0, len(data), 8192)]
    exp = O.deflater_parts(parts, level=6, format="deflate")
    t0 = time.perf_counter()
    got = run_deflater(parts, 6, "deflate")
    dt = time.perf_counter() - t0
    assert got == exp
    assert dt < 120, dt
