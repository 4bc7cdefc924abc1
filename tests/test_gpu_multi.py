"""Multi-GPU inside libsdz (SURVEY.md §8e, §4 "fake multi-GPU mode"), on the one GPU of the
test box: N logical shards of a C4-shaped mini batch (mixed sizes, raw / zlib / gzip), each
shard run by the real engine, records gathered -- over RCCL when the devices are distinct
(here: one device, a one-rank ncclAllGather), by the loopback gather when a device repeats.
Every record and payload is checked against ground truth and the oracle.  Also: the
per-rank RCCL communicator (one process per GPU), the batched span copy and the host-path
staging pools (repeated small calls, a skewed incremental batch)."""
import ctypes
import random
import zlib

import pytest

import oracle as O
import sdz
from conftest import golden

pytestmark = pytest.mark.gpu


def _mixed_batch(n, seed=7):
    """C4 shape at test size: log-uniform 1 KiB .. 1 MiB, formats cycling raw/zlib/gzip,
    compressible text (compressed by Python's zlib, an independent encoder)."""
    from run_configs import text, compress
    rng = random.Random(seed)
    plain, comp = [], []
    for i in range(n):
        size = int(2 ** rng.uniform(10, 20))
        data = text(rng, size)
        plain.append(data)
        comp.append(compress(data, i % 3))
    return plain, comp


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0]])
def test_inflate_batch_multi_shards(devices):
    plain, comp = _mixed_batch(48)
    recs, st = sdz.inflate_batch_multi(comp, devices, out_caps=[len(p) + 64 for p in plain])
    assert st["rccl"] == (len(set(devices)) == len(devices))
    assert sum(st["streams"]) == len(comp) and len(st["streams"]) == len(devices)
    assert sum(st["bytes_out"]) == sum(len(p) for p in plain)
    assert st["wall_ms"] >= st["compute_ms"] > 0
    # LPT balance: no shard exceeds the mean by more than the largest stream
    loads = st["bytes_in"]
    assert max(loads) - min(loads) <= max(len(c) for c in comp)
    for i, (r, p, c) in enumerate(zip(recs, plain, comp)):
        assert r["status"] == "OK" and r["success"] and r["data"] == p, i
        ref = O.inflate(c)                                # inflate(): the same auto-detect
        assert ref["data"] == p
        assert r["running_checksum"] == ref["running_checksum"] and r["checksum"] == ref["checksum"], i


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_deflate_batch_multi_bit_exact(devices):
    text = golden("paradiselost.txt")
    rng = random.Random(3)
    srcs = [text[o:o + n] for o, n in ((rng.randrange(300000), rng.choice([1000, 20000, 65536, 150000]))
                                       for _ in range(24))]
    outs, st = sdz.deflate_batch_multi(srcs, devices, level=6, format="gzip", mtime=0)
    assert sum(st["streams"]) == len(srcs)
    for i, (o, s) in enumerate(zip(outs, srcs)):
        assert o["status"] == "OK"
        assert o["data"] == O.deflate(s, level=6, format="gzip", mtime=0), i
        assert zlib.decompress(o["data"], 31) == s


def test_multi_matches_single_device_records():
    plain, comp = _mixed_batch(30, seed=11)
    caps = [len(p) + 64 for p in plain]
    one = sdz.inflate_batch(comp, caps)
    multi, _ = sdz.inflate_batch_multi(comp, [0, 0], out_caps=caps)
    for a, b in zip(one, multi):
        assert a == b


def test_multi_bad_devices():
    with pytest.raises(sdz.SdzError):
        sdz.inflate_batch_multi([b"x"], [99])
    with pytest.raises(sdz.SdzError):
        sdz.inflate_batch_multi([b"x"], [0] * 17)


def test_comm_one_rank():
    uid = sdz.Comm.unique_id()
    c = sdz.Comm(uid, 1, 0)
    try:
        assert c.allgather_bytes(b"records!") == [b"records!"]
        assert c.max(3.25) == 3.25
    finally:
        c.close()


def test_gather_device_spans():
    L = sdz.lib()
    rng = random.Random(5)
    src = bytes(rng.getrandbits(8) for _ in range(300000))
    spans = [(rng.randrange(250000), rng.randrange(0, 40000)) for _ in range(200)]
    spans.append((0, 0))
    spans.append((len(src) - 7, 7))
    dst_off, o = [], 0
    for so, n in spans:
        dst_off.append(o + rng.randrange(4))              # unaligned destinations too
        o = dst_off[-1] + n + 16
    d_src, d_dst = sdz.DeviceBuffer(len(src)), sdz.DeviceBuffer(o + 64)
    d_src.upload(src)
    meta = dst_off + [s for s, _ in spans] + [n for _, n in spans]
    d_meta = sdz.DeviceBuffer(8 * len(meta))
    d_meta.upload(bytes((ctypes.c_uint64 * len(meta))(*meta)))
    k = len(spans)
    assert L.sdz_gather_device(d_dst.ptr, d_meta.ptr, d_src.ptr, d_meta.ptr + 8 * k, d_meta.ptr + 16 * k, k, None) == 0
    assert L.sdz_sync(None) == 0
    got = d_dst.download(o)
    for (so, n), do in zip(spans, dst_off):
        assert got[do:do + n] == src[so:so + n]


def test_host_path_repeated_small_calls():
    """the drop-in's one-stream calls reuse the staging pools (no per-call allocation)"""
    simple = golden("simple.deflate")
    for _ in range(50):
        r = sdz.inflate_batch([simple], [64])[0]
        assert r["success"] and r["data"] == golden("simple.txt")
    for _ in range(20):
        d = sdz.deflate_batch([golden("simple.txt")], level=6)[0]
        assert d["data"] == simple
    # growth: a large call after small ones, then small again
    big = golden("paradiselost.deflate")
    assert sdz.inflate_batch([big] * 40, [471162] * 40)[39]["data"] == golden("paradiselost.txt")
    assert sdz.inflate_batch([simple], [64])[0]["data"] == golden("simple.txt")


def test_incremental_skewed_batch():
    """one long chunk beside many tiny ones -- staging slots are per stream
    (prefix sums of carry + chunk), not n x (carry + the longest chunk)"""
    text = golden("paradiselost.txt")
    big = zlib.compress(text * 8, 6)                      # ~1.5 MB compressed
    small = zlib.compress(b"hello world " * 10, 6)
    n = 2048
    st = sdz.InflateStreams(n)
    chunks = [big] + [small] * (n - 1)
    res = st.append(chunks, out_cap=[len(text) * 8 + 64] + [256] * (n - 1))
    assert res[0]["success"] and res[0]["data"] == text * 8
    assert all(r["success"] and r["data"] == b"hello world " * 10 for r in res[1:])


def _concurrent_multi(devices):
    import threading
    plain, comp = _mixed_batch(24, seed=5)
    caps = [len(p) + 64 for p in plain]
    res, errs = [None, None], []

    def run(k):
        try:
            res[k], _ = sdz.inflate_batch_multi(comp, devices, out_caps=caps)
        except Exception as e:                            # reported below, not swallowed
            errs.append(e)

    ts = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not any(t.is_alive() for t in ts), "multi calls deadlocked"
    assert not errs, errs
    for recs in res:
        for r, p in zip(recs, plain):
            assert r["status"] == "OK" and r["data"] == p


@pytest.mark.skipif(sdz.device_count() < 2, reason="needs two GPUs (distinct devices: the RCCL path)")
def test_concurrent_multi_calls_distinct_devices():
    """As below, on two distinct devices: each call's shards hold their device locks across the
    RCCL all-gather, the case the serialised multi calls (g_multi_mu) exist for."""
    _concurrent_multi([0, 1])


@pytest.mark.parametrize("devices", [[0], [0, 1]])
def test_gather_failure_aborts_and_recovers(monkeypatch, devices):
    """A rank whose collective fails (SDZ_TEST_GATHER_FAIL=k: rank k never enters the all-gather) ends
    the call with an error on every rank -- its peers stop waiting instead of hanging -- the
    communicators are aborted and dropped, and the next call builds new ones and succeeds."""
    if max(devices) >= sdz.device_count():
        pytest.skip("needs %d GPUs" % (max(devices) + 1))
    plain, comp = _mixed_batch(12, seed=11)
    caps = [len(p) + 64 for p in plain]
    monkeypatch.setenv("SDZ_TEST_GATHER_FAIL", str(len(devices) - 1))
    with pytest.raises(sdz.SdzError, match="ncclAllGather|collective failed"):
        sdz.inflate_batch_multi(comp, devices, out_caps=caps)
    monkeypatch.delenv("SDZ_TEST_GATHER_FAIL")
    recs, st = sdz.inflate_batch_multi(comp, devices, out_caps=caps)
    assert st["rccl"]
    assert all(r["status"] == "OK" and r["data"] == p for r, p in zip(recs, plain))


def test_concurrent_multi_calls_same_devices():
    """Two host threads call inflate_batch_multi on the same device list at once (ctypes drops the
    GIL): the library serialises multi calls, so neither waits on the other's shard at a barrier
    (overlapping device locks held across the all-gather deadlocked), and both
    return every record intact."""
    _concurrent_multi([0, 0])
