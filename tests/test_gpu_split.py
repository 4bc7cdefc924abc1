"""GPU parity of the block-parallel decode of long streams (k_split.hip): a batch whose
long streams are split at their block starts and decoded as parallel segments must give
exactly what the serial decoder gives -- bytes, records, verdicts -- including for damaged
streams, which fall back to the serial path.  SDZ_SPLIT=0 is the serial reference here.  Both
legs force the lane decoder (SDZ_WDEC=0), so neither depends on the wave decoder's hand-off
constant (kWdLaneAfter); the lane decoder itself is pinned to the oracle by test_gpu_lane.py."""
import os
import random
import zlib

import pytest

import sdz
from conftest import golden

pytestmark = pytest.mark.gpu

FIELDS = ("status", "zmsg", "out_len", "in_used", "stored_checksum", "running_checksum", "stored_size",
          "mtime", "container", "complete", "checksum", "fileSize", "success", "fileName")


def text(rng, n):
    words = golden("paradiselost.txt").split()
    out = bytearray()
    while len(out) < n:
        k = rng.randrange(len(words) - 64)
        out += b" ".join(words[k:k + rng.randint(4, 64)]) + (b".\n" if rng.random() < 0.2 else b" ")
    return bytes(out[:n])


def comp(data, fmt, level=6):
    if fmt == "raw":
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        return c.compress(data) + c.flush()
    if fmt == "gzip":
        c = zlib.compressobj(level, zlib.DEFLATED, 31)
        return c.compress(data) + c.flush()
    return zlib.compress(data, level)


@pytest.fixture(autouse=True)
def _lane_decoder(monkeypatch):
    monkeypatch.setenv("SDZ_WDEC", "0")


def run(streams, caps, split):
    old = os.environ.get("SDZ_SPLIT")
    os.environ["SDZ_SPLIT"] = "1" if split else "0"
    try:
        return sdz.inflate_batch(streams, caps, sdz.FMT_AUTO)
    finally:
        if old is None:
            del os.environ["SDZ_SPLIT"]
        else:
            os.environ["SDZ_SPLIT"] = old


def same(a, b):
    for k in FIELDS:
        assert a[k] == b[k], (k, a[k], b[k])
    assert a["data"] == b["data"]


def test_long_streams_split_like_serial():
    rng = random.Random(5)
    plain, streams = [], []
    for i, (n, fmt, lvl) in enumerate([(3_000_000, "deflate", 6), (2_000_000, "gzip", 9), (1_500_000, "raw", 1),
                                       (700_000, "deflate", 4)]):
        d = text(rng, n)
        if i == 1:                                        # incompressible runs: stored blocks inside
            d = d[:500_000] + bytes(rng.getrandbits(8) for _ in range(70_000)) + d[500_000:]
        plain.append(d)
        streams.append(comp(d, fmt, lvl))
    for k in range(60):                                   # the short streams that set the median
        d = text(rng, rng.randint(2000, 30000))
        plain.append(d)
        streams.append(comp(d, ("raw", "deflate", "gzip")[k % 3]))
    caps = [len(p) + 64 for p in plain]
    par = run(streams, caps, True)
    ser = run(streams, caps, False)
    for i, (a, b) in enumerate(zip(par, ser)):
        same(a, b)
        assert a["data"] == plain[i] and a["success"], i


def test_damaged_long_streams_fall_back_exactly():
    rng = random.Random(9)
    base = [comp(text(rng, 1_200_000), f) for f in ("deflate", "gzip", "raw")]
    streams = []
    for b in base:
        x = bytearray(b)
        x[len(x) // 2] ^= 0x5A                            # a damaged block mid-stream
        streams.append(bytes(x))
        streams.append(b[:len(b) * 2 // 3])               # truncated
        streams.append(b + b"\x00\x01")                   # trailing bytes
        streams.append(b)                                 # intact
    for k in range(40):
        streams.append(comp(text(rng, 5000), "deflate"))
    caps = [4_000_000] * len(streams)
    caps[3] = 100_000                                     # an output slot too small
    par = run(streams, caps, True)
    ser = run(streams, caps, False)
    for a, b in zip(par, ser):
        same(a, b)
