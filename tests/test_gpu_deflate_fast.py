"""The opt-in fast compressor (sdz_deflate_fast_batch_device): not the
reference's bytes, so the bar is validity -- every stream inflates back to its input with
this engine (checksum "match") and with Python's zlib (an independent inflater), the
trailer carries the reference's adler32 / crc32 of the input (oracle), and text compresses.
Edge cases: tile boundaries (16 KiB), incompressible input (stored tiles), runs (258-byte
matches), one byte, empty input (the reference throws: DATA_ERROR)."""
import random
import zlib

import pytest

import oracle as O
import sdz

pytestmark = pytest.mark.gpu


def inflate_py(data, fmt):
    wbits = {"raw": -15, "deflate": 15, "gzip": 31}[fmt]
    return zlib.decompress(data, wbits)


def test_round_trips(paradise):
    rng = random.Random(5)
    srcs = [paradise, paradise[:1], paradise[:16383], paradise[:16384], paradise[:16385], paradise[:32769],
            bytes(rng.getrandbits(8) for _ in range(40000)),          # incompressible: stored tiles
            b"a" * 70000, (b"abc" * 9000)[:20001], bytes(range(256)) * 300,
            paradise[1000:1000 + rng.randint(1, 200000)]]
    for fmt in ("deflate", "gzip", "raw"):
        res = sdz.deflate_fast_batch(srcs, format=fmt, file_name_latin1=b"f.txt" if fmt == "gzip" else b"",
                                     mtime=42)
        for src, r in zip(srcs, res):
            assert r["status"] == "OK"
            assert inflate_py(r["data"], fmt) == src, (fmt, len(src))
            if fmt != "raw":
                assert sdz.inflate(r["data"]) == src
            want = O.crc32(src) if fmt == "gzip" else O.adler32(src)
            assert r["checksum"] == want
    text = sdz.deflate_fast_batch([paradise])[0]["data"]
    assert len(text) < 0.55 * len(paradise), len(text)   # L6 of the reference: 0.41


def test_batch_of_slices_and_errors(paradise):
    rng = random.Random(9)
    srcs = []
    for _ in range(300):
        a = rng.randrange(0, len(paradise) - 70000)
        srcs.append(paradise[a:a + rng.randint(1, 70000)])
    srcs.insert(17, b"")
    res = sdz.deflate_fast_batch(srcs)
    for src, r in zip(srcs, res):
        if not src:
            assert r["status"] == "DATA_ERROR"
            continue
        assert r["status"] == "OK" and zlib.decompress(r["data"]) == src
