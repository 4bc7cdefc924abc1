"""GPU parity of the preset-dictionary path: Deflater({dictionary})
= deflateSetDictionary (deflate.ts:1184-1216) + the 78 20 + DICTID zlib header
(sd-deflate.ts:80-115), bit-exact against the oracle; and the reference's own
testRoundTripDictionary (test/index.html:173-208) with its dictionary fixture."""
import pytest

import oracle as O
import sdz
from conftest import golden

pytestmark = pytest.mark.gpu


def test_reference_round_trip_dictionary(paradise):
    terms = golden("dict_terms.txt")
    comp = sdz.deflate(paradise, {"format": "deflate", "dictionary": terms})
    assert comp[:2] == b"\x78\x20" and int.from_bytes(comp[2:6], "big") == O.adler32(terms) & 0xFFFFFFFF
    assert comp == O.deflate(paradise, level=6, dictionary=terms)
    inf = sdz.Inflater({"dictionary": terms})
    out = b"".join(inf.append(comp))
    res = inf.finish()
    assert out == paradise and res["success"] and res["checksum"] == "match"


@pytest.mark.parametrize("level", range(1, 10))
def test_dictionary_levels_and_lengths_bitexact(level, paradise):
    """Dictionary lengths below MIN_MATCH (header only), short, 5552 (the adler32 NMAX
    quirk of the DICTID), exactly MAX_DIST, and longer (only its tail is used)."""
    src = paradise[100000:100000 + 20000 + 997 * level]
    for dl in (1, 2, 3, 300, 5552, 32506, 40000):
        d = paradise[7:7 + dl] if dl != 5552 else paradise[-5552:]
        got = sdz.deflate_batch([src], level=level, format="deflate", dictionary=d)[0]
        assert got["status"] == "OK"
        assert got["data"] == O.deflate(src, level=level, dictionary=d), (level, dl)
        back = sdz.inflate_one(got["data"], sdz.FMT_CONTAINER, d)
        assert back["data"] == src and back["success"]


def test_dictionary_batch_and_errors(paradise):
    terms = golden("dict_terms.txt")
    srcs = [paradise[i * 3001:i * 3001 + 5000 + 37 * i] for i in range(40)]
    got = sdz.deflate_batch(srcs, level=9, format="deflate", dictionary=terms)
    for s, g in zip(srcs, got):
        assert g["data"] == O.deflate(s, level=9, dictionary=terms)
    with pytest.raises(TypeError, match="Can only provide a dictionary"):
        sdz.Deflater({"format": "gzip", "dictionary": terms})
    with pytest.raises(sdz.SdzError, match="Can only provide a dictionary"):
        sdz.deflate_batch(srcs[:1], level=6, format="raw", dictionary=terms)


def test_deflater_checksum_chains_per_append(paradise):
    """sd-deflate.ts:185-190: Deflater.append() folds each chunk into the running checksum, so
    an append of 5552 or 11104 bytes (adler32's NMAX quirk) changes the trailer; the merged
    output must match the reference's for the same appends."""
    for sizes in ([5552, 5552, 100], [11104, 7], [3000, 16384, 5552], [70000, 11104, 9]):
        parts, o = [], 0
        for z in sizes:
            parts.append(paradise[o:o + z])
            o += z
        for fmt in ("deflate", "gzip", "raw"):
            d = sdz.Deflater({"format": fmt, "level": 6})
            d.mtime = 0
            out = b"".join(b"".join(d.append(p)) for p in parts) + b"".join(d.finish())
            assert out == O.deflater_run(parts, level=6, format=fmt, mtime=0), (sizes, fmt)
