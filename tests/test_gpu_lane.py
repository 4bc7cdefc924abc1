"""The inflate parity tests of test_gpu_parity.py again, with the LANE decoder forced
(SDZ_WDEC=0).  The default policy (`inflate_wave_policy`) sends most of the suite's
small and mid-size batches to the wave decoder, while every 65,536-stream bench shape (C2, the
distinct leg, the mixed leg) runs on the lane decoder: this file pins that path -- the one behind
the headline numbers -- to the oracle and to ground truth on every inflate case (errors and their
messages, need-bits stalls, dictionaries, stored blocks, trailing bytes, slot edges, many rounds).
Reference: /root/reference/src/infcodes.ts:62-301 (inflate_fast), infblocks.ts:123-628 (proc)."""
import random
import zlib

import pytest

import oracle as O
import sdz
from conftest import golden
from test_gpu_parity import (  # noqa: F401  (collected here a second time, under SDZ_WDEC=0)
    assert_same,
    test_c2_mini_batch_copies_of_paradiselost,
    test_chunkwise_adler_quirk,
    test_concurrent_streams_do_not_share_scratch,
    test_corrupted_streams_match_reference_errors,
    test_dictionary_stream,
    test_fixtures_inflate_like_reference,
    test_inflate_auto_detect_matches_inflate_function,
    test_inflate_oracle_generated,
    test_inflate_zlib_generated,
    test_many_small_blocks,
    test_many_small_blocks_later_rounds,
    test_output_slot_edges,
    test_raw_need_bits_at_end_of_input,
    test_repetitive_data_long_match_chains,
    test_small_rounds_rebuild_the_window,
    test_stored_blocks_decode_correctly,
    test_trailing_bytes_reported,
)

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _lane_decoder(monkeypatch):
    monkeypatch.setenv("SDZ_WDEC", "0")


def _slices(n, size, seed):
    """n distinct `size`-byte windows of paradiselost.txt at random offsets (the distinct leg's
    shape: every lane of a wave decodes a different stream, so lanes diverge every step)."""
    text = golden("paradiselost.txt")
    rng = random.Random(seed)
    return [text[o:o + size] for o in (rng.randrange(len(text) - size) for _ in range(n))]


@pytest.mark.parametrize("fmt", ["deflate", "gzip", "raw"])
def test_distinct_64k_slices_lane_decoder(fmt):
    """256 distinct 64 KiB slices deflated by the oracle (levels 1-9) on the lane decoder: every
    record field and byte against the oracle's Inflater (the north star's stream shape)."""
    plain = _slices(256, 65536, 31 + len(fmt))
    streams = [O.deflate(p, level=1 + i % 9, format=fmt, mtime=i) for i, p in enumerate(plain)]
    raw = fmt == "raw"
    gpu = sdz.inflate_batch(streams, [65536 + 64] * len(streams), sdz.FMT_RAW if raw else sdz.FMT_CONTAINER)
    stalls = 0
    for g, s, p in zip(gpu, streams, plain):
        o = O.inflater_run([s], raw=raw)
        assert_same(g, o, s)
        if raw and not o["complete"]:
            # infcodes.ts:367-387: a raw stream whose last code ends within the table's root bits
            # of the input's end stalls in the reference too (TRUNCATED); its bytes so far agree
            stalls += 1
            assert g["status"] == "TRUNCATED" and p.startswith(g["data"])
            continue
        assert g["status"] == "OK" and g["data"] == p
    assert stalls < len(streams) // 4


def test_distinct_slices_lane_vs_wave_records(monkeypatch):
    """The same distinct batch on both decoders gives identical records and bytes."""
    plain = _slices(192, 40000, 77)
    streams = [O.deflate(p, level=6) for p in plain]
    lane = sdz.inflate_batch(streams, [40064] * len(streams), sdz.FMT_CONTAINER)
    monkeypatch.setenv("SDZ_WDEC", "1")
    wave = sdz.inflate_batch(streams, [40064] * len(streams), sdz.FMT_CONTAINER)
    for a, b, p in zip(lane, wave, plain):
        assert a == b and a["data"] == p


@pytest.mark.parametrize("lane_after", [3, 7])
def test_wave_decoder_restart_odd_lane_after(monkeypatch, lane_after):
    """Streams of many small blocks make the wave decoder start round 0 over on the lane decoder
    after SDZ_WD_LANE_AFTER launch pairs; with an odd count (pairs are queued two at a time) the
    restart still happens before any pair runs with the lane flag, and the records and bytes equal
    the lane decoder's (k_inflate.hip run_inflate_rounds)."""
    paradise = golden("paradiselost.txt")
    streams, plain = [], []
    for k, wbits in enumerate((15, -15, 31, 15)):
        data = paradise[k * 9000:k * 9000 + 60000]
        c = zlib.compressobj(6, zlib.DEFLATED, wbits)
        comp = b"".join(c.compress(data[i:i + 300]) + c.flush(zlib.Z_SYNC_FLUSH) for i in range(0, len(data), 300))
        streams.append(comp + c.flush())
        plain.append(data)
    streams.append(zlib.compress(paradise[:20000], 6))            # one ordinary stream beside them
    plain.append(paradise[:20000])
    caps = [len(p) + 64 for p in plain]
    lane = sdz.inflate_batch(streams, caps, sdz.FMT_AUTO)
    monkeypatch.setenv("SDZ_WDEC", "1")
    monkeypatch.setenv("SDZ_WD_LANE_AFTER", str(lane_after))
    wave = sdz.inflate_batch(streams, caps, sdz.FMT_AUTO)
    for a, b, p in zip(lane, wave, plain):
        assert a["status"] == "OK" and a["data"] == p
        assert a == b


def test_unchecked_runs_meet_stream_ends():
    """The symbol loop's 4-step runs without bit and room checks hand over
    to the checked loop once some lane of the wave is within 64 + 3 x 48 bits of its input's end or
    4 x 258 bytes of its output slot's end.  One wave of lanes whose ends fall at every distance
    from those bounds -- output slots from exact to 2,100 bytes short, inputs cut 0 to 40 bytes
    early -- beside lanes far from theirs: records and bytes against the oracle's Inflater (cut
    inputs) and the slot-edge rule (short slots)."""
    text = golden("paradiselost.txt")
    rng = random.Random(5)
    plain = [text[o:o + 30000] for o in (rng.randrange(len(text) - 30000) for _ in range(8))]
    comp = [zlib.compress(p, 6) for p in plain]
    streams, caps, kinds = [], [], []
    for i in range(64):                                   # short output slots
        p, c = plain[i % 8], comp[i % 8]
        k = (i * 33) % 2101
        streams.append(c); caps.append(len(p) - k); kinds.append(("slot", i % 8, k))
    for i in range(41):                                   # cut inputs
        c = comp[i % 8]
        streams.append(c[:len(c) - i]); caps.append(len(plain[i % 8]) + 64); kinds.append(("cut", i % 8, i))
    for i in range(23):                                   # lanes far from their ends
        streams.append(comp[i % 8]); caps.append(len(plain[i % 8]) + 64); kinds.append(("whole", i % 8, 0))
    gpu = sdz.inflate_batch(streams, caps, sdz.FMT_CONTAINER)
    for g, s, cap, (kind, j, k) in zip(gpu, streams, caps, kinds):
        p = plain[j]
        if kind == "slot" and k:
            assert g["status"] == "OUT_OVERFLOW" and not g["success"], (k, g["status"])
            n = g["out_len"]
            assert cap - 258 < n <= cap and g["data"][:n] == p[:n]
        elif kind == "cut" and k:
            assert_same(g, O.inflater_run([s]), s)
        else:
            assert g["success"] and g["data"] == p
