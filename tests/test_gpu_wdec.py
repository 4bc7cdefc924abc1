"""The inflate parity tests of test_gpu_parity.py again, with the wave decoder forced
(SDZ_WDEC=1).  By default it serves batches whose total is at most 24,576 times
their longest stream, of 16 KiB - 4 MiB of compressed input, so most of the suite's small batches
would not reach it: here every one-shot batch does -- errors and their messages, need-bits stalls at the end of the
input, dictionaries, stored blocks, trailing bytes, output slots at the edge, many rounds -- against
the same oracle and ground truth."""
import pytest

from test_gpu_parity import (  # noqa: F401  (collected here a second time, under SDZ_WDEC=1)
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
def _wave_decoder(monkeypatch):
    monkeypatch.setenv("SDZ_WDEC", "1")
