"""The inflate parity tests of test_gpu_parity.py again, with the batch-pipeline resolve kernel
forced (SDZ_RESOLVE=1, k_inflate_resolve_b): the same oracle and ground truth on
every inflate case -- errors, need-bits stalls, dictionaries, stored blocks, trailing bytes, slot
edges, many small blocks, many rounds (the ring rebuilt from the output), long-match chains (cut
batches, self-overlapping copies) -- plus the incremental Inflater's per-append output.
Reference: /root/reference/src/infcodes.ts:161-207 (the window copy), infblocks.ts:61-121."""
import pytest

from test_gpu_parity import (  # noqa: F401  (collected here a second time, under SDZ_RESOLVE=1)
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
from test_gpu_lane import test_distinct_64k_slices_lane_decoder  # noqa: F401
from test_gpu_stream import (  # noqa: F401
    test_batched_streams_with_small_output_slots,
    test_chunkwise_adler_quirk_across_appends,
    test_random_splits_match_oracle,
    test_small_pieces_cross_every_unit,
)

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _batch_resolve(monkeypatch):
    monkeypatch.setenv("SDZ_RESOLVE", "1")
