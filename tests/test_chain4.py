"""CPU check of the equivalence the 4-byte chain search (k_dfl_link4 / k_dfl_match4)
rests on: longest_match's result (deflate.ts:827-946, from best_len 2) equals the best over the chain
entries that share the first 4 bytes within max_chain ranks, else the first entry whose first 3
bytes agree.  tools/chain4_count.c counts both on the reference's own fixture text and reports any
position where they differ."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def chain4(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("chain4") / "chain4_count")
    subprocess.run(["gcc", "-O2", "-o", exe, os.path.join(ROOT, "tools", "chain4_count.c")], check=True)
    return exe


@pytest.mark.parametrize("max_chain,nice", [(16, 16), (32, 32), (128, 128), (256, 128), (4096, 258)])
def test_4byte_chains_give_longest_match(chain4, max_chain, nice):
    text = os.path.join(ROOT, "tests", "golden", "paradiselost.txt")
    out = subprocess.run([chain4, text, str(max_chain), str(nice)], check=True, capture_output=True,
                         text=True).stdout
    assert "mismatches 0" in out, out
    fields = out.split(",")
    full = float(fields[1].split()[-1])
    four = float(fields[2].split()[-1])
    assert four < full                                   # fewer candidates than the hash-chain walk
