"""The CPU restatement under sanitizers (SURVEY.md §5 "Race detection / sanitizers").

oracle/sanitize_main.c drives oracle/sdz_oracle.c through the reference's fixtures, all
levels and containers, window-slide edge sizes, stored (incompressible) inputs,
dictionaries, split appends and corrupted / truncated streams, built with
-fsanitize=address,undefined; a second build runs inflate + deflate from 8 threads at
once under ThreadSanitizer, the way bench.py's cpu_baseline calls the oracle (the lazily
built code tables raced there before they moved to pthread_once).  CPU only.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")

pytestmark = pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")


def _build(target):
    subprocess.run(["make", "-s", "-C", ORACLE, target], check=True)
    return os.path.join(ORACLE, "_build", "oracle_" + target)


@pytest.mark.timeout(300)
def test_oracle_asan_ubsan():
    exe = _build("asan")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, GOLDEN], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "0 failures" in r.stdout


@pytest.mark.timeout(300)
def test_oracle_tsan_threads():
    exe = _build("tsan")
    r = subprocess.run([exe, GOLDEN, "8"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
