"""CPU-side checks of the drop-in boundary: libsdz.so loads and exports exactly
the C ABI that include/sdz.h declares (no compute calls: no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "sdz.h")
LIB = os.path.join(ROOT, "sd-zlib_amd", "lib", "libsdz.so")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sdz_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "sd-zlib_amd")], check=True)
    return LIB


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ["sdz_inflate_batch_device", "sdz_deflate_batch_device", "sdz_adler32", "sdz_crc32",
                 "sdz_inflate_batch", "sdz_deflate_batch"]:
        assert must in names


def test_library_exports_every_declared_symbol(built):
    out = subprocess.run(["nm", "-D", "--defined-only", built], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (sdz_[a-z0-9_]+)", out))
    missing = set(declared_functions()) - exported
    assert not missing, missing
    extra = exported - set(declared_functions())
    assert not extra, extra


def test_library_loads_and_python_binding_matches(built):
    import sdz
    L = sdz.lib()
    assert L.sdz_version() == 4
    assert sorted(sdz.EXPORTS) == declared_functions()
    for name in sdz.EXPORTS:
        assert hasattr(L, name)
    assert sdz.zmsg(18) == "invalid literal/length code"
    assert sdz.zmsg(17) == "invalid distance code"
    assert L.sdz_deflate_bound(65536, 1, 0) >= 65536 + 6


def test_record_layouts():
    import sdz
    assert ctypes.sizeof(sdz.InflateRecord) == 64
    assert ctypes.sizeof(sdz.DeflateRecord) == 24


def test_no_cpu_fallback_without_device(built):
    """With no GPU the product path must fail loudly, never compute on the CPU."""
    import sdz
    if sdz.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(sdz.SdzError):
        sdz.inflate_batch([b"\x78\x01\x03\x00\x00\x00\x00\x01"])
    with pytest.raises(sdz.SdzError):
        sdz.deflate_batch([b"abc"])
    # checksums report the failure instead of returning a wrong value (0)
    with pytest.raises(sdz.SdzError):
        sdz.adler32(b"abc")
    with pytest.raises(sdz.SdzError):
        sdz.crc32(b"abc")
    r = ctypes.c_int32(7)
    assert sdz.lib().sdz_adler32_checked(b"abc", 3, 1, ctypes.byref(r)) == -2   # SDZ_API_NO_DEVICE
    assert r.value == 7


def test_gpu_sources_are_gfx950_only():
    """No compatibility layers: HIP sources for gfx950, no CUDA shims / dual paths."""
    csrc = os.path.join(ROOT, "sd-zlib_amd", "csrc")
    for f in os.listdir(csrc):
        text = open(os.path.join(csrc, f)).read()
        assert "__HIP_PLATFORM_NVIDIA__" not in text and "cuda_runtime" not in text
    mk = open(os.path.join(ROOT, "sd-zlib_amd", "Makefile")).read()
    assert "gfx950" in mk
