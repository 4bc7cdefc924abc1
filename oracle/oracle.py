"""ctypes binding for the CPU restatement in oracle/sdz_oracle.c.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- as the checker, never as the product path.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")

FORMAT = {"raw": 0, "deflate": 1, "gzip": 2}

ERRORS = {
    0: None,
    1: "inflate error: ",
    2: "inflate error: bad input data",
    3: "Custom dictionary is not valid for this data",
    4: "Custom dictionary required for this data",
    5: "Unexpected EOF during decompression",
    6: "Data integrity check failed",
    7: "Data size check failed",
    8: "Decompression error",
    9: "data buffer is too small",
    10: "HANG",
    11: "OUT_CAP",
    12: "Cannot call finish before at least 1 call to append",
    13: "PENDING_OVERFLOW",
    14: "BAD_ARG",
}


class InflateResult(ctypes.Structure):
    _fields_ = [
        ("error", ctypes.c_int32), ("zmsg", ctypes.c_int32), ("success", ctypes.c_int32),
        ("complete", ctypes.c_int32), ("checksum_verdict", ctypes.c_int32),
        ("size_verdict", ctypes.c_int32), ("stored_checksum", ctypes.c_int32),
        ("running_checksum", ctypes.c_int32), ("stored_size", ctypes.c_int32),
        ("container", ctypes.c_int32), ("mtime", ctypes.c_int32), ("name_len", ctypes.c_int32),
        ("total_out", ctypes.c_uint64), ("name", ctypes.c_char * 256),
    ]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.c_char_p
        L.oracle_adler32.restype = ctypes.c_int32
        L.oracle_adler32.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int32]
        L.oracle_crc32.restype = ctypes.c_int32
        L.oracle_crc32.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int32]
        L.oracle_zmsg.restype = ctypes.c_char_p
        L.oracle_inflater_run.restype = ctypes.c_int32
        L.oracle_inflater_run.argtypes = [
            ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_int32,
            ctypes.c_int32, u8p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
            ctypes.POINTER(InflateResult)]
        L.oracle_inflater_run_parts.restype = ctypes.c_int32
        L.oracle_inflater_run_parts.argtypes = L.oracle_inflater_run.argtypes + [
            ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int32)]
        L.oracle_inflater_run_chunks.restype = ctypes.c_int32
        L.oracle_inflater_run_chunks.argtypes = L.oracle_inflater_run_parts.argtypes + [
            ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int32), ctypes.c_size_t,
            ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_inflate.restype = ctypes.c_int32
        L.oracle_inflate.argtypes = [u8p, ctypes.c_size_t, u8p, ctypes.c_size_t, ctypes.c_void_p,
                                     ctypes.c_size_t, ctypes.POINTER(InflateResult)]
        L.oracle_deflater_run.restype = ctypes.c_int32
        L.oracle_deflater_run.argtypes = [
            ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_int32,
            ctypes.c_int32, ctypes.c_int32, u8p, ctypes.c_size_t, ctypes.c_int32, u8p,
            ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t,
            ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_deflater_run_parts.restype = ctypes.c_int32
        L.oracle_deflater_run_parts.argtypes = L.oracle_deflater_run.argtypes + [ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_fixed_table_entry.restype = ctypes.c_int32
        L.oracle_fixed_table_entry.argtypes = [ctypes.c_int, ctypes.c_int]
        L.oracle_tree_table.restype = ctypes.c_int32
        L.oracle_tree_table.argtypes = [ctypes.c_int, ctypes.c_int]
        _lib = L
    return _lib


def adler32(data: bytes, seed: int = 1) -> int:
    return lib().oracle_adler32(bytes(data), len(data), ctypes.c_int32(seed).value)


def crc32(data: bytes, seed: int = 0) -> int:
    return lib().oracle_crc32(bytes(data), len(data), ctypes.c_int32(seed).value)


def zmsg(idx: int) -> str:
    return lib().oracle_zmsg(idx).decode()


def _result_dict(res: InflateResult, out: bytes):
    err = res.error
    msg = ERRORS.get(err)
    if err == 1:
        msg = "inflate error: " + zmsg(res.zmsg)
    return {
        "error": err, "message": msg, "zmsg": res.zmsg, "success": bool(res.success),
        "complete": bool(res.complete),
        "checksum": ["unchecked", "match", "mismatch"][res.checksum_verdict],
        "fileSize": ["unchecked", "match", "mismatch"][res.size_verdict],
        "stored_checksum": res.stored_checksum, "running_checksum": res.running_checksum,
        "stored_size": res.stored_size, "container": res.container, "mtime": res.mtime,
        "fileName": res.name[:res.name_len].decode("latin-1"), "data": out,
    }


def inflater_run(parts, raw=False, dictionary=None, out_cap=None):
    parts = [bytes(p) for p in parts]
    n = len(parts)
    arr = (ctypes.c_char_p * n)(*parts)
    lens = (ctypes.c_size_t * n)(*[len(p) for p in parts])
    total_in = sum(len(p) for p in parts)
    cap = out_cap if out_cap is not None else max(1 << 16, total_in * 1100 + 65536)
    out = ctypes.create_string_buffer(cap)
    res = InflateResult()
    d = bytes(dictionary) if dictionary is not None else None
    lib().oracle_inflater_run(arr, lens, n, 1 if raw else 0, d, len(d) if d else 0, out, cap,
                              ctypes.byref(res))
    return _result_dict(res, out.raw[:res.total_out])


def inflater_chunks(parts, raw=False, dictionary=None, out_cap=None):
    """The arrays each append() returns, as the reference builds them (sd-inflate.ts:101-150):
    a list per append of the pushed Uint8Array lengths.  Also returns the result dict."""
    parts = [bytes(p) for p in parts]
    n = len(parts)
    arr = (ctypes.c_char_p * n)(*parts)
    lens = (ctypes.c_size_t * n)(*[len(p) for p in parts])
    total_in = sum(len(p) for p in parts)
    cap = out_cap if out_cap is not None else max(1 << 16, total_in * 1100 + 65536)
    out = ctypes.create_string_buffer(cap)
    res = InflateResult()
    pout = (ctypes.c_size_t * max(1, n))()
    ep = ctypes.c_int32(-1)
    ccap = cap // 16384 + 4 * n + 16
    clen = (ctypes.c_size_t * ccap)()
    cpart = (ctypes.c_int32 * ccap)()
    nch = ctypes.c_size_t(0)
    d = bytes(dictionary) if dictionary is not None else None
    lib().oracle_inflater_run_chunks(arr, lens, n, 1 if raw else 0, d, len(d) if d else 0, out, cap,
                                     ctypes.byref(res), pout, ctypes.byref(ep), clen, cpart, ccap, ctypes.byref(nch))
    per = [[] for _ in range(n)]
    for k in range(min(nch.value, ccap)):
        per[cpart[k]].append(clen[k])
    return per, _result_dict(res, out.raw[:res.total_out])


def inflater_parts(parts, raw=False, dictionary=None, out_cap=None):
    """inflater_run, plus the output of each append() (list of bytes) and the index of the
    append that threw (or None)."""
    parts = [bytes(p) for p in parts]
    n = len(parts)
    arr = (ctypes.c_char_p * n)(*parts)
    lens = (ctypes.c_size_t * n)(*[len(p) for p in parts])
    total_in = sum(len(p) for p in parts)
    cap = out_cap if out_cap is not None else max(1 << 16, total_in * 1100 + 65536)
    out = ctypes.create_string_buffer(cap)
    res = InflateResult()
    pout = (ctypes.c_size_t * max(1, n))()
    ep = ctypes.c_int32(-1)
    d = bytes(dictionary) if dictionary is not None else None
    lib().oracle_inflater_run_parts(arr, lens, n, 1 if raw else 0, d, len(d) if d else 0, out, cap,
                                    ctypes.byref(res), pout, ctypes.byref(ep))
    r = _result_dict(res, out.raw[:res.total_out])
    pieces, o = [], 0
    for k in range(n):
        pieces.append(r["data"][o:o + pout[k]])
        o += pout[k]
    r["parts_out"] = pieces
    r["error_part"] = None if ep.value < 0 else ep.value
    return r


def inflate(data, dictionary=None, out_cap=None):
    data = bytes(data)
    cap = out_cap if out_cap is not None else max(1 << 16, len(data) * 1100 + 65536)
    out = ctypes.create_string_buffer(cap)
    res = InflateResult()
    d = bytes(dictionary) if dictionary is not None else None
    lib().oracle_inflate(data, len(data), d, len(d) if d else 0, out, cap, ctypes.byref(res))
    return _result_dict(res, out.raw[:res.total_out])


def latin1_filename(name: str) -> bytes:
    """sd-deflate.ts:125-130: Array.from(name) code points, > 0xFF -> '_'."""
    return bytes((ord(ch) if ord(ch) <= 0xFF else 95) for ch in name)


def deflater_run(parts, level=6, format="deflate", dictionary=None, file_name=None, mtime=0):
    parts = [bytes(p) for p in parts]
    n = len(parts)
    arr = (ctypes.c_char_p * n)(*parts)
    lens = (ctypes.c_size_t * n)(*[len(p) for p in parts])
    total = sum(len(p) for p in parts)
    fn = latin1_filename(file_name) if file_name else b""
    cap = total + total // 8 + 4096 + len(fn)
    out = ctypes.create_string_buffer(cap)
    out_len = ctypes.c_size_t(0)
    d = bytes(dictionary) if dictionary is not None else None
    err = lib().oracle_deflater_run(arr, lens, n, level, FORMAT[format], d, len(d) if d else 0,
                                    1 if d is not None else 0, fn, len(fn), mtime & 0xFFFFFFFF,
                                    out, cap, ctypes.byref(out_len))
    if err:
        raise RuntimeError("oracle deflate error %d: %s" % (err, ERRORS.get(err)))
    return out.raw[:out_len.value]


def deflater_parts(parts, level=6, format="deflate", dictionary=None, file_name=None, mtime=0):
    """The reference Deflater's per-call outputs: [append(p) for p in parts] + [finish()],
    each the concatenation of the Uint8Arrays that call returns (sd-deflate.ts:173-253)."""
    parts = [bytes(p) for p in parts]
    n = len(parts)
    arr = (ctypes.c_char_p * n)(*parts)
    lens = (ctypes.c_size_t * n)(*[len(p) for p in parts])
    total = sum(len(p) for p in parts)
    fn = latin1_filename(file_name) if file_name else b""
    cap = total + total // 8 + 4096 + len(fn)
    out = ctypes.create_string_buffer(cap)
    out_len = ctypes.c_size_t(0)
    ends = (ctypes.c_size_t * (n + 1))()
    d = bytes(dictionary) if dictionary is not None else None
    err = lib().oracle_deflater_run_parts(arr, lens, n, level, FORMAT[format], d, len(d) if d else 0,
                                          1 if d is not None else 0, fn, len(fn), mtime & 0xFFFFFFFF,
                                          out, cap, ctypes.byref(out_len), ends)
    if err:
        raise RuntimeError("oracle deflate error %d: %s" % (err, ERRORS.get(err)))
    raw, res, prev = out.raw, [], 0
    for k in range(n + 1):
        res.append(raw[prev:ends[k]])
        prev = ends[k]
    return res


def deflate(data, level=6, format="deflate", dictionary=None, file_name=None, mtime=0):
    return deflater_run([data], level, format, dictionary, file_name, mtime)
