#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 PMC passes (tools/profile_inflate.sh).

One inflate launch = k_inflate_decode + k_inflate_resolve (per round) + k_inflate_finalize; one
deflate launch = the k_dfl_* / k_deflate* kernels + k_checksum.  Per MI355X_MICROARCH.md
(HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE come from separate passes and are in KiB; on gfx950
FETCH_SIZE reports half of the bytes of wide coalesced streaming reads, and other access widths are
uncalibrated.  So each kernel's counts are corrected by the factor measured for its access class
on a known byte count (tools/ubench/fetch_cal.sh -> profiles/rNN_fetch_cal.json): counter bytes /
known bytes for 16-B coalesced streams, per-lane 16-B and 8-B spans, scattered single bytes.  A
kernel with no calibrated class is reported uncorrected (factor 1) and flagged.
Usage: pmc_traffic.py <prof dir> <steps> <out.json> [kernel prefixes, comma-separated] [cal.json]
(default prefixes sdz::k_inflate; the deflate leg: sdz::k_dfl,sdz::k_deflate,sdz::k_checksum)
"""
import collections
import csv
import glob
import json
import os
import sys


PREFIXES = ("sdz::k_inflate",)

# access class of each kernel's dominant HBM reads / writes (the calibration kernel that mimics it)
READ_CLASS = {
    "sdz::k_inflate_decode": "lane16",      # per-lane 16-B refills of its own stream
    "sdz::k_inflate_resolve": "stream16",   # coalesced token rows, coalesced window reloads
    "sdz::k_dfl_chain": "stream16",         # coalesced input rows
    "sdz::k_dfl_match": "stream16",         # window and links staged by coalesced 16-B loads
    "sdz::k_dfl_tail": "scatter1",          # byte loads of the last positions' window walks
    "sdz::k_dfl_parse": "lane8",            # per-lane 8-B records, each lane its own stream
}
WRITE_CLASS = {
    "sdz::k_inflate_decode": "store8",      # per-lane token chunks (64 B per lane and flush)
    "sdz::k_dfl_parse": "store8",           # per-lane symbol words
}


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0]
        if not k.startswith(PREFIXES):
            continue
        tot[k] += float(r["Counter_Value"])
        n[k] += 1
    return tot, n


def load_cal(path):
    if not (path and os.path.exists(path)):
        cands = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles",
                                              "r[0-9][0-9]_fetch_cal.json")))
        path = cands[-1] if cands else None
    if not path:
        return {}, {}
    d = json.load(open(path))
    return d.get("counter_bytes_over_known", {}), d.get("read_GBps", {})


def kernel_ms(root, steps):
    """per-launch ms of each kernel from the kernel-trace pass (<root>/kt), if it is there"""
    path = os.path.join(root, "kt", "run_kernel_stats.csv")
    if not os.path.exists(path):
        return {}
    return {r["Name"].split("(")[0]: float(r["TotalDurationNs"]) / 1e6 / steps for r in csv.DictReader(open(path))}


def main():
    global PREFIXES
    root, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    if len(sys.argv) > 4 and sys.argv[4]:
        PREFIXES = tuple(sys.argv[4].split(","))
    cal, rates = load_cal(sys.argv[5] if len(sys.argv) > 5 else None)
    kms = kernel_ms(root, steps)
    peak = max(rates.values()) if rates else None
    fcal, wcal = cal.get("FETCH_SIZE", {}), cal.get("WRITE_SIZE", {})
    f, nf = per_kernel(os.path.join(root, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    w, nw = per_kernel(os.path.join(root, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    rows = {}
    total = total_raw = 0.0
    for k in sorted(set(f) | set(w)):
        fraw = 1024 * f.get(k, 0.0) / steps
        wraw = 1024 * w.get(k, 0.0) / steps
        rc, wc = READ_CLASS.get(k), WRITE_CLASS.get(k, "stream16")
        rr = fcal.get(rc) if rc else None
        wr = wcal.get(wc) if wc in ("store8",) else 1.0       # 16-B streaming stores read exactly
        fb = fraw / rr if rr else fraw
        wb = wraw / wr if wr else wraw
        rows[k] = {"fetch_bytes": fb, "write_bytes": wb, "fetch_raw_bytes": fraw, "write_raw_bytes": wraw,
                   "read_class": rc if rr else "uncalibrated (raw)", "fetch_counter_over_known": rr,
                   "write_class": wc, "dispatches_per_launch": nf.get(k, 0) / steps}
        if k in kms and kms[k] > 0:
            # the rate the corrected bytes imply over the kernel's time, against the fastest read
            # rate the calibration kernels reach: above it, the correction does not fit the kernel
            rows[k]["kernel_ms"] = kms[k]
            rows[k]["implied_GBps"] = (fb + wb) / (kms[k] * 1e6)
            if peak:
                rows[k]["implied_over_read_peak"] = rows[k]["implied_GBps"] / peak
        total += fb + wb
        total_raw += fraw + wraw
    res = {"hbm_bytes_per_launch": total, "hbm_raw_counter_bytes_per_launch": total_raw, "per_kernel": rows,
           "calibration": cal, "read_GBps": rates,
           "note": "KiB -> bytes; FETCH_SIZE / WRITE_SIZE divided by the counter-over-known-bytes ratio measured "
                   "for each kernel's access class (tools/ubench/fetch_cal.sh); kernels without a class are raw"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
