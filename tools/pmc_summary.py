"""Summarise rocprofv3 runs into profiles/: per-kernel time (kernel trace) and
HBM traffic (FETCH_SIZE / WRITE_SIZE passes), calibrated on tools/ubench_stream.

    python tools/pmc_summary.py <prof_dir> <config> <out_prefix>

<prof_dir> holds the csv outputs of
  trace/  : --kernel-trace --stats           (bench.py)
  fetch/  : --pmc FETCH_SIZE                 (bench.py)
  write/  : --pmc WRITE_SIZE                 (bench.py)
  cfetch/, cwrite/ : the same two passes over tools/ubench_stream (calibration)
"""
from __future__ import annotations

import csv
import glob
import json
import os
import statistics
import sys

KERNELS = ("k_ell_iter", "k_cg_iter")  # lane kernel, SELL kernel (whichever ran)


def rows(d, pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def counter_by_kernel(d, counter):
    """average counter value per dispatch, by kernel name substring."""
    vals = {}
    for r in rows(d, "*counter_collection.csv"):
        if r.get("Counter_Name") != counter:
            continue
        name = r["Kernel_Name"]
        vals.setdefault(name, []).append(float(r["Counter_Value"]))
    return {k: statistics.mean(v) for k, v in vals.items()}


def pick(d, sub):
    for k, v in d.items():
        if sub in k:
            return v
    return None


def main():
    prof, config, out_prefix = sys.argv[1], sys.argv[2], sys.argv[3]
    res = {"config": config}
    # --- kernel time
    tr = rows(os.path.join(prof, "trace"), "*kernel_stats.csv")
    if tr:
        res["kernel_stats"] = [
            {"name": r["Name"][:120], "calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
             "pct": float(r["Percentage"])} for r in tr[:12]]
        it = [r for r in tr if any(k in r["Name"] for k in KERNELS)]
        if it:
            res["iter_kernel"] = it[0]["Name"][:120]
            res["iter_avg_us_rocprof"] = float(it[0]["AverageNs"]) / 1e3
    # --- calibration: KB counted per byte moved, 8-B and 3×8-B per lane reads, 24-B writes
    cal_b = 768 << 20
    cf = counter_by_kernel(os.path.join(prof, "cfetch"), "FETCH_SIZE")
    cw = counter_by_kernel(os.path.join(prof, "cwrite"), "WRITE_SIZE")
    fac = {}
    if cf:
        for k in ("k_read8", "k_read24"):
            v = pick(cf, k)
            if v:
                fac[k] = cal_b / (v * 1024.0)
    if cw:
        v = pick(cw, "k_write24")
        if v:
            fac["k_write24"] = cal_b / (v * 1024.0)
    res["calibration_bytes_per_counted_byte"] = fac
    # --- traffic of the dominant kernel
    fk = counter_by_kernel(os.path.join(prof, "fetch"), "FETCH_SIZE")
    wk = counter_by_kernel(os.path.join(prof, "write"), "WRITE_SIZE")
    f = w = None
    for k in KERNELS:
        if pick(fk, k) is not None:
            f, w = pick(fk, k), pick(wk, k)
            break
    if f is not None and w is not None:
        rf = fac.get("k_read24", 1.0)
        rw = fac.get("k_write24", 1.0)
        res["fetch_kb_raw"] = f
        res["write_kb_raw"] = w
        res["bytes_per_launch"] = f * 1024.0 * rf + w * 1024.0 * rw
        res["bytes_per_launch_uncorrected"] = (f + w) * 1024.0
    os.makedirs(os.path.dirname(out_prefix), exist_ok=True)
    json.dump(res, open(out_prefix + ".json", "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
