"""Per-iteration time and HBM traffic of the GAMG-PCG iteration from rocprofv3
runs of tools/amg_profile.py (the last `reps` iterations = everything from the
last `reps` k_amg_cg_update dispatches on).

    python tools/amg_pmc_summary.py <prof_dir> <reps> <out.json>

<prof_dir>/trace (kernel trace), /fetch (--pmc FETCH_SIZE), /write (--pmc
WRITE_SIZE).  FETCH_SIZE is doubled (MI355X_MICROARCH.md § HBM: on gfx950 it
reports half the bytes of a wide coalesced read); WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, pattern):
    out = []
    for f in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def iterations(disp, reps):
    """disp: list of (dispatch_id, name, grid, value) sorted by id → the last
    reps iterations: GAMG kernels only, cut at every k_amg_cg_update, keeping
    the segments of the most common launch sequence (the profiled graph
    replays; a solve's first or last iteration, or a floating-row pass after
    the reps, has another)"""
    disp = [r for r in disp if "k_amg_" in r[1]]
    starts = [k for k, r in enumerate(disp) if "k_amg_cg_update" in r[1]]
    segs = [disp[s:(starts[a + 1] if a + 1 < len(starts) else len(disp))] for a, s in enumerate(starts)]
    sig = lambda seg: tuple((r[1], r[2]) for r in seg)
    counts = defaultdict(int)
    for seg in segs:
        counts[sig(seg)] += 1
    best = max(counts, key=counts.get) if counts else ()
    return [seg for seg in segs if sig(seg) == best][-reps:]


def short(n):
    n = n.replace("void mfea::", "").replace("mfea::", "")
    return n[: n.index("(")] if "(" in n else n


def main():
    prof, reps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    res = {"reps": reps}
    tr = load(os.path.join(prof, "trace"), "*kernel_trace.csv")
    if tr:
        disp = sorted(((int(r["Dispatch_Id"]), r["Kernel_Name"], int(r["Grid_Size_X"]),
                        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in tr))
        its = iterations(disp, reps)
        per = defaultdict(list)
        for it in its:
            for k, (_, n, g, us) in enumerate(it):
                per[(k, short(n), g)].append(us)
        res["launches_per_iteration"] = len(its[-1])
        res["iter_us_rocprof_sum"] = sum(sum(x[3] for x in it) for it in its) / len(its)
        res["iter_span_us_rocprof"] = None
        res["kernels"] = [{"k": k, "name": n, "grid": g, "avg_us": sum(v) / len(v)}
                          for (k, n, g), v in sorted(per.items())]
    for ctr, key, fac in (("FETCH_SIZE", "fetch", 2.0), ("WRITE_SIZE", "write", 1.0)):
        cc = load(os.path.join(prof, key), "*counter_collection.csv")
        if not cc:
            continue
        disp = sorted((int(r["Dispatch_Id"]), r["Kernel_Name"], int(r["Grid_Size"]), float(r["Counter_Value"]))
                      for r in cc if r["Counter_Name"] == ctr)
        its = iterations(disp, reps)
        tot = [sum(x[3] for x in it) * 1024.0 * fac for it in its]
        res[f"{key}_bytes_per_iteration"] = sum(tot) / len(tot)
        per = defaultdict(list)
        for it in its:
            for k, (_, n, g, v) in enumerate(it):
                per[(k, short(n), g)].append(v * 1024.0 * fac)
        for row in res.get("kernels", []):
            v = per.get((row["k"], row["name"], row["grid"]))
            if v:
                row[f"{key}_bytes"] = sum(v) / len(v)
    if "fetch_bytes_per_iteration" in res and "write_bytes_per_iteration" in res:
        res["hbm_bytes_per_iteration"] = res["fetch_bytes_per_iteration"] + res["write_bytes_per_iteration"]
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
