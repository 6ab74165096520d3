"""Per-kernel SQ / GRBM counters of the GAMG-PCG iteration from a rocprofv3
--pmc run of tools/amg_profile.py (the last `reps` iterations, as
tools/amg_pmc_summary.py): average of every counter per kernel position k of
the iteration, plus derived occupancy (SQ_WAVE_CYCLES / SQ_BUSY_CYCLES: the
mean resident waves while the SQ is busy) and the stall split.

    python tools/sq_summary.py <counter_dir> <reps> <out.json>
"""
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from amg_pmc_summary import iterations, load, short  # noqa: E402


def main():
    d, reps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    cc = load(d, "*counter_collection.csv")
    names = sorted({r["Counter_Name"] for r in cc})
    per = defaultdict(lambda: defaultdict(list))
    meta = {}
    for ctr in names:
        disp = sorted((int(r["Dispatch_Id"]), r["Kernel_Name"], int(r["Grid_Size"]), float(r["Counter_Value"]),
                       r.get("VGPR_Count"), r.get("SGPR_Count"))
                      for r in cc if r["Counter_Name"] == ctr)
        for it in iterations(disp, reps):
            for k, (_, n, g, v, vg, sg) in enumerate(it):
                per[(k, short(n), g)][ctr].append(v)
                meta[(k, short(n), g)] = {"vgpr": vg, "sgpr": sg}
    rows = []
    for key in sorted(per):
        k, n, g = key
        row = {"k": k, "name": n, "grid": g, **meta[key]}
        for ctr, v in per[key].items():
            row[ctr] = sum(v) / len(v)
        wc, bc = row.get("SQ_WAVE_CYCLES"), row.get("SQ_BUSY_CYCLES")
        if wc and bc:
            row["waves_resident_per_busy_cycle"] = wc / bc
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in row:
                    row[c + "_frac"] = row[c] / wc
        rows.append(row)
    json.dump({"reps": reps, "counters": names, "kernels": rows}, open(out, "w"), indent=1)
    for r in rows:
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))


if __name__ == "__main__":
    main()
