"""Per-kernel time and HBM traffic of the GAMG numeric setup (one solve's
setup: from the last k_amg_a0 dispatch up to the next k_amg_cg_init) from the
rocprofv3 passes of scripts/profile_amg.sh over tools/amg_profile.py.

    python tools/setup_pmc_summary.py <prof_dir> <out.json>

FETCH_SIZE is doubled (MI355X_MICROARCH.md § HBM, calibrated per access width
in profiles/r3/fetch_calib_widths.json); WRITE_SIZE is taken as is.
"""
import json
import os
import sys

from amg_pmc_summary import load, short


def setup_slice(disp):
    a0 = [k for k, r in enumerate(disp) if "k_amg_a0" in r[1]]
    if not a0:
        return []
    s = a0[-1]
    e = next((k for k in range(s, len(disp)) if "k_amg_cg_init" in disp[k][1]), len(disp))
    return disp[s:e]


def main():
    prof, out = sys.argv[1], sys.argv[2]
    rows = []
    tr = load(os.path.join(prof, "trace"), "*kernel_trace.csv")
    disp = sorted((int(r["Dispatch_Id"]), r["Kernel_Name"], int(r["Grid_Size_X"]),
                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in tr)
    for k, (_, n, g, us) in enumerate(setup_slice(disp)):
        rows.append({"k": k, "name": short(n), "grid": g, "us": us})
    for ctr, key, fac in (("FETCH_SIZE", "fetch", 2.0), ("WRITE_SIZE", "write", 1.0)):
        cc = load(os.path.join(prof, key), "*counter_collection.csv")
        d = sorted((int(r["Dispatch_Id"]), r["Kernel_Name"], int(r["Grid_Size"]), float(r["Counter_Value"]))
                   for r in cc if r["Counter_Name"] == ctr)
        for k, (_, n, g, v) in enumerate(setup_slice(d)):
            if k < len(rows) and rows[k]["name"] == short(n):
                rows[k][key + "_MB"] = v * 1024.0 * fac / 1e6
    for r in rows:
        b = r.get("fetch_MB", 0) + r.get("write_MB", 0)
        r["TBps"] = b * 1e6 / (r["us"] * 1e-6) / 1e12 if r["us"] else None
    res = {"setup_us_rocprof_sum": sum(r["us"] for r in rows), "launches": len(rows),
           "hbm_MB": sum(r.get("fetch_MB", 0) + r.get("write_MB", 0) for r in rows), "kernels": rows}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))
    for r in rows:
        print(f"{r['k']:3d} {r['name'][:34]:34s} {r['us']:7.1f} us  fetch {r.get('fetch_MB', 0):7.1f} MB  "
              f"write {r.get('write_MB', 0):6.1f} MB  {r['TBps'] or 0:5.2f} TB/s")


if __name__ == "__main__":
    main()
