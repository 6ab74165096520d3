"""PMC traffic file for bench.py from a GAMG iteration profile summary.

    python tools/amg_traffic.py <summary.json> <config> <out traffic_<config>.json>

<summary.json>: tools/amg_pmc_summary.py over scripts/profile_amg.sh passes
(kernel trace + FETCH_SIZE + WRITE_SIZE).  Writes the measured HBM bytes per
launch of the SpMV kernel (k_amg_cg_w) and per whole iteration, which bench.py
reports as roofline.traffic / roofline_iteration.traffic for that config.
"""
import json
import sys


def main():
    src, cfg, out = sys.argv[1], sys.argv[2], sys.argv[3]
    d = json.load(open(src))
    w = [k for k in d["kernels"] if k["name"].startswith("k_amg_cg_w")]
    if not w or "fetch_bytes" not in w[0] or "write_bytes" not in w[0]:
        sys.exit("summary has no PMC bytes for k_amg_cg_w")
    res = {
        "config": cfg,
        "source": src,
        "spmv_kernel": "k_amg_cg_w",
        "spmv_bytes_per_launch": w[0]["fetch_bytes"] + w[0]["write_bytes"],
        "spmv_avg_us_rocprof": w[0]["avg_us"],
        "iter_kernel": "GAMG-PCG iteration",
        "iteration_bytes": d.get("hbm_bytes_per_iteration"),
        "iteration_us_rocprof_sum": d.get("iter_us_rocprof_sum"),
        "note": "FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md), WRITE_SIZE x1; "
                "FETCH counts Infinity-Cache (MALL) hits as well",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
