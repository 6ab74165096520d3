"""Print the lines of a scripts/job_quick.sh run (gpurun_out/TAG_*)."""
import json
import os
import sys

T = sys.argv[1]
D = "gpurun_out"
st = os.path.join(D, f"{T}_status.txt")
if os.path.exists(st):
    print("".join(l for l in open(st) if " rc=" in l), end="")
for c in ("c3", "c2", "c5"):
    f = os.path.join(D, f"{T}_{c}.json")
    if os.path.exists(f) and os.path.getsize(f):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(c, round(d["ms_per_step"], 4), d["cg_iters"], {k: round(v, 4) for k, v in d["step_breakdown_ms"].items() if isinstance(v, float)},
              "spmv", round(d["roofline"]["frac"], 3), "iter_us", round(d["roofline_iteration"]["avg_iteration_us"], 2))
f = os.path.join(D, f"{T}_trace.json")
if os.path.exists(f):
    d = json.load(open(f))
    print("trace sum", round(d["iter_us_rocprof_sum"], 2))
    for k in d["kernels"]:
        print(" ", k["k"], k["name"], k["grid"], round(k["avg_us"], 2))
