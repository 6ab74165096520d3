"""Idle time inside bench steps from a rocprofv3 kernel trace (CSV): per step
(a step starts at each k_assemble launch) the summed kernel time, the summed
gaps between consecutive kernels and the largest gaps with their neighbours.

    python3 tools/step_gaps.py gpurun_out/X/trace/t_kernel_trace.csv [out.json]
"""
import csv
import json
import sys


def short(n):
    n = n.split("(")[0]
    return n.replace("void ", "").replace("mfea::", "")


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2].startswith("k_assemble")]
    steps = []
    for a, b in zip(starts, starts[1:] + [len(rows)]):
        ks = rows[a:b]
        busy = sum(e - s for s, e, _ in ks)
        gaps = []
        end = ks[0][1]
        over = 0  # kernel time overlapped with an earlier kernel (concurrent streams)
        for k in range(1, len(ks)):
            g = ks[k][0] - end
            if g > 0:
                gaps.append((g, ks[k - 1][2], ks[k][2]))
            else:
                over += min(end, ks[k][1]) - ks[k][0]
            end = max(end, ks[k][1])
        span = end - ks[0][0]
        gaps.sort(reverse=True)
        steps.append({"span_us": span / 1e3, "busy_us": busy / 1e3, "kernels": len(ks),
                      "gap_us": sum(g for g, _, _ in gaps) / 1e3, "overlap_us": over / 1e3,
                      "top_gaps": [(round(g / 1e3, 2), p, n) for g, p, n in gaps[:8]]})
    out = {"steps": steps[1:-1] if len(steps) > 2 else steps}
    for s in out["steps"]:
        print(f"span {s['span_us']:.1f} busy {s['busy_us']:.1f} gaps {s['gap_us']:.1f} overlap {s['overlap_us']:.1f} us, {s['kernels']} kernels")
        for g in s["top_gaps"]:
            print("   ", g)
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
