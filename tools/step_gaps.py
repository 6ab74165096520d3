"""Timeline of the last load step in a rocprofv3 kernel trace (bench.py under
`rocprofv3 --kernel-trace --output-format csv`): kernel time, idle gaps
between consecutive kernels, and the longest gaps with their neighbours.

    python tools/step_gaps.py gpurun_out/prof_x/trace/t_kernel_trace.csv
"""
import csv
import sys


def main(path, first="k_assemble", last="k_stress"):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if first in r[2]]
    ends = [i for i, r in enumerate(rows) if last in r[2]]
    a = starts[-1]
    b = max(i for i in ends if i >= a)
    seg = rows[a:b + 1]
    busy = sum(e - s for s, e, _ in seg)
    span = seg[-1][1] - seg[0][0]
    gaps = [(seg[i + 1][0] - seg[i][1], seg[i][2][:60], seg[i + 1][2][:60]) for i in range(len(seg) - 1)]
    print(f"step span {span / 1e3:.1f} us, kernels {len(seg)}, busy {busy / 1e3:.1f} us, "
          f"gaps {sum(g for g, _, _ in gaps) / 1e3:.1f} us")
    for g, x, y in sorted(gaps, reverse=True)[:12]:
        print(f"  gap {g / 1e3:8.1f} us  after {x}  before {y}")


if __name__ == "__main__":
    main(*sys.argv[1:])
