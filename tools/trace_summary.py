"""Per-kernel / per-grid summary of a rocprofv3 kernel trace (csv):
    python tools/trace_summary.py <t_kernel_trace.csv> [top]"""
import sys

import pandas as pd

t = pd.read_csv(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
t["dur_us"] = (t["End_Timestamp"] - t["Start_Timestamp"]) / 1e3
t["kernel"] = (t["Kernel_Name"].str.replace(r"\(.*", "", regex=True)
               .str.replace("void mfea::", "").str.replace("mfea::", "").str.slice(0, 44))
g = (t.groupby(["kernel", "Grid_Size_X"]).dur_us.agg(["count", "mean", "sum"])
     .reset_index().sort_values("sum", ascending=False))
print(f"total kernel time {t.dur_us.sum():.1f} us over {len(t)} launches")
print(g.head(top).to_string(index=False))
