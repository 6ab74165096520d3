"""FETCH_SIZE / WRITE_SIZE calibration per access width (tools/ubench_stream.hip).

Every kernel of the micro-benchmark reads (k_read*, k_gather8) or writes
(k_write24) exactly `bytes` once; the ratio counter × 1024 / bytes is the
factor rocprofv3 reports for that width (MI355X_MICROARCH.md § HBM: ½ for a
16-B/lane stream).  Output: per kernel the raw ratio and the factor that turns
the counter into bytes.

    python tools/fetch_calib.py <dir with fetch/ and write/ counter CSVs> [bytes] > out.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d, nbytes=768 << 20):
    out = {"bytes_per_kernel": nbytes, "kernels": {}}
    for key, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        vals = defaultdict(list)
        for f in glob.glob(os.path.join(d, key, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == ctr:
                    n = r["Kernel_Name"]
                    n = n[: n.index("(")] if "(" in n else n
                    vals[n.split()[-1]].append(float(r["Counter_Value"]) * 1024.0)
        for n, v in sorted(vals.items()):
            # the first of the three rounds reads a cold buffer; all three are
            # from HBM (the buffer is 3× the Infinity Cache)
            ratio = sum(v) / len(v) / nbytes
            out["kernels"].setdefault(n, {})[key] = {"ratio": round(ratio, 4),
                                                    "factor": round(1.0 / ratio, 3) if ratio else None,
                                                    "runs": len(v)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:]))
