#!/bin/bash
# GPU-box check of the current tree: gpu tests, smoke, bench (C3 default, C2).
#   gpurun -- bash scripts/job_check.sh TAG
TAG=${1:-chk}
exec bash scripts/gpu_job.sh "$TAG" \
  "tests:420:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py" \
  "bench_c2:200:python bench.py --config C2_100k --no-cpu"
