#!/bin/bash
# Round-end measurement on the GPU box (gpurun -- bash scripts/round_measure.sh TAG):
# PMC traffic of the GAMG iteration at C3 and C5 (scripts/profile_amg.sh →
# profiles/traffic_<config>.json, which bench.py reads), the GPU test suite,
# smoke(), the bench lines (C3 default with its CPU legs, C2, C5) and the
# rocprofv3 kernel stats of the default bench command.  Everything lands under
# gpurun_out/ (TAG_*.log, prof_TAG_*, traffic_*.json) for profiles/.
set -u
T=${1:-fin}
exec bash scripts/gpu_job.sh "$T" \
  "pc3:300:bash scripts/profile_amg.sh ${T}_c3 C3_1M 50 && python3 tools/amg_traffic.py gpurun_out/prof_${T}_c3/summary.json C3_1M profiles/traffic_C3_1M.json && cp profiles/traffic_C3_1M.json gpurun_out/" \
  "pc5:400:bash scripts/profile_amg.sh ${T}_c5 C5_10M_dense 20 && python3 tools/amg_traffic.py gpurun_out/prof_${T}_c5/summary.json C5_10M_dense profiles/traffic_C5_10M_dense.json && cp profiles/traffic_C5_10M_dense.json gpurun_out/" \
  "tests:500:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "c3:300:python bench.py" \
  "c2:200:python bench.py --config C2_100k --no-cpu" \
  "c5:300:python bench.py --config C5_10M_dense --no-cpu --steps 5 --warmup 2" \
  "prof:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_benchprof -o t -- python3 bench.py --no-cpu --steps 10 --warmup 3"
