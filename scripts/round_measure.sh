#!/bin/bash
# Round-end measurement on the GPU box, in two calls (each fits gpurun's limit):
#   gpurun -- bash scripts/round_measure.sh TAG a   PMC traffic of the GAMG iteration at
#             C3, C2 and C5 (scripts/profile_amg.sh → profiles/traffic_<config>.json,
#             which bench.py reads), the GPU test suite and smoke()
#   gpurun -- bash scripts/round_measure.sh TAG b   the bench lines (C3 default with its
#             CPU legs, C2, C5) and the rocprofv3 kernel stats of the default bench command
# Everything lands under gpurun_out/ (TAG_*.log, prof_TAG_*, traffic_*.json) for profiles/.
# Under rocprofv3 the HIP runtime submits each graph node as its own packet
# (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0): the tracer's queue interception walks a
# multi-packet batch past the end of the 1 MiB queue ring when one straddles
# it — kernel durations are unaffected.
set -u
T=${1:-fin}
PHASE=${2:-a}
traffic() {  # config reps
  echo "$1:400:bash scripts/profile_amg.sh ${T}_$1 $1 $2 && python3 tools/amg_traffic.py gpurun_out/prof_${T}_$1/summary.json $1 profiles/traffic_$1.json && cp profiles/traffic_$1.json gpurun_out/"
}
if [ "$PHASE" = a ]; then
  exec bash scripts/gpu_job.sh "$T" \
    "$(traffic C3_1M 50)" "$(traffic C2_100k 50)" "$(traffic C5_10M_dense 20)" \
    "tests:500:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
    "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'"
else
  exec bash scripts/gpu_job.sh "$T" \
    "c3:400:python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench_C3_1M.json" \
    "c2:200:python bench.py --config C2_100k --no-cpu --steps 20 --warmup 5 > gpurun_out/${T}_bench_C2_100k.json" \
    "c5:300:python bench.py --config C5_10M_dense --no-cpu --steps 5 --warmup 2 > gpurun_out/${T}_bench_C5_10M_dense.json" \
    "prof:400:cd /tmp && export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_benchprof -o t -- python3 tools/maps_bench.py --steps 20 --warmup 5"
fi
