#!/bin/bash
# GPU-box A/B + trace run: gpurun -- bash scripts/exp_ab.sh TAG OPTION "VALUES" [CONFIGS...]
#   the GAMG tests first (a kernel change must keep parity), then tools/amg_ab.py over the
#   option's values, then the C3 iteration trace at the first value.
set -u
T=$1; OPT=$2; VALS=$3; shift 3
CFGS=${*:-C3_1M C2_100k C5_10M_dense}
export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
FIRST=${VALS%% *}
bash scripts/gpu_job.sh $T \
  "tests:300:python -u -m pytest tests/test_gpu_amg.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ab:500:python3 tools/amg_ab.py --configs $CFGS --option $OPT --values $VALS --rounds 2 --steps 3 > gpurun_out/${T}_ab.jsonl" \
  "trace:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_tr/trace -o t -- python3 tools/amg_profile.py --config C3_1M --reps 30 --set $OPT=$FIRST && python3 tools/amg_pmc_summary.py gpurun_out/${T}_tr 30 gpurun_out/${T}_trace.json"
