#!/bin/bash
# A/B only (no tests): bash scripts/job_ab.sh TAG OPTION "VALUES" [CONFIGS...] [-- name=value ...]
set -u
T=$1; OPT=$2; VALS=$3; shift 3
CFGS=${*:-C3_1M C2_100k}
bash scripts/gpu_job.sh $T \
  "ab:500:python3 tools/amg_ab.py --configs $CFGS --option $OPT --values $VALS --rounds 3 --steps 3 ${SETS:+--set $SETS} > gpurun_out/${T}_ab.jsonl"
