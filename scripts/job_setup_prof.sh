#!/bin/bash
# kernel traces of one GAMG solve's numeric setup at C3 and C2 (tools/setup_pmc_summary.py)
set -u
T=${1:-sp}
bash scripts/gpu_job.sh $T \
  "c3:200:TRACE_ONLY=1 bash scripts/profile_amg.sh ${T}_C3 C3_1M 10 && python3 tools/setup_pmc_summary.py gpurun_out/prof_${T}_C3 gpurun_out/${T}_setup_C3.json" \
  "c2:200:TRACE_ONLY=1 bash scripts/profile_amg.sh ${T}_C2 C2_100k 10 && python3 tools/setup_pmc_summary.py gpurun_out/prof_${T}_C2 gpurun_out/${T}_setup_C2.json"
