#!/bin/bash
# Round-5 experiment on the GPU box: the compact down sweep's row sets and
# lanes.  (1) same-box A/B of the R̂ lanes per row at C3 / C2 / C5, (2) the
# C3 iteration traced with the two row sets as separate launches, (3) SQ
# counters (occupancy, stall split) of every iteration kernel at C3.
set -u
T=${1:-exp}
mkdir -p gpurun_out
export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
P="python3 tools/amg_profile.py --config C3_1M --reps 30"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU"
bash scripts/gpu_job.sh $T \
  "ab:500:python3 tools/amg_ab.py --configs C3_1M C2_100k C5_10M_dense --option amg_restrict_lanes --values 0 4 2 1 --rounds 2 --steps 3 > gpurun_out/${T}_ab_lanes.jsonl" \
  "split:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_split/trace -o t -- $P --set amg_down_split=1 && python3 tools/amg_pmc_summary.py gpurun_out/${T}_split 30 gpurun_out/${T}_split.json" \
  "sq:200:timeout -s KILL 150 rocprofv3 --pmc $SQ GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_sq -o s -- $P && python3 tools/sq_summary.py gpurun_out/${T}_sq 30 gpurun_out/${T}_sq.json" \
  "sqsplit:200:timeout -s KILL 150 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/${T}_sqs -o s -- $P --set amg_down_split=1 && python3 tools/sq_summary.py gpurun_out/${T}_sqs 30 gpurun_out/${T}_sqsplit.json"
