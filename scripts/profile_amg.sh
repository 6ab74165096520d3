#!/bin/bash
# rocprofv3 passes over the GAMG-PCG iteration (tools/amg_profile.py): kernel
# trace, then FETCH_SIZE and WRITE_SIZE in separate passes (counters never
# share a run with tracing domains).  Run on the GPU box.
#   bash scripts/profile_amg.sh TAG CONFIG [REPS] [name=value ...]   (engine options)
#   TRACE_ONLY=1: the kernel trace pass only
set -u
TAG=$1; CFG=${2:-C3_1M}; REPS=${3:-50}; shift 3 2>/dev/null || shift $#
SETS=${*:+--set $*}
export TMPDIR=/tmp
# one packet per graph node under the tracer (round_measure.sh)
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
D=gpurun_out/prof_$TAG
mkdir -p $D
P="python3 tools/amg_profile.py --config $CFG --reps $REPS --precond ${PRECOND:-gamg} $SETS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o t -- $P > $D/trace.log 2>&1 || exit $?
if [ "${TRACE_ONLY:-0}" = 1 ]; then python3 tools/amg_pmc_summary.py $D $REPS $D/summary.json; exit $?; fi
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o f -- $P > $D/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o w -- $P > $D/write.log 2>&1 || exit $?
python3 tools/amg_pmc_summary.py $D $REPS $D/summary.json
