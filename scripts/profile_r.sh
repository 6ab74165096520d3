#!/bin/bash
# rocprofv3 passes for the bench workload ($1 = tag, $2 = config): kernel trace,
# then FETCH_SIZE and WRITE_SIZE in separate passes (counters never share a run
# with tracing domains), plus the calibration kernels.  Run on the GPU box.
set -u
TAG=$1; CFG=${2:-C2_100k}
D=gpurun_out/prof_$TAG
mkdir -p $D
# rocprofv3 traces the hipGraph-replayed kernels too (no MFEA_NO_GRAPH: eager
# launches under the profiler inflate a 6 µs kernel's duration by ≈ 1.5 µs)
B="python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o t -- $B > $D/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o f -- $B > $D/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o w -- $B > $D/write.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/cfetch -o cf -- ./tools/ubench_stream > $D/cfetch.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/cwrite -o cw -- ./tools/ubench_stream > $D/cwrite.log 2>&1 || exit $?
python3 tools/pmc_summary.py $D $CFG $D/summary
