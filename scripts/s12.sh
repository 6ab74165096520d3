D=gpurun_out/prof_g2
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o t -- python3 bench.py --config C2_100k --steps 1 --warmup 0 --no-cpu > $D/trace.log 2>&1
echo rc=$?
find $D -name "*kernel_stats.csv" | head -1 | xargs head -4
