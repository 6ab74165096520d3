bash scripts/gpu_job.sh s4 \
 "tests:420:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "c2_256:120:MFEA_ELL_BS=256 python -u bench.py --no-cpu" \
 "c2_128:120:MFEA_ELL_BS=128 python -u bench.py --no-cpu" \
 "c2_64:120:MFEA_ELL_BS=64 python -u bench.py --no-cpu" \
 "c3_256:200:MFEA_ELL_BS=256 python -u bench.py --no-cpu --config C3_1M --steps 3 --warmup 1" \
 "c3_128:200:MFEA_ELL_BS=128 python -u bench.py --no-cpu --config C3_1M --steps 3 --warmup 1" \
 "tr2:200:python -u tools/trace_iter.py C2_100k --out gpurun_out/s4_trace.json"
