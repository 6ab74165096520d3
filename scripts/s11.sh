bash scripts/gpu_job.sh s11 \
 "tests:420:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:200:python -u bench.py" \
 "profc2:400:bash scripts/profile_r.sh fc2 C2_100k" \
 "profc3:500:bash scripts/profile_r.sh fc3 C3_1M" \
 "c3:200:python -u bench.py --config C3_1M --steps 3 --warmup 1 --cpu-steps 1" \
 "tr:200:python -u tools/trace_iter.py C2_100k C3_1M --out gpurun_out/s11_trace.json"
