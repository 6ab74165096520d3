bash scripts/gpu_job.sh s8 \
 "tests:420:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "c2:120:python -u bench.py" \
 "c3:200:python -u bench.py --no-cpu --config C3_1M --steps 3 --warmup 1" \
 "c5:600:python -u bench.py --config C5_10M_dense --steps 1 --warmup 0 --no-cpu"
