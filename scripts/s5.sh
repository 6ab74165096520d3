bash scripts/gpu_job.sh s5 \
 "cli:300:python -u -m pytest tests/test_cli.py -m gpu -x -v --timeout 200 --timeout-method thread" \
 "tests:420:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "bench:300:python -u bench.py" \
 "profc2:400:bash scripts/profile_r.sh r1b C2_100k" \
 "profc3:500:bash scripts/profile_r.sh r1b C3_1M" \
 "c5:700:python -u bench.py --config C5_10M_dense --steps 1 --warmup 1 --no-cpu"
