bash scripts/gpu_job.sh s6 \
 "tests:420:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "c2:120:python -u bench.py --no-cpu" \
 "c3:200:python -u bench.py --no-cpu --config C3_1M --steps 3 --warmup 1" \
 "c3nofin:200:MFEA_ELL_FIN=0 python -u bench.py --no-cpu --config C3_1M --steps 3 --warmup 1" \
 "c5:600:python -u bench.py --config C5_10M_dense --steps 1 --warmup 1 --no-cpu"
