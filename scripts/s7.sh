bash scripts/gpu_job.sh s7 \
 "geo:300:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k geometries --timeout 120 --timeout-method thread" \
 "c2a:120:MFEA_ELL_FIN=0 python -u bench.py --no-cpu" \
 "c2b:120:MFEA_ELL_FIN=0 python -u bench.py --no-cpu" \
 "c2sell:120:MFEA_CG_KERNEL=sell python -u bench.py --no-cpu" \
 "c5nofin:600:MFEA_ELL_FIN=0 python -u bench.py --config C5_10M_dense --steps 1 --warmup 0 --no-cpu" \
 "c5sell:600:MFEA_CG_KERNEL=sell python -u bench.py --config C5_10M_dense --steps 1 --warmup 0 --no-cpu"
