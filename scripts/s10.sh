O="MFEA_LIB=$PWD/ab/libmfea_8122a0b.so MFEA_ELL_BS=256"
bash scripts/gpu_job.sh s10 \
 "tests:420:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "old1:120:$O python -u bench.py --no-cpu --steps 10" \
 "new1:120:python -u bench.py --no-cpu --steps 10" \
 "old2:120:$O python -u bench.py --no-cpu --steps 10" \
 "new2:120:python -u bench.py --no-cpu --steps 10" \
 "newhc:120:MFEA_ELL_HC=1 python -u bench.py --no-cpu --steps 10" \
 "c3:200:python -u bench.py --no-cpu --config C3_1M --steps 3 --warmup 1" \
 "c3nohc:200:MFEA_ELL_HC=0 python -u bench.py --no-cpu --config C3_1M --steps 3 --warmup 1"
