bash scripts/gpu_job.sh s9 \
 "old1:120:MFEA_LIB=$PWD/ab/libmfea_8122a0b.so python -u bench.py --no-cpu --steps 10" \
 "new1:120:python -u bench.py --no-cpu --steps 10" \
 "old2:120:MFEA_LIB=$PWD/ab/libmfea_8122a0b.so python -u bench.py --no-cpu --steps 10" \
 "new2:120:python -u bench.py --no-cpu --steps 10" \
 "newbs256:120:MFEA_ELL_BS=256 python -u bench.py --no-cpu --steps 10"
