set -u
cd $GRAFT_REPO_ROOT
bash scripts/gpu_job.sh ln "amg:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_amg.py -k lane_splits" "ab:300:python -u tools/amg_ab.py --configs C5_10M_dense --option amg_restrict_lanes --values 8 16 --steps 2 --rounds 2" || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pj1 -o t -- python3 tools/amg_ab.py --configs C3_1M --option amg_w_k --values 0 --steps 2 --rounds 1 > gpurun_out/pj1.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pj2 -o t -- python3 bench.py --no-cpu --no-full-run --no-jacobi --steps 10 --warmup 3 > gpurun_out/pj2.log 2>&1
