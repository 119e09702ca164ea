cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_fused_dp_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_fused.log; exit 1; }
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
DMLC_SPLIT_WGRAD=1 timeout -k 10 200 python bench.py --steps 400 --warmup 40 > gpurun_out/bench_split.log 2>&1 || exit 1
rm -rf gpurun_out/prof; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --warmup 10 > gpurun_out/prof.log 2>&1 || exit 1
echo done
