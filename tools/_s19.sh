cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
timeout -k 10 200 python bench.py --steps 1000 --warmup 50 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
timeout -k 10 200 python bench.py --batch 1024 --steps 300 --warmup 30 > gpurun_out/bench_b1024.log 2>&1 || { tail -20 gpurun_out/bench_b1024.log; exit 1; }
timeout -k 10 200 python bench.py --batch 1024 --dtype fp8 --steps 300 --warmup 30 > gpurun_out/bench_b1024_fp8.log 2>&1 || exit 1
rm -rf gpurun_out/prof; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 100 --warmup 10 > gpurun_out/prof.log 2>&1 || exit 1
echo done
