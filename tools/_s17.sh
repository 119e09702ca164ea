cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_fused_gpu.py tests/test_fused_dp_gpu.py tests/test_fp8_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_fused.log; exit 1; }
for r in 4 2; do DMLC_HEAD_ROWS=$r timeout -k 10 120 python tools/kbench.py > gpurun_out/kbench_h$r.json 2> gpurun_out/kbench.err || { tail gpurun_out/kbench.err; exit 1; }; done
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
timeout -k 10 200 python tools/ktiming.py > gpurun_out/ktiming.json 2> gpurun_out/ktiming.err || { tail gpurun_out/ktiming.err; exit 1; }
echo done
