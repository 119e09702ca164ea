cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fused_resnet_gpu.py tests/test_fused_resnet_dp_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_rn.log 2>&1 || { echo pytest failed; tail -40 gpurun_out/pytest_rn.log; exit 1; }
timeout -k 10 200 python tools/rn_kbench.py > gpurun_out/rnk.json 2> gpurun_out/rnk.err || { tail gpurun_out/rnk.err; exit 1; }
timeout -k 10 200 python bench.py --model resnet20 --steps 100 --warmup 10 > gpurun_out/bench_rn.log 2>&1 || exit 1
DMLC_RN_MERGED_BWD=0 timeout -k 10 200 python bench.py --model resnet20 --steps 100 --warmup 10 > gpurun_out/bench_rn_split.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --model resnet20 --batch 1024 --steps 30 --warmup 5 > gpurun_out/bench_rn_b1024.log 2>&1 || exit 1
echo done
