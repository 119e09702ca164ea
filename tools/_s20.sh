cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python tools/rn_kbench.py > gpurun_out/rnk_b1.json 2> gpurun_out/rnk.err || { tail gpurun_out/rnk.err; exit 1; }
DMLC_RN_WGRAD_BRANCH=0 timeout -k 10 200 python tools/rn_kbench.py > gpurun_out/rnk_b0.json 2>> gpurun_out/rnk.err || { tail gpurun_out/rnk.err; exit 1; }
DMLC_RN_WGRAD_BRANCH=0 timeout -k 10 200 python bench.py --model resnet20 --steps 100 --warmup 10 > gpurun_out/bench_rn_b0.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --model resnet20 --steps 100 --warmup 10 > gpurun_out/bench_rn_b1.log 2>&1 || exit 1
echo done
