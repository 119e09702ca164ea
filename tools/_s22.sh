cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
DMLC_RN_MERGED_BWD=0 timeout -k 10 200 python bench.py --model resnet20 --batch 1024 --steps 30 --warmup 5 > gpurun_out/bench_rn_b1024_split.log 2>&1 || exit 1
DMLC_RN_WGRAD_BRANCH=1 timeout -k 10 200 python bench.py --model resnet20 --batch 1024 --steps 30 --warmup 5 > gpurun_out/bench_rn_b1024_branch.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --model resnet20 --batch 1024 --steps 30 --warmup 5 > gpurun_out/bench_rn_b1024.log 2>&1 || exit 1
echo done
