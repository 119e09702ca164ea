cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 2000 --warmup 100 > gpurun_out/bench_g.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 2000 --warmup 100 --no-graph > gpurun_out/bench_ng.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 2000 --warmup 100 > gpurun_out/bench_g2.log 2>&1 || exit 1
echo done
