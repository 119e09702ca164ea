cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for s in 8 6 4 3 2; do
  timeout -k 10 120 python tools/kbench.py --fc1-split $s > gpurun_out/kbench_s$s.json 2>/dev/null || exit 1
done
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > gpurun_out/bench.log 2>&1 || exit 1
echo done
