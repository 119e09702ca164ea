cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -m gpu -q -x --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -ge 2 ] && [ $rc -ne 5 ] && exit $rc
timeout -k 10 200 python tools/kbench.py > gpurun_out/kbench.log 2>&1 || exit 1
timeout -k 10 200 python tools/ktiming.py > gpurun_out/ktiming.json 2> gpurun_out/ktiming.err || exit 1
timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/bench.log 2>&1 || exit 1
echo done
