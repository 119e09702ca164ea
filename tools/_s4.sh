cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
ok() { rc=$1; echo "[$2] rc=$rc"; if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then exit $rc; fi; }
timeout -k 10 700 python -m pytest tests -m gpu -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; ok $? pytest_gpu
timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/bench.log 2>&1; ok $? bench
echo done
