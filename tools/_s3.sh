cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
ok() { rc=$1; echo "[$2] rc=$rc"; if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then exit $rc; fi; }
timeout -k 10 400 python -m pytest tests/test_fused_resnet_gpu.py tests/test_eager_graph_gpu.py -q -x --timeout 200 > gpurun_out/pytest_rn.log 2>&1; ok $? pytest_rn
timeout -k 10 200 python bench.py --model resnet20 --impl fused --steps 50 --warmup 5 > gpurun_out/bench_rn_fused.log 2>&1; ok $? rn_fused
rm -rf gpurun_out/prof_rn; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rn -o run -- python3 bench.py --model resnet20 --impl fused --steps 20 --warmup 5 > gpurun_out/prof_rn.log 2>&1; ok $? prof
echo done
