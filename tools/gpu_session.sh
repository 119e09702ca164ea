#!/bin/bash
# One gpurun session: smoke -> GPU tests -> bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash / abort / timeout (rc >= 124 or signal) ends the
# session immediately (plain test failures, rc 1, do not).
# usage: tools/gpu_session.sh [steps...]   (default: smoke tests bench prof; also: fused kbench ktiming xgmi rn eager)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${*:-smoke tests bench prof}
ok() { local rc=$1 name=$2; echo "[$name] rc=$rc"; if [ "$rc" -ge 2 ] && [ "$rc" -ne 5 ]; then echo "[$name] stopping session"; exit "$rc"; fi; }
for s in $STEPS; do
  case $s in
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; ok $? smoke ;;
    xgmi) timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_xgmi.log 2>&1; ok $? xgmi ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; ok $? tests ;;
    bench) timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.log 2>&1; ok $? bench ;;
    fused) timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_fused_dp_gpu.py tests/test_fp8_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1; ok $? fused ;;
    fault) timeout -k 10 400 python -u -m pytest tests/test_fault_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_fault.log 2>&1; ok $? fault ;;
    b20) timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20.log 2>&1; ok $? b20 ;;
    b400) timeout -k 10 200 python bench.py --steps 400 --warmup 20 > gpurun_out/bench400.log 2>&1; ok $? b400 ;;
    b1024) timeout -k 10 200 python bench.py --steps 200 --warmup 20 --batch 1024 > gpurun_out/bench1024.log 2>&1; ok $? b1024 ;;
    rnprof) rm -rf gpurun_out/rnprof; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rnprof -o run -- python3 bench.py --model resnet20 --steps 30 --warmup 5 > gpurun_out/rnprof.log 2>&1; ok $? rnprof ;;
    lat) timeout -k 10 200 python tools/launch_latency.py > gpurun_out/launch_latency.json 2> gpurun_out/launch_latency.err; ok $? lat ;;
    cnn) timeout -k 10 400 python -u -m pytest tests/test_cnn_kernels_gpu.py tests/test_fused_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_cnn.log 2>&1; ok $? cnn ;;
    kbench) timeout -k 10 200 python tools/kbench.py ${KBENCH_ARGS:-} > gpurun_out/kbench.json 2> gpurun_out/kbench.err; ok $? kbench ;;
    ktiming) DMLC_TIMING=1 timeout -k 10 200 python tools/ktiming.py > gpurun_out/ktiming.json 2> gpurun_out/ktiming.err; ok $? ktiming ;;
    rn) timeout -k 10 300 python bench.py --model resnet20 --steps 100 --warmup 10 > gpurun_out/bench_rn.log 2>&1; ok $? rn ;;
    eager) timeout -k 10 300 python bench.py --impl eager --steps 50 --warmup 5 > gpurun_out/bench_eager.log 2>&1; ok $? eager ;;
    prof) rm -rf gpurun_out/prof; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --warmup 10 > gpurun_out/prof.log 2>&1; ok $? prof ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "session done"
