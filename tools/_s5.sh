cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_fused_resnet_gpu.py tests/test_fused_resnet_dp_gpu.py -q -x --timeout 200 > gpurun_out/pytest_rn.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/pytest_rn.log; exit 1; }
timeout -k 10 200 python tools/rn_kbench.py > gpurun_out/rnk_base.json 2> gpurun_out/rnk.err || exit 1
DMLC_RN_WGRAD_BRANCH=0 timeout -k 10 200 python tools/rn_kbench.py > gpurun_out/rnk_nobranch.json 2>> gpurun_out/rnk.err || exit 1
DMLC_RN_SLAB_MB=8 timeout -k 10 200 python tools/rn_kbench.py > gpurun_out/rnk_slab8.json 2>> gpurun_out/rnk.err || exit 1
DMLC_RN_SLAB_MB=2 timeout -k 10 200 python tools/rn_kbench.py > gpurun_out/rnk_slab2.json 2>> gpurun_out/rnk.err || exit 1
echo done
