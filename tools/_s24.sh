cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/pmcA gpurun_out/pmcB
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d gpurun_out/pmcA -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/pmcA.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE -d gpurun_out/pmcB -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/pmcB.log 2>&1 || exit 1
echo done
