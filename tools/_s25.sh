cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
export DMLC_DIST_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 50 --warmup 10 > gpurun_out/bench_n2_xgmi.log 2>&1 || { tail -30 gpurun_out/bench_n2_xgmi.log; exit 1; }
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 50 --warmup 10 --allreduce rccl > gpurun_out/bench_n2_coll.log 2>&1 || { tail -30 gpurun_out/bench_n2_coll.log; exit 1; }
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 20 --warmup 5 --model resnet20 > gpurun_out/bench_n2_rn.log 2>&1 || { tail -30 gpurun_out/bench_n2_rn.log; exit 1; }
echo done
