cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/reh && export TMPDIR=/tmp DMLC_DIST_BACKEND=gloo
for m in cifar_cnn resnet20; do
  for n in 2 4 8; do
    # 8 ranks on ONE GPU oversubscribe its hardware queues: the xGMI exchange kernels of the 8
    # processes (which wait on each other) then time out; N=8 rehearses the RCCL path (gloo here)
    ar=auto; [ $n -ge 8 ] && ar=rccl
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 20 --warmup 5 --model $m --allreduce $ar > gpurun_out/reh/${m}_n$n.log 2>&1 || { echo "fail $m $n"; tail -20 gpurun_out/reh/${m}_n$n.log; exit 1; }
    grep -h '^{' gpurun_out/reh/${m}_n$n.log > gpurun_out/reh/${m}_n$n.json
    echo "$m $n $(python3 -c "import json;d=json.load(open('gpurun_out/reh/${m}_n$n.json'));print(d['value'], d['ms_per_step'], d['config']['comm'].get('allreduce'), d['config']['comm'].get('schedule'))")"
  done
done
