cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
ok() { rc=$1; echo "[$2] rc=$rc"; if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then exit $rc; fi; }
true
timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/bench.log 2>&1; ok $? bench
timeout -k 10 200 python bench.py --impl eager --steps 50 --warmup 5 > gpurun_out/bench_eager.log 2>&1; ok $? eager
timeout -k 10 200 python bench.py --model resnet20 --steps 30 --warmup 5 > gpurun_out/bench_resnet.log 2>&1; ok $? resnet
timeout -k 10 200 python bench.py --batch 1024 --steps 100 --warmup 10 > gpurun_out/bench_b1024.log 2>&1; ok $? b1024
timeout -k 10 200 python bench.py --batch 1024 --dtype fp8 --steps 100 --warmup 10 > gpurun_out/bench_b1024_fp8.log 2>&1; ok $? b1024fp8
timeout -k 10 200 python bench.py --dtype fp8 --steps 200 --warmup 20 > gpurun_out/bench_fp8.log 2>&1; ok $? fp8
timeout -k 10 300 python cifar10cnn.py --synthetic --batch_size=256 --generations=600 --output_every=200 --eval_every=300 --eval_batches=0 --log_dir=/tmp/run1 --learning_rate=0.0005 --relu_logits=false > gpurun_out/train_cli.log 2>&1; ok $? train
rm -rf gpurun_out/prof; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --warmup 10 > gpurun_out/prof.log 2>&1; ok $? prof
echo done
