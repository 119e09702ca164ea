#!/bin/bash
# CLI training throughput vs bench.py: the reference entry point on synthetic data,
# batch 256, chunked chained-graph replays between log points; prints the metrics.jsonl records.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
rm -rf /tmp/dmlc_cli_run
timeout -k 10 300 python cifar10cnn.py --synthetic --batch_size=256 --generations=6000 --output_every=1000 \
  --eval_every=100000 --log_dir=/tmp/dmlc_cli_run > gpurun_out/cli_train.log 2>&1 || exit $?
cp /tmp/dmlc_cli_run/metrics.jsonl gpurun_out/cli_metrics.jsonl
ls /tmp/dmlc_cli_run > gpurun_out/cli_logdir.txt
cat gpurun_out/cli_metrics.jsonl
