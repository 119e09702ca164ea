#!/usr/bin/env python3
"""Flag-compatible entry point of the reference script (/root/reference/cifar10cnn.py).

  python cifar10cnn.py --ps_hosts=localhost:2222 --worker_hosts=localhost:2223,localhost:2224 \\
      --job_name=ps --task_index=0            # rendezvous host (exits when the workers finish)
  python cifar10cnn.py ... --job_name=worker --task_index=0   # DP rank 0 (chief: checkpoints, logs)
  python cifar10cnn.py ... --job_name=worker --task_index=1   # DP rank 1

Same six flags as the reference (README.md:9-14); see ``python cifar10cnn.py --help`` for the
extension flags (batch size, steps, dtype, model, synthetic data, ...).  Training is synchronous data
parallel over RCCL (one process per GPU) with the fused MI355X HIP kernels, instead of the
reference's asynchronous gRPC parameter server.  For single-node multi-GPU runs, ``python -m
dmlc.launch --nproc N -- <flags>`` starts and supervises the N worker processes.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import dmlc  # noqa: E402,F401
from dmlc.engine.trainer import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
