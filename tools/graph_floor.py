#!/usr/bin/env python3
"""Per-kernel floor of back-to-back launches replayed from one HIP graph on this GPU.

Captures N dependent launches of a trivial elementwise kernel (n elements -> n/1024 .. workgroups)
into one graph and reports the replay time per launch -- the cost every kernel boundary of a
captured training step pays before doing any work (ResNet-20: 58 launches per step).
  python tools/graph_floor.py      -> one JSON line {elements: us_per_launch, ...}"""
import json

import torch


def main():
    res = {}
    for n in (256, 65536, 262144, 1 << 22):
        x = torch.zeros(n, device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                x.add_(1.0)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        N = 200
        with torch.cuda.graph(g):
            for _ in range(N):
                x.add_(1.0)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        R = 20
        for _ in range(R):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        res[n] = round(a.elapsed_time(b) * 1000.0 / (R * N), 3)
    print(json.dumps({"us_per_launch_by_elements": res}), flush=True)


if __name__ == "__main__":
    main()
