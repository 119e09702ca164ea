#!/usr/bin/env python3
"""Per-kernel device time and inter-kernel gaps of the training step from a rocprofv3 kernel trace.

  python tools/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv [--last N]

Takes the dmlc:: kernels of the last N complete steps (a step ends with k_sgd), prints the median
duration of each kernel position and the median idle gap before it (end of the previous kernel ->
start of this one), and the median step span (first kernel start -> k_sgd end).
"""
import argparse
import csv
import statistics as st


def short(name: str) -> str:
    n = name.split("(")[0].replace("dmlc::", "").replace("void ", "")
    return n.split("<")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=40)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            if "dmlc::" not in r["Kernel_Name"]:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    steps, cur = [], []
    for r in rows:
        cur.append(r)
        if r[2] == "k_sgd":
            steps.append(cur)
            cur = []
    steps = [s for s in steps if len(s) == len(steps[-1])][-args.last:]
    if not steps:
        raise SystemExit("no complete steps in the trace")
    k = len(steps[0])
    print(f"{len(steps)} steps x {k} kernels")
    tot_d = tot_g = 0.0
    for i in range(k):
        d = st.median((s[i][1] - s[i][0]) / 1e3 for s in steps)
        g = st.median((s[i][0] - s[i - 1][1]) / 1e3 for s in steps) if i else 0.0
        tot_d += d
        tot_g += g
        print(f"  {steps[0][i][2]:<16s} {d:7.2f} us   gap before {g:5.2f} us")
    spans = [(s[-1][1] - s[0][0]) / 1e3 for s in steps]
    inter = [(steps[j][0][0] - steps[j - 1][-1][1]) / 1e3 for j in range(1, len(steps))]
    print(f"  sum kernels {tot_d:.2f} us, sum gaps {tot_g:.2f} us, median step span {st.median(spans):.2f} us, "
          f"median gap between steps {st.median(inter) if inter else 0:.2f} us")


if __name__ == "__main__":
    main()
