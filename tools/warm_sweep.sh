#!/bin/bash
# bench.py at several (steps, warmup) pairs, one line each: steps warmup images/s ms/step graph_warmup_steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
out=gpurun_out/warm.txt
: > $out
for a in ${PAIRS:-"20:5" "20:200" "20:5" "400:5" "20:1000"}; do
  s=${a%%:*}; w=${a##*:}
  timeout -k 10 200 python bench.py --steps "$s" --warmup "$w" > gpurun_out/warm_one.log 2>&1 || exit $?
  python3 - >> $out <<PY
import json
d = json.loads([l for l in open("gpurun_out/warm_one.log") if l.startswith("{")][-1])
print(d["steps"], d["warmup"], d["value"], d["ms_per_step"], d["config"]["graph_warmup_steps"])
PY
done
cat $out
