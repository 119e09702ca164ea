#!/bin/bash
# A/B bench runner for one gpurun session: each argument is one case "ENV=V ... | bench args";
# appends "<case> images/s ms/step" to gpurun_out/ab.txt, stops at the first failing run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in "$@"; do
  envs="${c%%|*}"; args="${c#*|}"
  env $envs timeout -k 10 200 python bench.py $args > gpurun_out/b_one.log 2>&1 || { echo "case failed: $c"; tail -20 gpurun_out/b_one.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/b_one.log') if l.startswith('{')][-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" "$c" >> gpurun_out/ab.txt
done
cat gpurun_out/ab.txt
