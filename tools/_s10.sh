cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "" "nw2f:" "nfc2t:" "nboth:"; do
  DMLC_VARIANT="$v" timeout -k 10 120 python tools/kbench.py > gpurun_out/kbench_${v%%:*}.json 2>/dev/null || exit 1
done
echo done
