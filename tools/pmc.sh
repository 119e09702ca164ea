#!/bin/bash
# rocprofv3 PMC counter passes over the eager (non-graph) fused CNN step, one pass per counter group
# (rocprofv3 does not split counters over passes; each pass stays inside the per-block limits:
# <= 8 SQ, <= 4 TCC (FETCH_SIZE = 3, WRITE_SIZE = 2), <= 2 GRBM).  Output: gpurun_out/pmc/<pass>/.
# usage: tools/pmc.sh [args for bench.py]      (tools/pmc_summary.py turns it into a table)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS=${*:---steps 20 --warmup 5 --no-graph}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1 || true
pass() {
  local name=$1; shift
  rm -rf "gpurun_out/pmc/$name"
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "gpurun_out/pmc/$name" -o run -- \
    python3 bench.py $ARGS > "gpurun_out/pmc/$name.log" 2>&1
  local rc=$?
  echo "[pmc $name] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
PASSES=${PMC_PASSES:-sq fetch write}
for p in $PASSES; do
  case $p in
    sq) pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE ;;
    issue) pass issue SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU ;;
    fetch) pass fetch FETCH_SIZE ;;
    write) pass write WRITE_SIZE ;;
  esac
done
echo "pmc done"
exit 0
