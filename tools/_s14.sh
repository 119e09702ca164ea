cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python tools/ktiming.py > gpurun_out/ktiming.json 2> gpurun_out/ktiming.err || { tail gpurun_out/ktiming.err; exit 1; }
echo done
