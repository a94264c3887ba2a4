cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 200 python scripts/probe/topp_debug.py > gpurun_out/dbg.log 2>&1; rc=$?; tail -40 gpurun_out/dbg.log; exit $rc
