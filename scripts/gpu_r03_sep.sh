set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/probe/rw2_probe.py split > gpurun_out/r03_rw2_split.log 2>&1; rc=$?; cat gpurun_out/r03_rw2_split.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe/adv_leg_probe.py nt > gpurun_out/r03_adv_nt.log 2>&1; rc=$?; grep "^nt" gpurun_out/r03_adv_nt.log; [ $rc -eq 0 ] || { tail -20 gpurun_out/r03_adv_nt.log; exit $rc; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 360 --timeout-method thread -p no:cacheprovider tests/test_gpu_separated.py > gpurun_out/r03_separated.log 2>&1; rc=$?; tail -30 gpurun_out/r03_separated.log; exit $rc
