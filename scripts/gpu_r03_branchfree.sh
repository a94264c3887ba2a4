set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_grpo_loss_fused.py tests/test_gpu_parity.py tests/test_gpu_e2e.py > gpurun_out/r03_bf_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r03_bf_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe/adv_leg_probe.py > gpurun_out/r03_adv_bf.log 2>&1; rc=$?; grep "^mode" gpurun_out/r03_adv_bf.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/probe/phase_probe_deferred.py > gpurun_out/r03_phase_bf.log 2>&1; rc=$?; tail -2 gpurun_out/r03_phase_bf.log; exit $rc
