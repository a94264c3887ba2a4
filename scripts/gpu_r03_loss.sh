set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_grpo_loss_fused.py tests/test_gpu_parity.py > gpurun_out/r03_loss_tests.log 2>&1 || { tail -30 gpurun_out/r03_loss_tests.log; exit 1; }
tail -2 gpurun_out/r03_loss_tests.log
timeout -k 10 300 python -u scripts/probe/adv_leg_probe.py > gpurun_out/r03_adv_leg_probe5.log 2>&1 || { tail -20 gpurun_out/r03_adv_leg_probe5.log; exit 1; }
grep ^mode gpurun_out/r03_adv_leg_probe5.log
timeout -k 10 200 python -u scripts/probe/phase_probe_deferred.py > gpurun_out/r03_phase_deferred2.log 2>&1 && tail -2 gpurun_out/r03_phase_deferred2.log
