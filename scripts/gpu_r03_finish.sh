set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_grpo_loss_fused.py "tests/test_gpu_engine.py::test_lmhead_gemm_vs_flinear_logits_and_argmax" > gpurun_out/r03_finish_tests.log 2>&1; rc=$?; tail -6 gpurun_out/r03_finish_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe/adv_leg_probe.py > gpurun_out/r03_adv_finish3.log 2>&1; rc=$?; grep "^mode" gpurun_out/r03_adv_finish3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/e2e_bench.py --steps 1 --warmup 1 > gpurun_out/r03_e2e.json 2> gpurun_out/r03_e2e.err; rc=$?; tail -c 1500 gpurun_out/r03_e2e.json; exit $rc
