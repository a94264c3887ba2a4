set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_policy_train_split.py tests/test_gpu_trainer_e2e.py tests/test_gpu_worker.py > gpurun_out/r03_ragged_tests.log 2>&1; rc=$?; tail -15 gpurun_out/r03_ragged_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/e2e_bench.py --steps 1 --warmup 1 > gpurun_out/r03_e2e2.json 2> gpurun_out/r03_e2e2.err; rc=$?; tail -c 1200 gpurun_out/r03_e2e2.json; exit $rc
