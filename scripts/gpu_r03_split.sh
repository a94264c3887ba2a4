set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_policy_train_split.py tests/test_gpu_vocabs.py > gpurun_out/r03_split_tests.log 2>&1; rc=$?; tail -15 gpurun_out/r03_split_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/kbench.py --only fused --rounds 5 > gpurun_out/r03_kbench_split.json 2>gpurun_out/r03_kbench_split.err; rc=$?; tail -c 2500 gpurun_out/r03_kbench_split.json; exit $rc
