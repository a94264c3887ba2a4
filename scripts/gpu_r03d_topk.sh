set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampler_topk_fast.py tests/test_sampler_filters.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03d_topk_tests.log 2>&1; rc=$?
tail -25 gpurun_out/r03d_topk_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/probe/sampler_filtered_leg.py > gpurun_out/r03d_topk_leg.json 2>&1; rc=$?
cat gpurun_out/r03d_topk_leg.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r03d_topk_prof -o run -- python scripts/probe/sampler_filtered_leg.py > gpurun_out/r03d_topk_prof.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -5 gpurun_out/r03d_topk_prof.log; exit $rc; }
find gpurun_out/r03d_topk_prof -name '*kernel_stats.csv' | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -12'
timeout -k 10 400 python -u -m pytest tests/test_gpu_vocabs.py tests/test_gpu_parity.py -x -q -k "sampl" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03d_sampler_suites.log 2>&1; rc=$?
tail -4 gpurun_out/r03d_sampler_suites.log; exit $rc
