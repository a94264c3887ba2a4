set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_sampler_topp_fast.py > gpurun_out/r04b_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r04b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe/topp_probe.py > gpurun_out/r04b_topp_probe.json 2> gpurun_out/r04b_topp_probe.err; rc=$?
cat gpurun_out/r04b_topp_probe.json; exit $rc
