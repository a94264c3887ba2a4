set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 200 $T -x tests/test_gpu_sampler_topp_fast.py > gpurun_out/r04f_topp.log 2>&1; rc=$?
tail -3 gpurun_out/r04f_topp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe/topp_probe.py > gpurun_out/r04f_topp_probe.json 2> gpurun_out/r04f_topp_probe.err; rc=$?
cat gpurun_out/r04f_topp_probe.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 $T tests -m gpu > gpurun_out/r04f_pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r04f_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r04f_smoke.log; exit $rc
