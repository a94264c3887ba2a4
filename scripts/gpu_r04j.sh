set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests -m gpu > gpurun_out/r04j_pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/r04j_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04j_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r04j_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/probe/topp_probe.py > gpurun_out/r04j_topp_probe.json 2>/dev/null; rc=$?; tail -c 300 gpurun_out/r04j_topp_probe.json; exit $rc
