set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.err; rc=$?
echo "bench rc=$rc"; tail -c 1500 gpurun_out/r03c_bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/r03c_bench.err; exit $rc; }
PMC=1 bash scripts/profile.sh > gpurun_out/r03c_profile.log 2>&1; rc=$?; tail -5 gpurun_out/r03c_profile.log; exit $rc
