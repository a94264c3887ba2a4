set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03d_topk_prof -o run -- python3 scripts/probe/sampler_filtered_leg.py > gpurun_out/r03d_topk_prof.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -5 gpurun_out/r03d_topk_prof.log; exit $rc; }
f=$(find gpurun_out/r03d_topk_prof -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -14
