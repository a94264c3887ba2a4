set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests -m gpu > gpurun_out/r04h_pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/r04h_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04h_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r04h_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > gpurun_out/r04h_bench.json 2> gpurun_out/r04h_bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04h_bench.err; exit $rc; }
python -c "import json;d=json.loads(open('gpurun_out/r04h_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d.get('sampler_filtered',{}).get('top_p0.95'))"
rm -rf gpurun_out/prof
PMC=1 PMC_REGEX="logprob|grpo|ppo_loss|sample_kernel|sample_topk|sample_topp|pack|policy_train|paged_decode|lmhead_gemm" bash scripts/profile.sh > gpurun_out/r04h_profile.log 2>&1; rc=$?; tail -2 gpurun_out/r04h_profile.log; exit $rc
