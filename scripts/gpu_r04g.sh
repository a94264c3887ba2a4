set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py > gpurun_out/r04g_bench.json 2> gpurun_out/r04g_bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r04g_bench.err; exit $rc; }
python -c "import json;d=json.loads(open('gpurun_out/r04g_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],d.get('sampler_filtered',{}).get('top_p0.95'))"
rm -rf gpurun_out/prof
PMC=1 PMC_REGEX="logprob|grpo|ppo_loss|sample_kernel|sample_topk|sample_topp|pack|policy_train|paged_decode|lmhead_gemm" bash scripts/profile.sh > gpurun_out/r04g_profile.log 2>&1; rc=$?; tail -3 gpurun_out/r04g_profile.log; exit $rc
