set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04c
export TMPDIR=/tmp
for c in 2048 4096 8192 16384; do
  timeout -k 10 120 python scripts/probe/lmhead_chunk_hbm.py --chunk $c --iters 5 >> gpurun_out/r04c/times.jsonl 2>> gpurun_out/r04c/times.err || exit 1
done
cat gpurun_out/r04c/times.jsonl
for c in 2048 16384; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/r04c/pmc_${c}_$ctr -o run -- python3 scripts/probe/lmhead_chunk_hbm.py --chunk $c --iters 2 > gpurun_out/r04c/pmc_${c}_$ctr.log 2>&1 || exit 1
  done
done
echo pmc done
