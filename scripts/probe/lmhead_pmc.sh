#!/bin/bash
# Two rocprofv3 PMC passes (FETCH_SIZE; TCC_HIT_sum + TCC_MISS_sum) over the persistent learner
# lm_head forward at T = 8192 (scripts/probe/lmhead_persist_probe.py), into gpurun_out/<tag>_pmc_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONPATH=$PWD
TAG=${1:-r06s}
for CT in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $CT | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $CT --kernel-trace --kernel-include-regex "pkernel|label_merge" --output-format csv \
    -d gpurun_out/${TAG}_pmc_$N -o run -- python3 scripts/probe/lmhead_persist_probe.py --T 8192 --variants 4 --check 0 \
    --no-chunked --rounds 1 --iters 2 > gpurun_out/${TAG}_pmc_$N.log 2>&1 || exit $?
done
