#!/bin/bash
# r05c: split-sampler rework (sc1 last-arriver merge, DPP folds, winner's raw logit carried):
# parity first, then the per-rank row-count sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/test_gpu_sampler_splits.py tests/test_gpu_parity.py tests/test_gpu_vocabs.py \
  tests/test_gpu_sampler_stats.py tests/test_gpu_sampler_topk_fast.py tests/test_gpu_sampler_topp_fast.py \
  tests/test_gpu_lmhead_sample.py tests/test_sampler_filters.py > gpurun_out/r05c_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r05c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe/sampler_rows_probe.py > gpurun_out/r05c_rows.json 2> gpurun_out/r05c_rows.err
rc=$?; cat gpurun_out/r05c_rows.json; exit $rc
