#!/bin/bash
# r05ah: the final sampler tree (bar published on improvement in the unfiltered race, top_p pass 1 and pass-2 pieces): sampler test files
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_sampler_topp_fast.py tests/test_gpu_sampler_topk_fast.py tests/test_gpu_edges.py tests/test_gpu_vocabs.py \
  tests/test_gpu_sampler_splits.py tests/test_gpu_parity.py tests/test_gpu_sampler_stats.py > gpurun_out/r05ah_tests.log 2>&1
