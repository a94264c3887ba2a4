#!/bin/bash
# r05z: min_p below 256 rows on the two-kernel path by default: filtered-sampler tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_sampler_topp_fast.py tests/test_gpu_sampler_topk_fast.py tests/test_gpu_edges.py tests/test_gpu_vocabs.py > gpurun_out/r05z_tests.log 2>&1
