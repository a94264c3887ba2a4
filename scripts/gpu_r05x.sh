#!/bin/bash
# r05x: split-mode T = 1 through MODE 1: sampler GPU tests, then the split shape sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_sampler_splits.py tests/test_gpu_sampler_stats.py tests/test_gpu_vocabs.py tests/test_gpu_lmhead_sample.py > gpurun_out/r05x_tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/probe/sampler_split_sweep.py > gpurun_out/r05x_split_sweep.json 2> gpurun_out/r05x.err
