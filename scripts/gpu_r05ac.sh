#!/bin/bash
# r05ac: split sampler tests with the 512-thread split workgroups
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sampler_splits.py > gpurun_out/r05ac_tests.log 2>&1
