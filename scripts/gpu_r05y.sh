#!/bin/bash
# r05y: split shape sweep through step_ptr; top_p / min_p one-pass kernel vs the two-kernel path by row count
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/probe/sampler_split_sweep.py > gpurun_out/r05y_split_sweep.json 2> gpurun_out/r05y.err &&
timeout -k 10 400 python -u scripts/probe/topp_rows_probe.py > gpurun_out/r05y_topp_rows.json 2>> gpurun_out/r05y.err
