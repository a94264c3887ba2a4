#!/bin/bash
# r05v: split-mode sampler phase stamps at 64 / 128 rows (T = 1 vs greedy)
set -o pipefail
mkdir -p gpurun_out
ROWS=64,128 timeout -k 10 240 python -u scripts/probe/sampler_split_phase.py run > gpurun_out/r05v_split_phase.json 2> gpurun_out/r05v.err
