#!/bin/bash
# r05w: T = 1 through MODE 3 (multiplicative bound on the lse exponentials) vs MODE 1 (additive bound)
set -o pipefail
mkdir -p gpurun_out
AB_DEFINE=SKYRL_T1_MODE AB_VALUES=3,1 timeout -k 10 300 python -u scripts/probe/sampler_ab.py run > gpurun_out/r05w_t1mode_ab.json 2> gpurun_out/r05w.err
