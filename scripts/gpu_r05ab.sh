#!/bin/bash
# r05ab: MODE 3 candidate evaluation deferred to the end of each iteration (one ballot, one bar raise) A/B
set -o pipefail
mkdir -p gpurun_out
AB_DEFINE=SKYRL_DEFER_EVAL AB_VALUES=0,1 timeout -k 10 300 python -u scripts/probe/sampler_ab.py run > gpurun_out/r05ab_defer_eval.json 2> gpurun_out/r05ab.err
