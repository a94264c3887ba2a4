#!/bin/bash
# r05ae: candidate handling forms A/B (bit 0: publish the bar only when a lane improved; bit 1: exact E_g bound before the hash)
set -o pipefail
mkdir -p gpurun_out
AB_DEFINE=SKYRL_EVAL_FORM AB_VALUES=0,1,2,3 timeout -k 10 400 python -u scripts/probe/sampler_ab.py run > gpurun_out/r05ae_eval_form.json 2> gpurun_out/r05ae.err
