#!/bin/bash
# r05ad: T = 1 cost split: the bound test kept live (asm use) but no candidate evaluated (timing only, tokens differ)
set -o pipefail
mkdir -p gpurun_out
AB_DEFINE=SKYRL_SV_NOCAND_LIVE AB_VALUES=0,1 timeout -k 10 300 python -u scripts/probe/sampler_ab.py run > gpurun_out/r05ad_nocand_live.json 2> gpurun_out/r05ad.err
