#!/bin/bash
# r05r: sampler A/B of the seeding barrier
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_DEFINE=SKYRL_SEED_BARRIER timeout -k 10 200 python -u scripts/probe/sampler_ab.py run > gpurun_out/r05r_ab_seedbar.json 2>&1
rc=$?; tail -1 gpurun_out/r05r_ab_seedbar.json; [ $rc -eq 0 ] || exit $rc
