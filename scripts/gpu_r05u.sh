#!/bin/bash
# r05u: top_p pass 2 with per-piece tie lists: the top_p suite + the probe
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_sampler_topp_fast.py > gpurun_out/r05u_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05u_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/probe/topp_probe.py > gpurun_out/r05u_topp_probe.json 2>&1
rc=$?; tail -c 1500 gpurun_out/r05u_topp_probe.json; echo; [ $rc -eq 0 ] || exit $rc
