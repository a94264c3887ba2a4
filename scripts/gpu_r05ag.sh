#!/bin/bash
# r05ag: bar published only on improvement in top_p pass 2 (pieces) and the in-row min_p pass 2: A/B, then the filtered-sampler tests
set -o pipefail
mkdir -p gpurun_out
AB_DEFINE=SKYRL_TP2_BAR_FORM AB_VALUES=0,1 timeout -k 10 300 python -u scripts/probe/sampler_ab.py run > gpurun_out/r05ag_tp2_bar_form.json 2> gpurun_out/r05ag.err &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_sampler_topp_fast.py tests/test_gpu_sampler_topk_fast.py tests/test_gpu_edges.py tests/test_gpu_vocabs.py > gpurun_out/r05ag_tests.log 2>&1
