#!/bin/bash
# r05af: top_p kernel pass-1 bar published only on improvement: A/B, then the filtered-sampler tests
set -o pipefail
mkdir -p gpurun_out
AB_DEFINE=SKYRL_TP_BAR_FORM AB_VALUES=0,1 timeout -k 10 300 python -u scripts/probe/sampler_ab.py run > gpurun_out/r05af_tp_bar_form.json 2> gpurun_out/r05af.err &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_sampler_topp_fast.py tests/test_gpu_sampler_topk_fast.py tests/test_gpu_edges.py > gpurun_out/r05af_tests.log 2>&1
