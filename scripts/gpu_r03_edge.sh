#!/bin/bash
# EDGE (misaligned-row) form of the split training kernel: parity tests, then GPT-2 timing
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_policy_train_split.py tests/test_gpu_vocabs.py tests/test_gpu_gpt2_grpo.py tests/test_gpu_trainer_e2e.py \
    > gpurun_out/edge_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/kbench.py --only fused_gpt2,fused --rounds 5 > gpurun_out/edge_kbench.json 2> gpurun_out/edge_kbench.err
