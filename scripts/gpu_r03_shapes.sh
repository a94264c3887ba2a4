#!/bin/bash
# split training kernel shapes: parity first, then the vocabulary x shape sweep and the bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_policy_train_split.py tests/test_gpu_vocabs.py tests/test_gpu_trainer_e2e.py tests/test_gpu_gpt2_grpo.py \
    > gpurun_out/shape_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/kbench.py --only fused_vocab --rounds 5 > gpurun_out/shape_sweep3.json 2> gpurun_out/shape_sweep3.err && \
timeout -k 10 400 python -u bench.py > gpurun_out/shape_bench.json 2> gpurun_out/shape_bench.err
