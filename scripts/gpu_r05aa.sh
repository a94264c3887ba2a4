#!/bin/bash
# r05aa: split-mode sampler with 512-thread workgroups (sampler_split_nt) x workgroup target
set -o pipefail
mkdir -p gpurun_out
SWEEP_NT=256,512 SWEEP_WGS=256,512,1024 SWEEP_GRAN=8192,16384 timeout -k 10 400 python -u scripts/probe/sampler_split_sweep.py > gpurun_out/r05aa_split_nt.json 2> gpurun_out/r05aa.err
