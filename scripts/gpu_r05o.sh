#!/bin/bash
# r05o: a fresh PMC of the lm_head MFMA GEMM at T = 8192 (VERDICT r04 item 3's first step)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05o
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05o/trace -o run -- python3 scripts/probe/gemm_once.py 8192 > gpurun_out/r05o/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex lmhead_gemm --output-format csv -d gpurun_out/r05o/pmc_sq -o run -- python3 scripts/probe/gemm_once.py 8192 > gpurun_out/r05o/pmc_sq.log 2>&1
rc=$?; echo "pmc sq rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex lmhead_gemm --output-format csv -d gpurun_out/r05o/pmc_fetch -o run -- python3 scripts/probe/gemm_once.py 8192 > gpurun_out/r05o/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
PYTHONPATH=. timeout -k 10 200 python3 scripts/probe/lmhead_bench.py --T 8192 > gpurun_out/r05o/lmhead_bench.json 2>&1
rc=$?; tail -5 gpurun_out/r05o/lmhead_bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/probe/sampler_seed.py run > gpurun_out/r05o/sampler_seed.json 2>&1
rc=$?; tail -1 gpurun_out/r05o/sampler_seed.json; [ $rc -eq 0 ] || exit $rc
