set -u
mkdir -p gpurun_out/gemm_pmc
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex lmhead_gemm --output-format csv -d gpurun_out/gemm_pmc/p1 -o run -- python3 scripts/probe/gemm_once.py 512 > gpurun_out/gemm_pmc/p1.log 2>&1; echo "p1 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT FETCH_SIZE --kernel-include-regex lmhead_gemm --output-format csv -d gpurun_out/gemm_pmc/p2 -o run -- python3 scripts/probe/gemm_once.py 512 > gpurun_out/gemm_pmc/p2.log 2>&1; echo "p2 rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gemm_pmc/t -o run -- python3 scripts/probe/gemm_once.py 512 > gpurun_out/gemm_pmc/t.log 2>&1; echo "t rc=$?"
