set -u
mkdir -p gpurun_out/gemm_pmc2
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc VmemLatency LdsLatency --kernel-include-regex lmhead_gemm --output-format csv -d gpurun_out/gemm_pmc2/p2 -o run -- python3 scripts/probe/gemm_once.py 512 > gpurun_out/gemm_pmc2/p2.log 2>&1; echo "p2 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE --kernel-include-regex lmhead_gemm --output-format csv -d gpurun_out/gemm_pmc2/p3 -o run -- python3 scripts/probe/gemm_once.py 512 > gpurun_out/gemm_pmc2/p3.log 2>&1; echo "p3 rc=$?"
