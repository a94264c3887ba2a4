set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lmhead_sample.py -x -q --timeout 200 --timeout-method thread -k "pipeline or exact" > gpurun_out/r02_lms_test.log 2>&1; rc=$?; echo "tests rc=$rc" >> gpurun_out/r02_lms_test.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/probe/lmhead_sample_bench.py --T 1.0 0.0 --M 512 256 --pipes 0 3 > gpurun_out/r02_lms_bench2.json 2> gpurun_out/r02_lms_bench2.err || exit $?
timeout -k 10 300 python scripts/probe/rw_size_probe.py > gpurun_out/r02_rw_size_probe.log 2>&1
