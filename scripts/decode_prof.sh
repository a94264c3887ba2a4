set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/dprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dprof -o run -- python3 scripts/probe/decode_prof.py 512 400 > gpurun_out/dprof/log.txt 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/dprof/log.txt; find gpurun_out/dprof -name "*stats.csv"
