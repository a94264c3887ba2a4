set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/probe/rw2_probe.py > gpurun_out/r03_rw2_probe.log 2>&1 || { tail -20 gpurun_out/r03_rw2_probe.log; exit 1; }
cat gpurun_out/r03_rw2_probe.log
for v in "" NOSTATS NOMATH; do
  timeout -k 10 200 python -u scripts/probe/phase_probe_deferred.py $v > gpurun_out/r03_phase_deferred_$v.log 2>&1 || { tail -20 gpurun_out/r03_phase_deferred_$v.log; exit 1; }
  echo "== $v"; tail -3 gpurun_out/r03_phase_deferred_$v.log
done
