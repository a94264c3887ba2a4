set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/gpu_r04b.sh; rb=$?
echo "r04b rc=$rb"
[ $rb -eq 124 ] || [ $rb -eq 137 ] || [ $rb -eq 134 ] || [ $rb -eq 139 ] && exit $rb
rm -rf gpurun_out/r04c
bash scripts/gpu_r04c.sh > gpurun_out/r04c.log 2>&1; rc=$?
tail -8 gpurun_out/r04c.log
exit $(( rb != 0 ? rb : rc ))
