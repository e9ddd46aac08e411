set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r2_n.log
for m in 0 128 384; do
  echo "== mask $m" >> gpurun_out/r2_n.log
  CH_PHASE_MASK=$m timeout -k 10 200 python -u tools/wg_trace.py ctde 4096 4 16 >> gpurun_out/r2_n.log 2>&1 || exit 1
  CH_PHASE_MASK=$m timeout -k 10 200 python -u tools/wg_trace.py marl 4096 4 32 >> gpurun_out/r2_n.log 2>&1 || exit 1
done
