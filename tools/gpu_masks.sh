set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/masks.log
for m in 0 8 2 10; do
  echo "== mask $m" >> gpurun_out/masks.log
  CH_PHASE_MASK=$m timeout -k 10 200 python -u tools/wg_trace.py ctde 4096 4 16 >> gpurun_out/masks.log 2>&1 || exit 1
done
