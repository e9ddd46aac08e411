set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6c
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6c/pytest.log 2>&1 || exit 1
for cfg in "ctde 4096 4 16" "ctde 4096 2 8" "ctde 1024 2 8" "marl 4096 4 32"; do
  CH_TRACE_SLOTS=1 timeout -k 10 120 python -u tools/wg_trace.py $cfg >> gpurun_out/r6c/trace.log 2>&1 || exit 1
done
echo DONE >> gpurun_out/r6c/trace.log
