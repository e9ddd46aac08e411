# diagnostic: deferred truncation bootstrap vs the Python step loop (tests/diag/rollout_defer.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3o
mkdir -p $OUT
timeout -k 10 120 python -u tests/diag/rollout_defer.py 24 > $OUT/defer.log 2>&1 || exit 1
