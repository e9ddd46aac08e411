# diagnostic: the env's obs buffer after a device rollout collection (tests/diag/rollout_last_obs.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3i
mkdir -p $OUT
timeout -k 10 120 python -u tests/diag/rollout_last_obs.py 5 > $OUT/diag.log 2>&1 || exit 1
CH_ROLLOUT_COPY=1 timeout -k 10 120 python -u tests/diag/rollout_last_obs.py 5 > $OUT/diag_copy.log 2>&1 || exit 1
