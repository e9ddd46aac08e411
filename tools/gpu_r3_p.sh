# the 2-rank sharded HIP rollout test (tests/test_gpu_distributed.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3p
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_dist.log 2>&1 || exit 1
