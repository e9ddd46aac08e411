# k_mlp2 phase clocks, single pass and 3 passes per launch (warm caches on the last)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3k
mkdir -p $OUT
timeout -k 10 120 python -u tools/mlp_probe.py trace > $OUT/trace2.log 2>&1 || exit 1
