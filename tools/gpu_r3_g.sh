# Round 3, seventh GPU pass: f32 observation offsets from the f64 positions; v1/v2 f32 bit identity.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u tests/diag/f32_probe.py > $OUT/f32_probe.log 2>&1 || exit 1
AB_TAG=r3g/ab32 AB_VARIANTS="_base DEFAULT _base DEFAULT" AB_TRACE="" AB_BENCH="--steps 2000 --warmup 200 --no-cpu-baseline --precision f32" SKIP_TESTS=1 bash tools/gpu_ab.sh || exit 1
AB_TAG=r3g/ab64 AB_VARIANTS="_base DEFAULT" AB_TRACE="" AB_BENCH="--steps 2000 --warmup 200 --no-cpu-baseline" SKIP_TESTS=1 bash tools/gpu_ab.sh || exit 1
echo ALL_DONE > $OUT/done
