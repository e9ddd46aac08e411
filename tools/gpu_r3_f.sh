# Round 3, sixth GPU pass: f32 mode with f64 positions / centroids / prev_cent (StepParams::pos64).
# GPU tests on the new library, then f64 and f32 benches of the committed kernel (_base) and the new one.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
AB_TAG=r3f/ab64 AB_VARIANTS="_base DEFAULT _base DEFAULT" AB_TRACE="" AB_BENCH="--steps 2000 --warmup 200 --no-cpu-baseline" SKIP_TESTS=1 bash tools/gpu_ab.sh || exit 1
AB_TAG=r3f/ab32 AB_VARIANTS="_base DEFAULT _base DEFAULT" AB_TRACE="" AB_BENCH="--steps 2000 --warmup 200 --no-cpu-baseline --precision f32" SKIP_TESTS=1 bash tools/gpu_ab.sh || exit 1
timeout -k 10 300 python -u tests/diag/f32_probe.py > $OUT/f32_probe.log 2>&1 || exit 1
echo ALL_DONE > $OUT/done
