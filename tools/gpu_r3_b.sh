# Round 3, second GPU pass: A/B of the early reset decision + early Euler math (default build) against the
# previous kernel (_base) -- workgroup traces and 2000-step benches on one box -- then the GPU tests on the new
# kernel, its rocprof kernel stats at C4, and a kernel trace of the policy / PPO-collection legs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3b
mkdir -p $OUT
AB_TAG=r3b/ab AB_VARIANTS="_base DEFAULT" AB_TRACE="ctde 4096 4 16" AB_BENCH="--steps 2000 --warmup 200 --no-cpu-baseline" SKIP_TESTS=1 bash tools/gpu_ab.sh || exit 1
AB_TAG=r3b/ab2 AB_VARIANTS="DEFAULT _base" AB_TRACE="" AB_BENCH="--steps 2000 --warmup 200 --no-cpu-baseline" SKIP_TESTS=1 bash tools/gpu_ab.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c4 -o trace -- python3 bench.py --steps 400 --warmup 100 --no-cpu-baseline > $OUT/trace_c4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_policy -o trace -- python3 bench.py --policy --steps 100 --warmup 20 --no-cpu-baseline > $OUT/trace_policy.log 2>&1 || exit 1
echo ALL_DONE > $OUT/done
