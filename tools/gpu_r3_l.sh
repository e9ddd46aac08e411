# multi-segment MLP launches in the rollout collection: policy/rollout tests, C4/C3 policy benches (+ NW8 A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3l
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_policy.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c4_policy.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload c3 --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c3_policy.log 2>&1 || exit 1
CH_ROLLOUT_STORE_KERNEL=1 timeout -k 10 300 python3 bench.py --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c4_policy_storekernel.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_policy -o trace -- python3 bench.py --policy --steps 50 --warmup 10 --burn-in 100 --no-cpu-baseline > $OUT/trace_policy.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_adapters.py tests/test_gpu_eval.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_adapters.log 2>&1 || exit 1
