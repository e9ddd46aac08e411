# pipelined halves in the PPO collection: policy/rollout tests, C4/C3 policy benches against one chain
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3u
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_policy.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_policy.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c4_policy.log 2>&1 || exit 1
CH_ROLLOUT_SPLIT=0 timeout -k 10 300 python3 bench.py --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c4_policy_onechain.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload c3 --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c3_policy.log 2>&1 || exit 1
CH_ROLLOUT_SPLIT=0 timeout -k 10 300 python3 bench.py --workload c3 --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c3_policy_onechain.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_policy -o trace -- python3 bench.py --policy --steps 50 --warmup 10 --burn-in 100 --no-cpu-baseline > $OUT/trace_policy.log 2>&1 || exit 1
echo ALL_DONE > $OUT/done
