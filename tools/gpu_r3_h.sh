# Round 3 (second session), first GPU pass: k_mlp2 (weights streamed from global into the MFMA operand layout):
# policy / rollout / adapter tests, then the C4 and C3 policy + PPO legs, and their rocprof kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3h
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_rollout.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_policy.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c4_policy.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload c3 --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c3_policy.log 2>&1 || exit 1
CH_MLP_V1=1 CH_ROLLOUT_COPY=1 timeout -k 10 300 python3 bench.py --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c4_policy_v1.log 2>&1 || exit 1
CH_ROLLOUT_COPY=1 timeout -k 10 300 python3 bench.py --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c4_policy_copy.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_policy -o trace -- python3 bench.py --policy --steps 50 --warmup 10 --burn-in 100 --no-cpu-baseline > $OUT/trace_policy.log 2>&1 || exit 1
echo ALL_DONE > $OUT/done
