set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r4c
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_marl_rollout.py -v -rf --timeout 200 --timeout-method thread > $OUT/pytest_marl_rollout.log 2>&1
echo "pytest rc=$?" >> $OUT/steps.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_policy -o run -- python3 bench.py --workload c5 --policy --steps 100 --warmup 10 --no-cpu-baseline --no-extras > $OUT/bench_c5_policy.log 2>&1 || exit 1
echo "c5 policy done" >> $OUT/steps.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4_policy -o run -- python3 bench.py --workload c4 --policy --steps 100 --warmup 10 --no-cpu-baseline --no-extras > $OUT/bench_c4_policy.log 2>&1 || exit 1
echo "c4 policy done" >> $OUT/steps.log
timeout -k 10 600 python -u tools/flock_roofline.py --out $OUT/counters > $OUT/flock_roofline.log 2>&1 || exit 1
echo ALL_DONE >> $OUT/steps.log
