# Round 3, final pass on the committed tree: the whole GPU suite, smoke, the driver's default bench line, its
# rocprof kernel stats, and the policy / PPO legs at C4 and C3.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3s
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $OUT/bench_default.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_default -o trace -- python3 bench.py --no-cpu-baseline > $OUT/trace_default.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c4_policy.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload c3 --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c3_policy.log 2>&1 || exit 1
echo ALL_DONE > $OUT/done
