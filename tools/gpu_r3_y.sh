# Round 3 final numbers after the co-SIMD change: smoke, driver-form and default bench lines, rocprof kernel stats,
# C4/C3 policy legs, C5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3y
mkdir -p $OUT
timeout -k 10 200 python -u __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver_form.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $OUT/bench_default.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_default -o trace -- python3 bench.py --no-cpu-baseline > $OUT/trace_default.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c4_policy.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload c3 --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c3_policy.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload c5 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 || exit 1
echo ALL_DONE > $OUT/done
