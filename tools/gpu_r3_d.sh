# Round 3, fourth GPU pass: the late-mode observation segments + early Euler math (default build) against the
# round-start kernel (_base): tests, A/B benches in both orders, the new kernel's workgroup trace, its PMC traffic
# at C4, its rocprof kernel stats, and the policy / PPO legs (8-wave 256-wide MLP kernel, posts folded).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
AB_TAG=r3d/ab AB_VARIANTS="_base DEFAULT" AB_TRACE="" AB_BENCH="--steps 2000 --warmup 200 --no-cpu-baseline" SKIP_TESTS=1 bash tools/gpu_ab.sh || exit 1
AB_TAG=r3d/ab2 AB_VARIANTS="DEFAULT _base" AB_TRACE="" AB_BENCH="--steps 2000 --warmup 200 --no-cpu-baseline" SKIP_TESTS=1 bash tools/gpu_ab.sh || exit 1
timeout -k 10 150 python -u tools/wg_trace.py ctde 4096 4 16 > $OUT/wg_trace_c4.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c4_policy.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c4 -o trace -- python3 bench.py --steps 400 --warmup 100 --no-cpu-baseline > $OUT/trace_c4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_policy -o trace -- python3 bench.py --policy --steps 50 --warmup 10 --burn-in 100 --no-cpu-baseline > $OUT/trace_policy.log 2>&1 || exit 1
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $group --output-format csv -d $OUT/pmc_c4/pmc$i -o pmc -- python3 bench.py --steps 60 --warmup 100 --burn-in 200 --no-cpu-baseline > $OUT/pmc_c4_$i.log 2>&1 || exit 1
done < tools/pmc_groups.txt
python3 tools/parse_pmc.py $OUT/pmc_c4 --json $OUT/traffic_c4_f64.json --workload c4 --dtype f64 > $OUT/pmc_summary_c4.txt || exit 1
echo ALL_DONE > $OUT/done
