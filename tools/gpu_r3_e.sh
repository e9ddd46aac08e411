# Round 3, fifth GPU pass: observation segments written by the final pass's idle lanes (default build) against
# the round-start kernel (_base): tests, A/B benches in both orders, workgroup trace, PMC write traffic at C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3e
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
AB_TAG=r3e/ab AB_VARIANTS="_base DEFAULT" AB_TRACE="" AB_BENCH="--steps 2000 --warmup 200 --no-cpu-baseline" SKIP_TESTS=1 bash tools/gpu_ab.sh || exit 1
AB_TAG=r3e/ab2 AB_VARIANTS="DEFAULT _base" AB_TRACE="" AB_BENCH="--steps 2000 --warmup 200 --no-cpu-baseline" SKIP_TESTS=1 bash tools/gpu_ab.sh || exit 1
timeout -k 10 150 python -u tools/wg_trace.py ctde 4096 4 16 > $OUT/wg_trace_c4.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_c4/$c -o pmc -- python3 bench.py --steps 60 --warmup 100 --burn-in 200 --no-cpu-baseline > $OUT/pmc_c4_$c.log 2>&1 || exit 1
done
python3 tools/parse_pmc.py $OUT/pmc_c4 --json $OUT/traffic_c4_f64.json --workload c4 --dtype f64 > $OUT/pmc_summary_c4.txt || exit 1
echo ALL_DONE > $OUT/done
