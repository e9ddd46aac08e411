# Round-2 (second session) profiles of the current step kernel: driver-form and long benches for every
# workload, rocprofv3 kernel trace + stats and PMC passes for c4/c5 (one counter group per pass), traffic
# summaries for bench.py.  Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_r2s
mkdir -p $OUT
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_c4_driver.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/bench_c4_2000.log 2>&1 || exit 1
for wl in c5 c2 c3; do
  timeout -k 10 200 python3 bench.py --workload $wl --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/bench_$wl.log 2>&1 || exit 1
done
for wl in c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$wl -o trace -- python3 bench.py --workload $wl --steps 400 --warmup 100 --no-cpu-baseline > $OUT/trace_$wl.log 2>&1 || exit 1
  i=0
  while read -r group; do
    [ -z "$group" ] && continue
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $group --output-format csv -d $OUT/pmc_$wl/pmc$i -o pmc -- python3 bench.py --workload $wl --steps 60 --warmup 100 --no-cpu-baseline > $OUT/pmc_${wl}_$i.log 2>&1 || exit 1
  done < tools/pmc_groups.txt
  python3 tools/parse_pmc.py $OUT/pmc_$wl --json $OUT/traffic_${wl}_f64.json --workload $wl --dtype f64 > $OUT/pmc_summary_$wl.txt || exit 1
done
echo ALL_DONE > $OUT/done
