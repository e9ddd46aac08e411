# Round-2 profiles: rocprofv3 kernel trace + stats of bench.py (c4, c5), PMC passes per counter group,
# the flock phase on its own (timing + counters).  Each GPU step has its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_r2
mkdir -p $OUT
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
timeout -k 10 400 python3 tools/flock_phase.py > $OUT/flock_phase.jsonl 2>&1 || exit 1
for E in 4096 262144; do
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $OUT/flock_pmc_$E -o pmc -- python3 tools/flock_phase.py --only 13 --envs $E --launches 20 > $OUT/flock_pmc_$E.log 2>&1 || exit 1
done
echo ALL_DONE
