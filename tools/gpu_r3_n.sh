# Round 3 (second session), pass B: the driver-form bench (20 steps after the burn-in), a 2000-step C4 bench,
# rocprofv3 kernel stats of C4 / C3 / C2 / C5, and the C4 PMC traffic passes of the shipped step kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3n
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c4_driver.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/bench_c4_2000.log 2>&1 || exit 1
for wl in c4 c3 c2 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$wl -o trace -- python3 bench.py --workload $wl --steps 400 --warmup 100 --no-cpu-baseline > $OUT/trace_$wl.log 2>&1 || exit 1
done
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $group --output-format csv -d $OUT/pmc_c4/pmc$i -o pmc -- python3 bench.py --steps 60 --warmup 100 --burn-in 200 --no-cpu-baseline > $OUT/pmc_c4_$i.log 2>&1 || exit 1
done < tools/pmc_groups.txt
python3 tools/parse_pmc.py $OUT/pmc_c4 --json $OUT/traffic_c4_f64.json --workload c4 --dtype f64 > $OUT/pmc_summary_c4.txt || exit 1
echo ALL_DONE > $OUT/done
