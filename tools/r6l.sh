# round 6 final, part 2: counter records (single and multi), rocprof, flock roofline, policy legs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6l; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name" >> $O/steps.log; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $O/steps.log; return $rc; }
step counters 500 python -u tools/counter_record.py --workloads c4 c5 --out $O/counters --raw $O/counters_raw || exit 1
step counters_multi 500 python -u tools/counter_record.py --workloads c4 c5 --multi 20 --out $O/counters --raw $O/counters_raw_multi || exit 1
step rocprof 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2000 --warmup 100 --no-cpu-baseline --no-extras || exit 1
step flock 400 python -u tools/flock_roofline.py --out $O/counters || exit 1
step bench_c5_single 300 python -u bench.py --workload c5 --steps-per-launch 1 --no-cpu-baseline --no-extras || exit 1
echo ALL_DONE >> $O/steps.log
