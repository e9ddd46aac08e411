# round 6: the ch_step_n headline -- tests, benches, counter records (single and multi), rocprof, flock roofline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6f; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name" >> $O/steps.log; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $O/steps.log; return $rc; }
step pytest_stepn 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_runtime.py -k step_n || exit 1
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
step smoke 300 python -u __graft_entry__.py smoke || exit 1
step bench_driver 300 python -u bench.py --steps 20 --warmup 5 || exit 1
step bench 400 python -u bench.py || exit 1
step counters 900 python -u tools/counter_record.py --workloads c4 c5 --out $O/counters --raw $O/counters_raw || exit 1
step counters_multi 900 python -u tools/counter_record.py --workloads c4 c5 --multi 20 --out $O/counters --raw $O/counters_raw_multi || exit 1
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2000 --warmup 100 --no-cpu-baseline --no-extras || exit 1
step flock 900 python -u tools/flock_roofline.py --out $O/counters || exit 1
echo ALL_DONE >> $O/steps.log
