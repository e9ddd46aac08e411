# round 6 final, part 1: tests, smoke, the driver's and the default bench, the other BASELINE configs
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6k; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 to=$2; shift 2; echo "=== $name" >> $O/steps.log; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $O/steps.log; return $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
step smoke 200 python -u __graft_entry__.py smoke || exit 1
step bench_driver 200 python -u bench.py --steps 20 --warmup 5 || exit 1
step bench 300 python -u bench.py || exit 1
step bench_c3 200 python -u bench.py --workload c3 --no-cpu-baseline || exit 1
step bench_c2 200 python -u bench.py --workload c2 --no-cpu-baseline || exit 1
step bench_c5 300 python -u bench.py --workload c5 --no-cpu-baseline || exit 1
echo ALL_DONE >> $O/steps.log
