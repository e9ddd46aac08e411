#!/bin/bash
# One GPU session over the committed tree, in steps chained so that the first crash / timeout ends it:
#   TAG=r4a STEPS="tests smoke bench_driver bench counters rocprof" tools/gpu_run.sh
# tests: pytest -m gpu (PYTEST_ARGS to select); smoke; bench_driver: the driver's 20-step form; bench: the default
# line; counters: tools/counter_record.py (COUNTER_WORKLOADS) into gpurun_out/$TAG/counters; rocprof: kernel stats of
# a default bench run; flock: tools/flock_roofline.py; extra: $EXTRA_CMD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >> "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> "$OUT/steps.log"
  return $rc
}
for s in ${STEPS:-tests smoke bench}; do
  case $s in
    tests) step pytest_gpu ${TEST_TIMEOUT:-1100} python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
           rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    smoke) step smoke 300 python -u __graft_entry__.py smoke || exit 1 ;;
    bench_driver) step bench_driver 400 python -u bench.py --steps 20 --warmup 5 || exit 1 ;;
    bench) step bench 400 python -u bench.py ${BENCH_ARGS:-} || exit 1 ;;
    counters) step counters 900 python -u tools/counter_record.py --workloads ${COUNTER_WORKLOADS:-c4 c5} --out $OUT/counters --raw $OUT/counters_raw || exit 1 ;;
    rocprof) step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} || exit 1 ;;
    flock) step flock 900 python -u tools/flock_roofline.py --out $OUT/counters || exit 1 ;;
    extra) step extra ${EXTRA_TIMEOUT:-600} bash -c "${EXTRA_CMD}" || exit 1 ;;
  esac
done
echo ALL_DONE >> "$OUT/steps.log"
