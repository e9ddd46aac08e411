#!/bin/bash
# One GPU session: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel stats.  Stops at the first
# crash / timeout (exit >= 2 or killed); plain test failures (pytest exit 1) let the bench still run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step pytest_gpu ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
step bench ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} || exit 1
if [ "${SKIP_PROF:-0}" != "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
       python bench.py --steps 300 --warmup 50 --no-cpu-baseline ${BENCH_ARGS:-} || exit 1
fi
echo ALL_DONE | tee -a "$OUT/steps.log"
