#!/bin/bash
# Counter collection: one rocprofv3 --pmc pass per counter group (no tracing domains combined).
# Stops at the first crash/timeout; an unknown counter (rc 1) just skips that group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
WORK="python bench.py --steps ${STEPS:-40} --warmup 10 --no-cpu-baseline ${BENCH_ARGS:-}"
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  echo "=== pmc$i: $group" | tee -a "$OUT/steps.log"
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d "$OUT/pmc$i" -o pmc -- $WORK > "$OUT/pmc$i.log" 2>&1
  rc=$?
  echo "=== pmc$i rc=$rc" | tee -a "$OUT/steps.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done < "${GROUPS_FILE:-tools/pmc_groups.txt}"
echo ALL_DONE | tee -a "$OUT/steps.log"
