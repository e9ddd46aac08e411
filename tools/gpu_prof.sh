#!/bin/bash
# Counter collection for the step kernel: one rocprofv3 --pmc pass per counter group (no tracing
# domains combined), then tools/parse_pmc.py.  Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
export TMPDIR=/tmp
WORK="python bench.py --steps ${STEPS:-60} --warmup 200 --no-cpu-baseline ${BENCH_ARGS:-}"
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
python tools/parse_pmc.py "$OUT" --json "$OUT/traffic.json" --workload "${WORKLOAD:-c4}" --dtype "${DTYPE:-f64}" > "$OUT/pmc_summary.txt"
echo ALL_DONE | tee -a "$OUT/steps.log"
