#!/bin/bash
# Throughput sweep on one GPU: envs per GPU (latency vs bytes), precision, the other BASELINE
# configs and the physics variants.  One bench.py process per line; stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-sweep}
mkdir -p "$OUT"
: > "$OUT/sweep.jsonl"
run() {
  echo "=== $*" | tee -a "$OUT/steps.log"
  timeout -k 10 240 python bench.py --no-cpu-baseline "$@" > "$OUT/last.log" 2>&1
  local rc=$?
  echo "=== rc=$rc" | tee -a "$OUT/steps.log"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/last.log"; exit $rc; fi
  tail -1 "$OUT/last.log" >> "$OUT/sweep.jsonl"
}
while read -r line; do
  [ -z "$line" ] && continue
  run $line
done <<LINES
${SWEEP:---workload c4 --steps 2000
--workload c4 --envs 16384 --steps 1000
--workload c4 --envs 65536 --steps 400
--workload c4 --envs 262144 --steps 200
--workload c4 --precision f32 --steps 2000
--workload c4 --precision f32 --envs 262144 --steps 200
--workload c2 --steps 2000
--workload c3 --steps 2000
--workload c5 --steps 1000
--workload c4 --physics dyn --steps 1000
--workload c4 --physics pyb_gnd_drag_dw --steps 1000}
LINES
echo ALL_DONE | tee -a "$OUT/steps.log"
