#!/bin/bash
# C5 (MARL 4 x 32, per-wave env tables) workgroup traces: random steady state and synchronised flocking
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 150 python -u tools/wg_trace.py marl 4096 4 32 > $OUT/c5_trace_rand.log 2>&1 || exit 1
CH_TRACE_NOBURN=1 timeout -k 10 150 python -u tools/wg_trace.py marl 4096 4 32 > $OUT/c5_trace_sync.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python3 bench.py --workload c5 --steps 1000 --warmup 100 --no-cpu-baseline --no-extras > $OUT/prof_c5.log 2>&1 || exit 1
echo ALL_DONE >> $OUT/steps.log
