# Instruction-fetch counters of the step kernel (one rocprofv3 --pmc pass per group).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/icache
mkdir -p $OUT
for wl in c4 c5; do
  i=0
  for group in "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" \
               "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $group --output-format csv -d $OUT/${wl}_$i -o pmc -- python3 bench.py --workload $wl --steps 100 --warmup 10 --no-cpu-baseline > $OUT/${wl}_$i.log 2>&1 || exit 1
  done
done
