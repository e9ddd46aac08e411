# The flock phase on its own with the current kernel (tools/flock_phase.py: phase masks, timing) and its
# counters at 4096 and 262144 envs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/flock_r2s
mkdir -p $OUT
for E in 4096 262144; do
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $OUT/flock_pmc_$E/a -o pmc -- python3 tools/flock_phase.py --only 13 --envs $E --launches 20 > $OUT/flock_pmc_${E}_a.log 2>&1 || exit 1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/flock_pmc_$E/b -o pmc -- python3 tools/flock_phase.py --only 13 --envs $E --launches 20 > $OUT/flock_pmc_${E}_b.log 2>&1 || exit 1
done
echo done > $OUT/done
