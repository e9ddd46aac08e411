# Round 3, third GPU pass: GPU tests (fused actor-critic), C4 with the policy + PPO legs (fused and separate
# nets) and its kernel trace, the workgroup trace with the cow waves' final-pass stamps, and the clean
# flock-only counter record (every step-kernel launch of the counted processes is a phase-mask-13 launch).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 150 python -u tools/wg_trace.py ctde 4096 4 16 > $OUT/wg_trace_c4.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c4_policy.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload c3 --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c3_policy.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_policy -o trace -- python3 bench.py --policy --steps 50 --warmup 10 --burn-in 100 --no-cpu-baseline > $OUT/trace_policy.log 2>&1 || exit 1
# flock-only counters: a warmed-up state per size (outside gpurun_out: large), then masked-only processes
FL=$OUT/flock
mkdir -p $FL
: > $FL/times.jsonl
for E in 4096 262144; do
  timeout -k 10 200 python3 tools/flock_phase.py --envs $E --state-out /tmp/flock_state_$E.npz > $FL/state_$E.log 2>&1 || exit 1
  timeout -k 10 200 python3 tools/flock_phase.py --only 13 --envs $E --state-in /tmp/flock_state_$E.npz --launches 50 >> $FL/times.jsonl 2> $FL/time_$E.err || exit 1
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $FL/E$E/a -o pmc -- python3 tools/flock_phase.py --only 13 --envs $E --state-in /tmp/flock_state_$E.npz --launches 20 > $FL/pmc_${E}_a.log 2>&1 || exit 1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $FL/E$E/b -o pmc -- python3 tools/flock_phase.py --only 13 --envs $E --state-in /tmp/flock_state_$E.npz --launches 20 > $FL/pmc_${E}_b.log 2>&1 || exit 1
done
python3 tools/flock_pmc.py $FL --times $FL/times.jsonl --json $OUT/flock_only_pmc.json > $FL/summary.log 2>&1 || exit 1
echo ALL_DONE > $OUT/done
