#!/bin/bash
# Round-4 A/B: streamed full pass (C4: _base vs default), batched per-wave cheap pass (C5: _nob vs default), the
# row-tiled MLP for the RLlib nets (C5 PPO: CH_MLP_RT=1 vs default), then the GPU suite on the default library.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4e
mkdir -p $OUT
export TMPDIR=/tmp
L=$PWD/rl-cattle-herding_amd/cattleherd
for v in _base ""; do
  tag=${v:-default}
  CH_LIB_PATH=$L/libcattleherd$v.so timeout -k 10 150 python -u tools/wg_trace.py --json ctde 4096 4 16 > $OUT/c4_trace_rand_$tag.log 2>&1 || exit 1
  CH_LIB_PATH=$L/libcattleherd$v.so CH_TRACE_NOBURN=1 timeout -k 10 150 python -u tools/wg_trace.py --json ctde 4096 4 16 > $OUT/c4_trace_sync_$tag.log 2>&1 || exit 1
  CH_LIB_PATH=$L/libcattleherd$v.so timeout -k 10 200 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-extras > $OUT/c4_bench_$tag.log 2>&1 || exit 1
  CH_LIB_PATH=$L/libcattleherd$v.so timeout -k 10 300 python -u bench.py --policy --steps 100 --warmup 10 --no-cpu-baseline --no-extras > $OUT/c4_policy_$tag.log 2>&1 || exit 1
  echo "c4 $tag done" >> $OUT/steps.log
done
for v in _nob ""; do
  tag=${v:-default}
  CH_LIB_PATH=$L/libcattleherd$v.so timeout -k 10 200 python -u bench.py --workload c5 --steps 1000 --warmup 100 --no-cpu-baseline --no-extras > $OUT/c5_bench_$tag.log 2>&1 || exit 1
  echo "c5 $tag done" >> $OUT/steps.log
done
CH_MLP_RT=1 timeout -k 10 300 python -u bench.py --workload c5 --policy --steps 100 --warmup 10 --no-cpu-baseline --no-extras > $OUT/c5_policy_rt1.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --policy --steps 100 --warmup 10 --no-cpu-baseline --no-extras > $OUT/c5_policy_default.log 2>&1 || exit 1
echo "c5 policy done" >> $OUT/steps.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/steps.log
echo ALL_DONE >> $OUT/steps.log
