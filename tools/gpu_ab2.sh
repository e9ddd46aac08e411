#!/bin/bash
# A/B of step-kernel builds on one box (AB_VARIANTS: library suffixes, DEFAULT = libcattleherd.so): per variant a
# random-action workgroup trace, a synchronised-flocking trace, a C4 bench and (AB_POLICY=1) the C4 PPO leg; then the
# GPU test suite on the default library.  Output: gpurun_out/$AB_TAG/
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${AB_TAG:-ab2}
mkdir -p $OUT
export TMPDIR=/tmp
for v in ${AB_VARIANTS:-_base DEFAULT}; do
  [ "$v" = DEFAULT ] && v=""
  lib=$PWD/rl-cattle-herding_amd/cattleherd/libcattleherd${v}.so
  tag=${v:-default}
  CH_LIB_PATH=$lib timeout -k 10 150 python -u tools/wg_trace.py --json ctde 4096 4 16 > $OUT/trace_rand_$tag.log 2>&1 || exit 1
  CH_LIB_PATH=$lib CH_TRACE_NOBURN=1 timeout -k 10 150 python -u tools/wg_trace.py --json ctde 4096 4 16 > $OUT/trace_sync_$tag.log 2>&1 || exit 1
  CH_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline --no-extras ${AB_BENCH:-} > $OUT/bench_$tag.log 2>&1 || exit 1
  if [ "${AB_POLICY:-0}" = 1 ]; then
    CH_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --policy --steps 100 --warmup 10 --no-cpu-baseline --no-extras > $OUT/policy_$tag.log 2>&1 || exit 1
  fi
  echo "variant $tag done" >> $OUT/steps.log
done
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest.log 2>&1
  echo "pytest rc=$?" >> $OUT/steps.log
fi
echo AB_DONE >> $OUT/steps.log
