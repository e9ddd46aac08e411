#!/bin/bash
# A/B of step-kernel builds on one box: for each library variant (libcattleherd${v}.so) a workgroup trace
# and a bench run; then, unless SKIP_TESTS=1, the GPU parity tests on the default library.
#   AB_VARIANTS="_base ''" AB_TRACE="ctde 4096 4 16" AB_BENCH="--steps 1000 --warmup 100"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/${AB_TAG:-ab}.log
: > $out
export TMPDIR=/tmp
for v in ${AB_VARIANTS:-_base DEFAULT}; do
  [ "$v" = DEFAULT ] && v=""
  lib=rl-cattle-herding_amd/cattleherd/libcattleherd${v}.so
  [ -f $lib ] || { echo "missing $lib" >> $out; continue; }
  echo "== variant '${v}'" >> $out
  if [ -n "${AB_TRACE-ctde 4096 4 16}" ]; then
    CH_LIB_PATH=$PWD/$lib timeout -k 10 150 python -u tools/wg_trace.py ${AB_TRACE:-ctde 4096 4 16} >> $out 2>&1 || exit 1
  fi
  CH_LIB_PATH=$PWD/$lib timeout -k 10 150 python -u bench.py ${AB_BENCH:---steps 1000 --warmup 100 --no-cpu-baseline} >> $out 2>&1 || exit 1
done
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${AB_TAG:-ab}_pytest.log 2>&1
  echo "pytest rc=$?" >> $out
  tail -3 gpurun_out/${AB_TAG:-ab}_pytest.log >> $out
fi
echo AB_DONE >> $out
