#!/bin/bash
# Round 4: fast tanh + packed-only wide MLP variants -- MARL forward probes per RT, PPO legs, the GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4g
mkdir -p $OUT
export TMPDIR=/tmp
for rt in 1 2 4; do
  CH_MLP_RT=$rt timeout -k 10 120 python -u tools/mlp_marl_probe.py > $OUT/marl_probe_rt$rt.log 2>&1 || exit 1
done
echo probes >> $OUT/steps.log
for rt in 2 4; do
  CH_MLP_RT=$rt timeout -k 10 300 python -u bench.py --workload c5 --policy --steps 50 --warmup 5 --burn-in 100 --no-cpu-baseline --no-extras > $OUT/c5_policy_rt$rt.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --policy --steps 100 --warmup 10 --no-cpu-baseline --no-extras > $OUT/c4_policy_auto.log 2>&1 || exit 1
CH_MLP_RT=1 timeout -k 10 300 python -u bench.py --policy --steps 100 --warmup 10 --no-cpu-baseline --no-extras > $OUT/c4_policy_rt1.log 2>&1 || exit 1
echo policy >> $OUT/steps.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/steps.log
echo ALL_DONE >> $OUT/steps.log
