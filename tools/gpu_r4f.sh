#!/bin/bash
# Round 4: the row-tiled MLP forward -- the RLlib-shaped forward alone per RT, CTDE / MARL PPO collection with RT
# forced to 1 vs the automatic choice, kernel stats of both PPO legs, the policy / rollout tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r4f
mkdir -p $OUT
export TMPDIR=/tmp
for rt in 1 2 4; do
  CH_MLP_RT=$rt timeout -k 10 120 python -u tools/mlp_marl_probe.py > $OUT/marl_probe_rt$rt.log 2>&1 || exit 1
done
echo probes >> $OUT/steps.log
CH_MLP_RT=1 timeout -k 10 300 python -u bench.py --policy --steps 100 --warmup 10 --no-cpu-baseline --no-extras > $OUT/c4_policy_rt1.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --policy --steps 100 --warmup 10 --no-cpu-baseline --no-extras > $OUT/c4_policy_auto.log 2>&1 || exit 1
echo c4 policy >> $OUT/steps.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4_policy -o run -- python3 bench.py --policy --steps 50 --warmup 5 --burn-in 100 --no-cpu-baseline --no-extras > $OUT/prof_c4_policy.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_policy -o run -- python3 bench.py --workload c5 --policy --steps 50 --warmup 5 --burn-in 100 --no-cpu-baseline --no-extras > $OUT/prof_c5_policy.log 2>&1 || exit 1
echo profiles >> $OUT/steps.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_marl_rollout.py tests/test_gpu_policy.py -q -rf --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?" >> $OUT/steps.log
echo ALL_DONE >> $OUT/steps.log
