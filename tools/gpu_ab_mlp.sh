set -o pipefail
# A/B of the policy-forward kernel: default build vs variants (CH_LIB_PATH), bench.py --policy
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/ab_mlp.log
: > $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_policy.py tests/test_gpu_rollout.py >> $out 2>&1 || exit 1
for v in "" ${AB_VARIANTS:-_d2}; do
  lib=rl-cattle-herding_amd/cattleherd/libcattleherd${v}.so
  [ -f $lib ] || continue
  echo "== variant '${v}'" >> $out
  CH_LIB_PATH=$PWD/$lib timeout -k 10 100 python -u tools/mlp_probe.py sweep >> $out 2>&1 || exit 1
  CH_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u bench.py --steps 300 --warmup 50 --policy --no-cpu-baseline >> $out 2>&1 || exit 1
done
