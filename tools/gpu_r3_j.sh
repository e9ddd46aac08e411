# k_mlp2 phase clocks and forward sweep (tools/mlp_probe.py), policy tests, C4 policy bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3j
mkdir -p $OUT
timeout -k 10 120 python -u tools/mlp_probe.py trace > $OUT/trace.log 2>&1 || exit 1
CH_MLP2_NW8=1 timeout -k 10 120 python -u tools/mlp_probe.py trace > $OUT/trace_nw8.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_policy.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c4_policy.log 2>&1 || exit 1
