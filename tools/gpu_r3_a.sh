# Round 3, first GPU pass: the GPU tests (new: configs[2] full size + training leg, MARL vec env, Monitor
# episode info, obs-buffer tags, error-word clear), smoke, the driver-form bench, configs[2] with the policy
# and PPO legs, configs[4] through the batched multi-agent surface, kernel traces of C2/C3/C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c4_driver.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload c3 --policy --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c3_policy.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload c5 --marl-vec --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c5_marlvec.log 2>&1 || exit 1
for wl in c4 c3 c2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$wl -o trace -- python3 bench.py --workload $wl --steps 400 --warmup 100 --no-cpu-baseline > $OUT/trace_$wl.log 2>&1 || exit 1
done
echo ALL_DONE > $OUT/done
