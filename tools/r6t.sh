# A/B: phase 0 without the drone lanes' zero-inits (default) against them (CH_PHASE0_DRONE_ZERO)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6t; mkdir -p $O
step() { local name=$1 to=$2; shift 2; echo "=== $name" >> $O/steps.log; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc" >> $O/steps.log; return $rc; }
step pytest 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_runtime.py tests/test_gpu_parity.py -k "step_n or v1_v2_bit" || exit 1
for r in 1 2; do
step c4_new_$r 200 python -u bench.py --no-extras --no-cpu-baseline || exit 1
CH_LIB_PATH=$PWD/rl-cattle-herding_amd/cattleherd/libcattleherd_p0.so step c4_p0_$r 200 python -u bench.py --no-extras --no-cpu-baseline || exit 1
done
step c5_new 200 python -u bench.py --workload c5 --no-extras --no-cpu-baseline || exit 1
CH_LIB_PATH=$PWD/rl-cattle-herding_amd/cattleherd/libcattleherd_p0.so step c5_p0 200 python -u bench.py --workload c5 --no-extras --no-cpu-baseline || exit 1
step c3_new 200 python -u bench.py --workload c3 --no-extras --no-cpu-baseline || exit 1
CH_LIB_PATH=$PWD/rl-cattle-herding_amd/cattleherd/libcattleherd_p0.so step c3_p0 200 python -u bench.py --workload c3 --no-extras --no-cpu-baseline || exit 1
CH_TRACE_MULTI=1 step trace_new 200 python -u tools/wg_trace.py --json ctde 4096 4 16 || exit 1
CH_TRACE_MULTI=1 CH_LIB_PATH=$PWD/rl-cattle-herding_amd/cattleherd/libcattleherd_p0.so step trace_p0 200 python -u tools/wg_trace.py --json ctde 4096 4 16 || exit 1
echo ALL_DONE >> $O/steps.log
