set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_runtime.py -k step_n > $O/pytest_stepn.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_runtime.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $O/bench_single.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 200 --steps-per-launch 2000 --no-cpu-baseline --no-extras > $O/bench_multi.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --steps-per-launch 20 --no-cpu-baseline --no-extras > $O/bench_multi_driver.log 2>&1 || exit 1
for w in c2 c3 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 2000 --warmup 200 --steps-per-launch 2000 --no-cpu-baseline --no-extras > $O/bench_multi_$w.log 2>&1 || exit 1
done
echo DONE > $O/done
