set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6e; mkdir -p $O
export TMPDIR=/tmp
P=rl-cattle-herding_amd/cattleherd
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_runtime.py -k step_n > $O/pytest_stepn.log 2>&1 || exit 1
for v in _base "" _nolicm _base "" _nolicm; do
  CH_LIB_PATH=$PWD/$P/libcattleherd$v.so timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-extras >> $O/single$v.log 2>&1 || exit 1
done
for v in "" _nolicm; do
  for w in c4 c3 c2 c5; do
    CH_LIB_PATH=$PWD/$P/libcattleherd$v.so timeout -k 10 200 python -u bench.py --workload $w --steps 2000 --warmup 200 --steps-per-launch 2000 --no-cpu-baseline --no-extras >> $O/multi_$w$v.log 2>&1 || exit 1
  done
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --steps-per-launch 20 --no-cpu-baseline --no-extras > $O/multi_driver.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $O/single_driver.log 2>&1 || exit 1
echo DONE > $O/done
