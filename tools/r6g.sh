set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6g; mkdir -p $O
export TMPDIR=/tmp
P=rl-cattle-herding_amd/cattleherd
for v in "" _m768 _unr "" _m768 _unr; do
  CH_LIB_PATH=$PWD/$P/libcattleherd$v.so timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-extras >> $O/c4$v.log 2>&1 || exit 1
done
for v in "" _m768 _unr; do
  CH_TRACE_MULTI=1 CH_LIB_PATH=$PWD/$P/libcattleherd$v.so timeout -k 10 200 python -u tools/wg_trace.py --json ctde 4096 4 16 >> $O/trace$v.log 2>&1 || exit 1
done
for v in "" _unr; do
  for w in c5 c3; do
    CH_LIB_PATH=$PWD/$P/libcattleherd$v.so timeout -k 10 200 python -u bench.py --workload $w --steps 2000 --warmup 200 --no-cpu-baseline --no-extras >> $O/${w}$v.log 2>&1 || exit 1
  done
done
echo DONE > $O/done
