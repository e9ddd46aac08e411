# Round 3 closing check on the committed tree: the GPU suite, smoke, a synchronised-flocking workgroup trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3w
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || exit 1
CH_TRACE_NOBURN=1 timeout -k 10 150 python -u tools/wg_trace.py ctde 4096 4 16 > $OUT/wg_trace_sync.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_driver_form.log 2>&1 || exit 1
echo ALL_DONE > $OUT/done
