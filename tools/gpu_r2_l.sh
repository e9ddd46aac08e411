set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/r2_l_pytest.log 2>&1 && \
timeout -k 10 200 python -u tools/wg_trace.py ctde 4096 4 16 > gpurun_out/r2_l_trace.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/r2_l_bench.json 2> gpurun_out/r2_l_bench.err && \
timeout -k 10 200 python -u bench.py --workload c5 --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/r2_l_bench_c5.json 2>> gpurun_out/r2_l_bench.err
