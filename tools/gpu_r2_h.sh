set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_runtime.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r2_pytest_h.log 2>&1 && \
timeout -k 10 200 python tools/wg_trace.py ctde 4096 4 16 > gpurun_out/r2_c4_trace_h.log 2>&1 && \
timeout -k 10 200 python bench.py --workload c5 --no-cpu-baseline --steps 1000 --warmup 100 > gpurun_out/r2_c5_bench.json 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r2_c4_bench.json 2>&1
