set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r2_pytest1.log 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2_b20.json 2> gpurun_out/r2_b20.err && \
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r2_b2000.json 2> gpurun_out/r2_b2000.err
