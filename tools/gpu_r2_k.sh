set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_seeded.py tests/test_gpu_eval.py tests/test_gpu_runtime.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r2_pytest_k.log 2>&1
