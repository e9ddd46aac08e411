set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/ -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r2_pytest_j.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r2_c4_bench.json 2>&1
