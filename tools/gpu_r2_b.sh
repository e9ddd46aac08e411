set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r2_b2000.json 2> gpurun_out/r2_b2000.err && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r2_b20.json 2> gpurun_out/r2_b20.err
