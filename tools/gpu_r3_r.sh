# the driver-form bench (timed region = the K steps only) twice, and its 2000-step form
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3r
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_c4_driver.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_c4_driver2.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 2000 --warmup 200 --no-cpu-baseline > $OUT/bench_c4_2000.log 2>&1 || exit 1
