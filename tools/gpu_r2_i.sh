set -o pipefail
cd $GRAFT_REPO_ROOT
CH_SWEEP_G=8,16 timeout -k 10 300 python tools/geom_sweep.py ctde 4096 4 16 f64 > gpurun_out/r2_geom_c4.log 2>&1 && \
CH_SWEEP_G=4,8,16,32 timeout -k 10 300 python tools/geom_sweep.py ctde 4096 2 8 f64 > gpurun_out/r2_geom_c3.log 2>&1 && \
CH_SWEEP_G=1,2,4,8 timeout -k 10 300 python tools/geom_sweep.py ctde 1024 2 8 f64 > gpurun_out/r2_geom_c2.log 2>&1
