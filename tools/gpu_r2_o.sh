set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CH_SWEEP_G=4,8,16 timeout -k 10 300 python -u tools/geom_sweep.py marl 4096 4 32 > gpurun_out/r2_o_geom_c5.log 2>&1 && \
CH_SWEEP_G=8,16 timeout -k 10 300 python -u tools/geom_sweep.py ctde 4096 4 16 > gpurun_out/r2_o_geom_c4.log 2>&1 && \
CH_SWEEP_G=1,2,4,8 timeout -k 10 300 python -u tools/geom_sweep.py ctde 1024 2 8 > gpurun_out/r2_o_geom_c2.log 2>&1
