set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/phase_probe.py marl 4096 4 32 f64 4/256 2/128 2/192 1/128 8/512 > gpurun_out/r2_c5_phase.log 2>&1 && \
timeout -k 10 200 python tools/wg_trace.py marl 4096 4 32 > gpurun_out/r2_c5_trace.log 2>&1 && \
timeout -k 10 300 python tools/geom_sweep.py marl 4096 4 32 f64 > gpurun_out/r2_c5_geom.log 2>&1
