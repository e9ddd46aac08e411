set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/wg_trace.py marl 4096 4 32 > gpurun_out/r2_c5_trace_f0.log 2>&1 && \
CH_PHASE_MASK=2 timeout -k 10 200 python tools/wg_trace.py marl 4096 4 32 > gpurun_out/r2_c5_trace_f2.log 2>&1
