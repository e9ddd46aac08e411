set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/wg_trace.py ctde 4096 4 16 > gpurun_out/r2_m_trace_c4.log 2>&1 && \
timeout -k 10 200 python -u tools/wg_trace.py marl 4096 4 32 > gpurun_out/r2_m_trace_c5.log 2>&1
