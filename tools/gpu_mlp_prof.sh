set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/mlp
cd $R
timeout -k 10 120 python -u tools/mlp_probe.py sweep > gpurun_out/mlp/sweep.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mlp/kt -o kt --output-format csv -- python3 tools/mlp_probe.py 100 > gpurun_out/mlp/kt.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/mlp/p1 -o p1 --output-format csv -- python3 tools/mlp_probe.py 20 > gpurun_out/mlp/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM -d gpurun_out/mlp/p2 -o p2 --output-format csv -- python3 tools/mlp_probe.py 20 > gpurun_out/mlp/p2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/mlp/p3 -o p3 --output-format csv -- python3 tools/mlp_probe.py 20 > gpurun_out/mlp/p3.log 2>&1
