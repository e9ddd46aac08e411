set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "bit_identical or vs_oracle or step_vs" > gpurun_out/r2_pw_pytest.log 2>&1 && \
timeout -k 10 200 python tools/phase_probe.py marl 4096 4 32 f64 16/512 8/512 8/256 > gpurun_out/r2_c5_phase_pw.log 2>&1 && \
timeout -k 10 200 python tools/wg_trace.py marl 4096 4 32 > gpurun_out/r2_c5_trace_pw.log 2>&1 && \
timeout -k 10 200 python bench.py --workload c5 --no-cpu-baseline --steps 1000 --warmup 100 > gpurun_out/r2_c5_bench.json 2>&1
