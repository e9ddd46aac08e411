# PPO collection eager vs HIP-graph replay (tools/ppo_graph_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r3q
mkdir -p $OUT
timeout -k 10 200 python -u tools/ppo_graph_probe.py > $OUT/ppo_graph.log 2>&1 || exit 1
