# The driver's short bench form (--steps 20 --warmup 5) with one host launch per step vs whole-rollout HIP
# graph replays, three runs each, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/graph_ab.log
: > $out
for i in 1 2 3; do
  for g in 0 20 10; do
    echo "== graph $g run $i" >> $out
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph $g >> $out 2>&1 || exit 1
  done
done
