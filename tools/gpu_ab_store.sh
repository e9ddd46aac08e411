set -o pipefail
# A/B of the step kernel's store cache policy: default (write-through sc1), nt (-DCH_NT_STORES), plain
# (-DCH_NO_NT_STORES).  Build the variants first:
#   cd rl-cattle-herding_amd/cattleherd && python3 -c "import _build; \
#     _build.build(extra_flags=['-DCH_NT_STORES'], out=_build.LIB.replace('.so','_nt.so')); \
#     _build.build(extra_flags=['-DCH_NO_NT_STORES'], out=_build.LIB.replace('.so','_plain.so'))"
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/ab_store.log
: > $out
for v in "" ${AB_VARIANTS:-_nt _plain}; do
  lib=rl-cattle-herding_amd/cattleherd/libcattleherd${v}.so
  [ -f $lib ] || continue
  echo "== variant '${v}'" >> $out
  CH_LIB_PATH=$PWD/$lib timeout -k 10 120 python -u tools/wg_trace.py >> $out 2>&1 || exit 1
  CH_LIB_PATH=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 1000 --warmup 100 --no-cpu-baseline >> $out 2>&1 || exit 1
done
