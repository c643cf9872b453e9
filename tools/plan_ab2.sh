# sparse-plan build time: next-pass histograms fused into the scatters (default) or not
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for E in "CTR_PLAN_FUSED_HIST=0" "CTR_PLAN_FUSED_HIST=1" "CTR_PLAN_FUSED_HIST=0" "CTR_PLAN_FUSED_HIST=1"; do
  echo "$E"
  env $E timeout -k 10 120 python tools/plan_bench.py 2>&1 | grep "{" || exit 1
done
