# sparse-plan build time per tile size (CTR_PLAN_IPT) and digit width (CTR_PLAN_BITS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for E in "CTR_PLAN_IPT=4" "CTR_PLAN_IPT=8" "CTR_PLAN_IPT=16" "CTR_PLAN_IPT=4 CTR_PLAN_BITS=11" "CTR_PLAN_IPT=8 CTR_PLAN_BITS=11"; do
  echo "$E"
  env $E timeout -k 10 120 python tools/plan_bench.py 2>&1 | grep "{" || exit 1
done
