# sparse-plan build time per digit width (CTR_PLAN_BITS) and tile size (CTR_PLAN_IPT)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for E in "A=1" "CTR_PLAN_BITS=8" "CTR_PLAN_BITS=10" "CTR_PLAN_BITS=10 CTR_PLAN_IPT=4" "CTR_PLAN_BITS=10 CTR_PLAN_IPT=16"; do
  echo "$E"
  env $E timeout -k 10 120 python tools/plan_bench.py 2>&1 | grep "{" || exit 1
done
