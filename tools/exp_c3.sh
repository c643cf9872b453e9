# C3 / IPNN bench A/B: plan lookahead on/off, alternating, 3 repetitions
cd $GRAFT_REPO_ROOT
for c in ${CFGS:-c3}; do
for rep in 1 2 3; do
for la in 0 1; do
CTR_PLAN_LOOKAHEAD=$la timeout -k 10 200 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$c', 'CTR_PLAN_LOOKAHEAD=$la', round(d['value']/1e6,3), round(d['ms_per_step'],4))" || exit 1
done
done
done
