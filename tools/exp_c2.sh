# C2 bench A/B: lookahead plans on one or two streams, alternating, 2 repetitions
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for ns in 1 2; do
CTR_PLAN_STREAMS=$ns timeout -k 10 200 python bench.py --config ${CFG:-c2} --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('${CFG:-c2}', 'CTR_PLAN_STREAMS=$ns', round(d['value']/1e6,3), round(d['ms_per_step'],4))" || exit 1
done
done
