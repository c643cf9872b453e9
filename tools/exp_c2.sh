# A/B of the plan lookahead depth on the C2 / C3 benches (graph-replayed steps)
cd $GRAFT_REPO_ROOT
for c in ${CFGS:-c2 c3}; do
for la in 2 1 0; do
timeout -k 10 200 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline --lookahead $la 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$c', 'lookahead $la', d['value']/1e6, d['ms_per_step'])" || exit 1
done
done
