# C3 / IPNN bench A/B: catch-up ahead off / on with grid caps
cd $GRAFT_REPO_ROOT
for c in ${CFGS:-c3}; do
for v in "CTR_CATCHUP_AHEAD=0" "CTR_CATCHUP_AHEAD=1 CTR_CATCHUP_AHEAD_BLOCKS=64" "CTR_CATCHUP_AHEAD=1 CTR_CATCHUP_AHEAD_BLOCKS=16" "CTR_CATCHUP_AHEAD=1 CTR_CATCHUP_AHEAD_BLOCKS=256"; do
env $v timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$c', '$v', round(d['value']/1e6,3), round(d['ms_per_step'],4))" || exit 1
done
done
