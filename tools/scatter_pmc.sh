#!/bin/bash
# Counters of the embedding scatter (seg_chunk + seg_combine_apply), standalone
# (tools/scatter_bench.py) and in the C3 step (bench.py), one rocprofv3 --pmc pass per
# counter set plus a kernel trace of each, then a per-kernel summary
# (tools/scatter_pmc_summary.py). Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/scatter_pmc
rm -rf $OUT; mkdir -p $OUT
CFGS=${CFGS:-c3 c5}
run() {  # $1 = tag, rest = program
  local tag=$1; shift
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${tag}_trace -o run -- "$@" \
    > $OUT/${tag}_trace.log 2>&1 || { echo "trace $tag failed"; tail -5 $OUT/${tag}_trace.log; return 1; }
  local i=0
  for P in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/${tag}_p$i -o run -- "$@" \
      > $OUT/${tag}_p$i.log 2>&1 || { echo "pmc $tag $i failed"; tail -5 $OUT/${tag}_p$i.log; return 1; }
  done
  echo "$tag ok"
}
for C in $CFGS; do
  run alone_$C python3 tools/scatter_bench.py --config $C --reps 10 || exit 1
done
run step_c3 python3 bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline --no-driver-loop || exit 1
python3 tools/scatter_pmc_summary.py $OUT | tee $OUT/summary.txt
