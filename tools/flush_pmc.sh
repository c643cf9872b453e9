#!/bin/bash
# VALU / wait / HBM counters of the deferred flush (tools/flush_bench.py) at 1 and 20
# replayed steps: one rocprofv3 --pmc pass per counter set (never combined with tracing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/flush_pmc
mkdir -p $OUT
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  for S in 1 20; do
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p${i}_s$S -o run -- \
      python3 tools/flush_bench.py --steps $S --reps 2 > $OUT/p${i}_s$S.log 2>&1 || { tail -5 $OUT/p${i}_s$S.log; exit 1; }
  done
done
python3 tools/pmc_summary.py $OUT deferred_flush > $OUT/summary.txt; cat $OUT/summary.txt
