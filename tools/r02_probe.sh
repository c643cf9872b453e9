#!/bin/bash
# Round-2 probe: flush timing (VALU vs HBM), flush PMC (VALU counters), GEMM baseline table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/probe
mkdir -p $OUT
for S in 1 5 20; do
  timeout -k 10 120 python3 tools/flush_bench.py --steps $S >> $OUT/flush.jsonl 2>>$OUT/flush.err || exit $?
done
timeout -k 10 180 python3 tools/flush_bench.py --V 40000000 --K 128 --steps 10 --reps 3 >> $OUT/flush.jsonl 2>>$OUT/flush.err || exit $?
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/fpmc$i -o run -- \
    python3 tools/flush_bench.py --steps 20 --reps 2 > $OUT/fpmc$i.log 2>&1 || exit $?
done
timeout -k 10 300 python3 tools/gemm_bench.py --reps 20 --configs auto > $OUT/gemm.jsonl 2>$OUT/gemm.err || exit $?
echo done
