#!/bin/bash
# A/B of a variant library against the main one: kernel stats of the bench per config.
#   VARIANT=rl_ctr_prediction_amd/variants/lib_X.so CFGS="c2 c3" bash tools/ab_lib.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for CFG in ${CFGS:-c2 c3}; do
  for L in main variant; do
    if [ $L = variant ]; then export CTR_HIP_LIB=$PWD/$VARIANT; else unset CTR_HIP_LIB; fi
    OUT=gpurun_out/ab_${CFG}_$L
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
      python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline > $OUT.log 2>&1 || exit $?
    echo "$CFG $L $(tail -1 $OUT.log | cut -c1-200)"
  done
done
