#!/bin/bash
# Round-4 GPU session 3: the deferred / sharded / driver-loop tests after the DMA flush's
# removal, then kernel traces of the C2 / C3 step for plan v1 / v2 and the direct scatter
# (per-kernel stats in gpurun_out/r04_ab_<tag>_<cfg>.txt). Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_STOP=--maxfail=5 bash tools/gpu_tests.sh tests/test_gpu_deferred.py tests/test_gpu_sharded.py tests/test_gpu_driver_loop.py || exit 1
for CFG in c2 c3; do
  for TAG in v2 v1 direct; do
    case $TAG in v2) E="CTR_PLAN_V2=1";; v1) E="CTR_PLAN_V2=0";; direct) E="CTR_SEG_DIRECT=1";; esac
    OUT=gpurun_out/r04_ab_${TAG}_${CFG}
    rm -rf $OUT; mkdir -p $OUT
    export $E
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
      python3 bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-driver-loop > $OUT/bench.log 2>&1 || exit 1
    unset ${E%%=*}
    S=$(find $OUT -name "*kernel_stats.csv" | head -1)
    python3 tools/kstats.py $S 25 > gpurun_out/r04_ab_${TAG}_${CFG}.txt
    echo "$CFG $TAG $(tail -1 $OUT/bench.log | grep -o '"value": [0-9.]*')"
  done
done
