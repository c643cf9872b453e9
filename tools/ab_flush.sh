#!/bin/bash
# A/B of the deferred flush: the main library vs variants (CTR_HIP_LIB), C3 and C5 shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for LIBV in "" ${VARIANTS}; do
  for A in "--steps 1" "--steps 20" "--V 40000000 --K 128 --steps 10 --reps 3"; do
    if [ -n "$LIBV" ]; then export CTR_HIP_LIB=rl_ctr_prediction_amd/variants/lib_$LIBV.so; else unset CTR_HIP_LIB; fi
    timeout -k 10 120 python3 tools/flush_bench.py $A > gpurun_out/ab.tmp 2>&1 || { cat gpurun_out/ab.tmp; exit 1; }
    echo "${LIBV:-main} $A $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.tmp').read().splitlines()[-1]); print(round(d['ms'],3), 'ms', round(d['GBps']), 'GB/s')")"
  done
done
