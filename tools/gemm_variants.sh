#!/bin/bash
# GEMM tuning session on the GPU box: parity of every tiling, then the C3 shapes per tiling
# for the main library and each variant in rl_ctr_prediction_amd/variants/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider -k "gemm" > gpurun_out/tg.log 2>&1; tail -1 gpurun_out/tg.log
C=${CONFIGS:-"auto,0x1,1x1,2x1,3x1,4x1,5x1,6x1,7x1,0x9,0x16,3x4,6x9,6x8,4x2"}
timeout -k 10 300 python tools/gemm_bench.py --reps 20 --configs $C > gpurun_out/gemm_base.log 2>&1 || exit $?
for v in ${VARIANTS:-}; do
  CTR_HIP_LIB=rl_ctr_prediction_amd/variants/lib_$v.so timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider -k "gemm" > gpurun_out/tg_$v.log 2>&1 || exit $?
  tail -1 gpurun_out/tg_$v.log
  CTR_HIP_LIB=rl_ctr_prediction_amd/variants/lib_$v.so timeout -k 10 300 python tools/gemm_bench.py --reps 20 --configs $C > gpurun_out/gemm_$v.log 2>&1 || exit $?
done
echo done
