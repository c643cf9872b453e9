set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "transpose" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_dw0.log 2>&1
for i in 1 2 3; do
  for v in 1 2 0; do
    CTR_DW0_KC=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_${v}_${i}.log 2>&1
    echo "kc=$v $(tail -1 gpurun_out/ab_${v}_${i}.log | cut -c100-135)"
  done
done
