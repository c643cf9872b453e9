#!/bin/bash
# round 3, GPU run 14: batched-bounds combine passes (same sums) — GPU suite, then C2 / C3 / C5
# against the previous scatter (variant library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest14.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest14.log | tail -8
[ $rc -eq 0 ] || exit 1
: > gpurun_out/ab14.txt
run() {  # label, env, args
  env $2 timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline $3 \
    > gpurun_out/b14.json 2> gpurun_out/b14.err || { tail -5 gpurun_out/b14.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b14.json'));k=d['kernels'];print('$1', round(d['value']/1e6,3), round(d['ms_per_step'],4), 'scatter', round(k['scatter (fm_embedding_grad segmented sums)']['ms_per_step'],4))" | tee -a gpurun_out/ab14.txt
}
OLD=CTR_HIP_LIB=$PWD/rl_ctr_prediction_amd/variants/lib_seg_before.so
for r in 1 2; do
  run "c2 new" "CTR_X=0" "--config c2"
  run "c2 old" "$OLD" "--config c2"
  run "c3 new" "CTR_X=0" "--config c3"
  run "c3 old" "$OLD" "--config c3"
done
run "c5 new" "CTR_X=0" "--config c5"
run "c5 old" "$OLD" "--config c5"
