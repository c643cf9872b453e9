#!/bin/bash
# Round-5 GPU evidence batch A: sharded suite, sharded host cost, ws=2 gloo rehearsal,
# GEMM tiling sweeps (fwd0 128x160, dX N-major XCD walk). Logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_gpu_sharded.py > gpurun_out/r05_t1.log 2>&1; rc=$?
tail -3 gpurun_out/r05_t1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/gemm_planes_bench.py --sweep --only 8,29 --splits 1,2 --shapes fwd0 > gpurun_out/r05_fwd0_sweep.jsonl 2>&1 || exit 1
timeout -k 10 120 python -u tools/gemm_planes_bench.py --sweep --only 7 --splits 1 --xg 1,3 --shapes dX > gpurun_out/r05_dx_sweep.jsonl 2>&1 || exit 1
grep best gpurun_out/r05_fwd0_sweep.jsonl gpurun_out/r05_dx_sweep.jsonl
timeout -k 10 240 python -u tools/sharded_host_cost.py --config c3 > gpurun_out/r05_host_c3.log 2>&1 || exit 1
tail -1 gpurun_out/r05_host_c3.log
CTR_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --config c3 --steps 10 --warmup 3 --no-cpu-baseline --no-driver-loop > gpurun_out/r05_gloo2.log 2>&1; rc=$?
tail -1 gpurun_out/r05_gloo2.log | cut -c1-300
exit $rc
