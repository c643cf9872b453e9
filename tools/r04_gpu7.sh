#!/bin/bash
# Round-4 GPU session 7b: C2 regions over one process under plan-stream variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { local tag=$1; shift
  env "$@" timeout -k 10 200 python tools/c2_repeat.py $ARGS > gpurun_out/r04_c2_rep_$tag.txt 2>&1 || exit 1
  echo "== $tag $* $ARGS"; grep -v amdgpu.ids gpurun_out/r04_c2_rep_$tag.txt | grep rep; }
ARGS="" run base CTR_PLAN_STREAMS=2
ARGS="" run one_stream CTR_PLAN_STREAMS=1
ARGS="" run lsd CTR_PLAN_COLS=0
ARGS="--lookahead 0" run inplan CTR_PLAN_STREAMS=2
ARGS="--lookahead 3" run la3 CTR_PLAN_STREAMS=2
