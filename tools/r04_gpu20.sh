#!/bin/bash
# Round-4: HIP runtime launch knobs on the graph-replayed steps (alternating bench runs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ENV_A="HIP_FORCE_DEV_KERNARG=1" ENV_B="HIP_FORCE_DEV_KERNARG=0" CFGS="c2 c3" RUNS=3 BENCH_ARGS="--no-driver-loop" bash tools/env_ab.sh || exit 1
