# rocprofv3 kernel stats of the C4 bench (PolicyGradient.learn), top kernels printed
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4t
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4t -o run -- \
  python3 bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c4t/b.log 2>&1 || exit $?
python3 tools/kstats.py $(find gpurun_out/c4t -name "*kernel_stats.csv" | head -1) 2>/dev/null || \
  head -25 $(find gpurun_out/c4t -name "*kernel_stats.csv" | head -1)
