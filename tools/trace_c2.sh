# rocprofv3 kernel trace of the C2 bench (graph-replayed steps) + per-step timeline
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/trace_c2${TAG}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 bench.py --config ${CFG:-c2} --steps 30 --warmup 5 --no-cpu-baseline --breakdown-steps 1 $EXTRA > $OUT/bench.log 2>&1 || exit $?
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $f > $OUT/timeline.txt
s=$(find $OUT -name "*kernel_stats.csv" | head -1)
cp $s $OUT/kernel_stats.csv
head -60 $OUT/timeline.txt
