# C5 batch-write bench (pinned host -> HBM, and the writer kernel alone) + rocprof stats of it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/bench_c5.log 2> gpurun_out/bench_c5.err || { echo C5_FAIL; tail -20 gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.log
if [ -n "$C5_PROF" ]; then
  rm -rf gpurun_out/prof_c5
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/prof_c5.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_c5.log; exit 1; }
  f=$(find gpurun_out/prof_c5 -name '*kernel_stats.csv' | head -1)
  cut -d, -f1-4 "$f" | head -12
fi
