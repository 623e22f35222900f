set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/prof_g
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g -o run -- python3 bench.py --no-cpu --steps 10 ${BENCH_ARGS} > gpurun_out/bench_prof.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/bench_prof.log; exit 1; }
f=$(find gpurun_out/prof_g -name '*kernel_stats.csv' | head -1); echo "$f"; cut -d, -f1-8 "$f" | head -40
