# Round 3: full GPU suite + smoke + default bench + rocprof kernel trace (stats + per-step timeline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
cat gpurun_out/smoke_$TAG.log
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-600 gpurun_out/bench_$TAG.json
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu --steps 20 ${BENCH_ARGS} > gpurun_out/bench_prof_$TAG.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/bench_prof_$TAG.log; exit 1; }
f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/kernel_stats_$TAG.csv
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/kernel_stats_$TAG.csv')):
    print(f\"{r['Name'][:58]:58s} {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us\")
" | head -30
t=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1); python3 tools/trace_gaps.py "$t" 2 > gpurun_out/trace_gaps_$TAG.txt; tail -30 gpurun_out/trace_gaps_$TAG.txt
