# Session 4: C3 kernel breakdown (rocprof stats + trace gaps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 bench.py --no-cpu --config c3 --steps 5 --warmup 1 > gpurun_out/prof_c3.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_c3.log; exit 1; }
f=$(find gpurun_out/prof_c3 -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/kernel_stats_c3_r3s4.csv
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/kernel_stats_c3_r3s4.csv')):
    print(f\"{r['Name'][:58]:58s} {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us\")
" | head -30
t=$(find gpurun_out/prof_c3 -name '*kernel_trace.csv' | head -1); python3 tools/trace_gaps.py "$t" 2 > gpurun_out/trace_gaps_c3_r3s4.txt; tail -20 gpurun_out/trace_gaps_c3_r3s4.txt
