# rocprof kernel stats of the C2 bench (optionally under an env setting), summarised per step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_e
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e -o run -- python3 bench.py --no-cpu --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/prof_e.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_e.log; exit 1; }
grep '^{' gpurun_out/prof_e.log | cut -c1-300
f=$(find gpurun_out/prof_e -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    print(f\"{r['Name'][:58]:58s} {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us\")
" | head -40
