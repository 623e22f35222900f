# per-kernel rocprof stats of ab_scan runs, one lib per process (debug)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "$@"; do
  n=$(basename $lib .so)
  rm -rf gpurun_out/p_$n
  AB_NOCHECK=1 ROUNDS=3 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_$n -o run -- python3 tools/ab_scan.py $lib > gpurun_out/p_$n.log 2>&1 || { echo PROF_FAIL $n; tail -5 gpurun_out/p_$n.log; exit 1; }
  f=$(find gpurun_out/p_$n -name '*kernel_stats.csv' | head -1)
  echo "== $n"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'synth' in r['Name']: continue
    print(f\"{r['Name'][:50]:50s} {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us\")
" | head -8
done
