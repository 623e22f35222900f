# Round 3: extra bench configs (torn tail, forced full pass, e2e, C3, C5) -- each with its own limit
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3}
for cfg in ${CONFIGS:-c2torn e2e}; do
  case $cfg in
    e2e) args="--e2e --no-cpu --steps 10" ;;
    c2torn) args="--config c2torn --no-cpu --steps 20 --warmup 3" ;;
    c2full) args="--config c2full --no-cpu --steps 20 --warmup 3" ;;
    c3) args="--config c3 --no-cpu --steps 10 --warmup 2" ;;
    c5) args="--config c5 --steps 5 --warmup 2" ;;
    ops) args="--config ops" ;;
  esac
  timeout -k 10 400 python bench.py $args > gpurun_out/bench_${cfg}_$TAG.json 2> gpurun_out/bench_${cfg}_$TAG.err || { echo BENCH_FAIL $cfg; tail -30 gpurun_out/bench_${cfg}_$TAG.err; exit 1; }
  echo "== $cfg"; cut -c1-400 gpurun_out/bench_${cfg}_$TAG.json
  if [ "$cfg" = e2e ]; then grep '^{' gpurun_out/bench_${cfg}_$TAG.err | cut -c1-1500; fi
done
if [ -n "$PROF_CFG" ]; then
  rm -rf gpurun_out/prof_${PROF_CFG}_$TAG
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${PROF_CFG}_$TAG -o run -- python3 bench.py --no-cpu --config $PROF_CFG --steps 5 --warmup 1 > gpurun_out/prof_${PROF_CFG}_$TAG.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_${PROF_CFG}_$TAG.log; exit 1; }
  f=$(find gpurun_out/prof_${PROF_CFG}_$TAG -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/kernel_stats_${PROF_CFG}_$TAG.csv
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/kernel_stats_${PROF_CFG}_$TAG.csv')):
    print(f\"{r['Name'][:58]:58s} {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us  tot {float(r['TotalDurationNs'])/1e6:8.2f} ms\")
" | head -40
fi
