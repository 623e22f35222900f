# One parameterised GPU-box script (replaces the per-session gpu_*.sh lease scripts).
#   bash tools/gpu.sh STEP [STEP ...]     run on the box: gpurun -- 'bash tools/gpu.sh tests bench prof'
# Steps (each under its own time limit; the first failure ends the call):
#   tests        pytest -m gpu ($PYTEST_TARGETS, default: tests)   smoke   __graft_entry__.smoke()
#   bench        python bench.py $BENCH_ARGS           prof    rocprofv3 kernel stats of a 20-step bench
#   pmc          the standard PMC passes + traffic     pmcx    one extra PMC pass: counters in $PMC
#   list         rocprofv3 -L (available counters)     ab      python $AB (an A/B timing tool) $AB_ARGS
#   pmcab        one PMC pass ($PMC) over python $AB $AB_ARGS
# TAG names the outputs (gpurun_out/*_$TAG*); BENCH_ARGS is passed to every bench.py run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4}
for step in "$@"; do
  case "$step" in
  tests)
    timeout -k 10 600 python -u -m pytest ${PYTEST_TARGETS:-tests} -x -v -m gpu --timeout 400 --timeout-method thread \
      > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
    tail -2 gpurun_out/pytest_gpu_$TAG.log ;;
  smoke)
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
      || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
    cat gpurun_out/smoke_$TAG.log ;;
  bench)
    timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
      || { echo BENCH_FAIL; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
    cut -c1-900 gpurun_out/bench_$TAG.json ;;
  prof)
    rm -rf gpurun_out/prof_$TAG
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
      python3 bench.py --no-cpu --steps 20 ${BENCH_ARGS} > gpurun_out/bench_prof_$TAG.log 2>&1 \
      || { echo PROF_FAIL; tail -20 gpurun_out/bench_prof_$TAG.log; exit 1; }
    f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/kernel_stats_$TAG.csv
    python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/kernel_stats_$TAG.csv')):
    print(f\"{r['Name'][:58]:58s} {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us  min {float(r['MinNs'])/1e3:9.1f}\")
" | head -30
    t=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
    python3 tools/trace_gaps.py "$t" 2 > gpurun_out/trace_gaps_$TAG.txt; tail -12 gpurun_out/trace_gaps_$TAG.txt ;;
  pmc)
    bash tools/gpu_pmc.sh > gpurun_out/pmc_summary_$TAG.txt 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/pmc_summary_$TAG.txt; exit 1; }
    head -32 gpurun_out/pmc_summary_$TAG.txt
    python3 tools/traffic_json.py gpurun_out/pmc_c gpurun_out/pmc_d gpurun_out/traffic_$TAG.json || { echo TRAFFIC_FAIL; exit 1; } ;;
  pmcx)
    rm -rf gpurun_out/pmc_x_$TAG
    timeout -s KILL 120 rocprofv3 --pmc ${PMC} --output-format csv -d gpurun_out/pmc_x_$TAG -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS} > gpurun_out/pmc_x_$TAG.log 2>&1 \
      || { echo PMCX_FAIL; tail -8 gpurun_out/pmc_x_$TAG.log; exit 1; }
    python3 tools/pmc_sum.py gpurun_out/pmc_x_$TAG | tee gpurun_out/pmc_x_summary_$TAG.txt | head -20 ;;
  pmcab)
    # one PMC pass over an A/B tool run (e.g. a single timing-only variant): counters in $PMC
    rm -rf gpurun_out/pmc_ab_$TAG
    timeout -s KILL 150 rocprofv3 --pmc ${PMC} --output-format csv -d gpurun_out/pmc_ab_$TAG -o run -- \
      python3 ${AB} ${AB_ARGS} > gpurun_out/pmc_ab_$TAG.log 2>&1 || { echo PMCAB_FAIL; tail -8 gpurun_out/pmc_ab_$TAG.log; exit 1; }
    python3 tools/pmc_sum.py gpurun_out/pmc_ab_$TAG | tee gpurun_out/pmc_ab_summary_$TAG.txt | head -24 ;;
  list)
    timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_$TAG.txt 2>&1 || { echo LIST_FAIL; exit 1; }
    grep -o "SQ_[A-Z_0-9]*LDS[A-Z_0-9]*" gpurun_out/counters_$TAG.txt | sort -u | head -40 ;;
  ab)
    timeout -k 10 ${AB_TIMEOUT:-300} python -u ${AB} ${AB_ARGS} > gpurun_out/ab_$TAG.txt 2>&1 \
      || { echo AB_FAIL; tail -20 gpurun_out/ab_$TAG.txt; exit 1; }
    cat gpurun_out/ab_$TAG.txt ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
