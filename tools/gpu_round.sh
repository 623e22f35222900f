# One GPU call: parity tests, smoke, full bench (with CPU baseline), rocprof kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -50 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.log
rm -rf gpurun_out/prof_g
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_g -o run -- python3 bench.py --no-cpu --steps 20 > gpurun_out/bench_prof.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/bench_prof.log; exit 1; }
f=$(find gpurun_out/prof_g -name '*kernel_stats.csv' | head -1); echo "$f"; cut -d, -f1-8 "$f" | head -40
