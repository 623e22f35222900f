# Session 4 (round 3) first call: GPU tests on the rebuilt tree, the default bench, and a
# same-box A/B of the scan's age-group weights and of the per-call timing level.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_s4a.log 2>&1 || { echo PYTEST_FAIL; grep -E "^E|FAILED" gpurun_out/pytest_gpu_s4a.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu_s4a.log
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/bench_s4a.json 2> gpurun_out/bench_s4a.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_s4a.err; exit 1; }
cat gpurun_out/bench_s4a.json
timeout -k 10 300 python tools/ab_ctx.py 'def:@1' 'w2:SRD_SCAN_WEIGHTS=1,0.924,0.861,0.801@1' 'w3:SRD_SCAN_WEIGHTS=1,0.90,0.82,0.75@1' 'lvl0:@0' > gpurun_out/ab_s4a.json 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_s4a.json; exit 1; }
cat gpurun_out/ab_s4a.json
