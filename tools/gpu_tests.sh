# GPU parity suite (optionally a subset via PYTEST_K) with per-test timeouts, then smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${SUITE_TIMEOUT:-800} python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -80 gpurun_out/pytest_gpu.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -80
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
