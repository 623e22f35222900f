# A/B timing of library variants (scan ms per launch + total ms) + the GPU tests of the current build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/ab_scan.py ${AB_LIBS} > gpurun_out/ab.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab.log; exit 1; }
cat gpurun_out/ab.log
