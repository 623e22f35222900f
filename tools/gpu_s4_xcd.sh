# Session 4: per-XCD block weights -- GPU tests (partition correctness), then the in-context A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
# timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_s4xcd.log 2>&1 || { echo PYTEST_FAIL; grep -E "^E|FAILED" gpurun_out/pytest_gpu_s4xcd.log | head -30; exit 1; }
# tail -1 gpurun_out/pytest_gpu_s4xcd.log
NCTX=4 LEARN=8 timeout -k 10 300 python tools/xcd_ab.py > gpurun_out/xcd_ab.txt 2> gpurun_out/xcd_ab.err || { echo XAB_FAIL; tail -20 gpurun_out/xcd_ab.err; exit 1; }
cat gpurun_out/xcd_ab.txt
