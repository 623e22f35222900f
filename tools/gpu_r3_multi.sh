# Round 3: the device-resident multi-GPU open (tests + C4 + one-GPU --gpus 2 rehearsal)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_multi_device.py tests/test_gpu_multi.py -x -v -m gpu --timeout 400 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_multi.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_multi.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_multi.log | tail -40
SRD_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/bench_n2.log 2>gpurun_out/bench_n2.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_n2.err; exit 1; }
cat gpurun_out/bench_n2.log
