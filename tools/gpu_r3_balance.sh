# Round 3: scan wave-slot balance A/B (ScanPart weights): parity suite, stamps, bench alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_bal.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu_bal.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_bal.log
fi
for W in default 1,1,1,1; do
  if [ $W = default ]; then unset SRD_SCAN_WEIGHTS; else export SRD_SCAN_WEIGHTS=$W; fi
  echo "== stamps weights=$W"
  timeout -k 10 200 python tools/wave_stamps.py > gpurun_out/stamps_$W.json 2>&1 || { echo STAMPS_FAIL; tail -20 gpurun_out/stamps_$W.json; exit 1; }
  tail -2 gpurun_out/stamps_$W.json | cut -c1-700
done
for rep in 1 2 3; do
for W in default 1,1,1,1; do
  if [ $W = default ]; then unset SRD_SCAN_WEIGHTS; else export SRD_SCAN_WEIGHTS=$W; fi
  timeout -k 10 200 python bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/bench_bal_$W.json 2> gpurun_out/bench_bal.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_bal.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_bal_$W.json').read().strip().splitlines()[-1])
print('$W', 'ms_per_step', d['ms_per_step'], 'scan_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"
done
done
