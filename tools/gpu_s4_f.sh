# Session 4: record regions at 8 slots per span -- GPU tests, then same-box bench A/B (new vs HEAD build) on
# C2 (one context per process: the first-allocated workspace), C2FULL and C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_s4f.log 2>&1 || { echo PYTEST_FAIL; grep -E "^E|FAILED" gpurun_out/pytest_gpu_s4f.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu_s4f.log
for cfg in ${CONFIGS:-c2 c2full c3}; do
for rep in 1 2 3; do
for V in new prev; do
  unset SRD_LIB_PATH
  [ $V = prev ] && export SRD_LIB_PATH=$PWD/rust-simd-r-drive_amd/build/var/lib_prev.so
  steps=30; [ $cfg = c3 ] && steps=8
  timeout -k 10 200 python bench.py --no-cpu --config $cfg --steps $steps > gpurun_out/abf_${cfg}_$V.json 2> gpurun_out/abf.err || { echo BENCH_FAIL; tail -30 gpurun_out/abf.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/abf_${cfg}_$V.json').read().strip().splitlines()[-1])
print('$cfg', '$V', 'ms_per_step', d['ms_per_step'], 'scan_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"
done
done
[ $cfg = c3 ] && break
done
