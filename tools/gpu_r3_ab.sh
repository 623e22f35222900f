# Round 3: same-box A/B of the product build vs build/var/lib_prev.so (previous commit), + stamps, + GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_ab.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu_ab.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_ab.log
fi
if [ -n "$STAMPS" ]; then
timeout -k 10 200 python tools/wave_stamps.py > gpurun_out/stamps_ab.json 2>&1 || { echo STAMPS_FAIL; tail -20 gpurun_out/stamps_ab.json; exit 1; }
tail -2 gpurun_out/stamps_ab.json
fi
for rep in 1 2 3; do
for V in ${VARIANTS:-new prev}; do
  unset SRD_LIB_PATH SRD_SCAN_DYN
  case $V in
    prev) export SRD_LIB_PATH=$PWD/rust-simd-r-drive_amd/build/var/lib_prev.so ;;
    nodyn) export SRD_SCAN_DYN=0 ;;
    dyn5) export SRD_SCAN_DYN=5 ;;
    dyn20) export SRD_SCAN_DYN=20 ;;
  esac
  timeout -k 10 200 python bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/bench_ab_$V.json 2> gpurun_out/bench_ab.err || { echo BENCH_FAIL; tail -30 gpurun_out/bench_ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_ab_$V.json').read().strip().splitlines()[-1])
print('$V', 'ms_per_step', d['ms_per_step'], 'scan_ms', d['roofline']['kernel_ms'], 'frac', d['roofline']['frac'])"
done
done
