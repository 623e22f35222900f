# Round 3: GPU tests, then same-box A/B of the product build vs build/var/lib_prev.so on C2 and C2FULL
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_ab2.log 2>&1 || { grep -E "^E|FAILED|srd:" gpurun_out/pytest_gpu_ab2.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu_ab2.log
for cfg in ${CONFIGS:-c2 c2full}; do
for rep in 1 2 3; do
for V in new prev; do
  unset SRD_LIB_PATH
  [ $V = prev ] && export SRD_LIB_PATH=$PWD/rust-simd-r-drive_amd/build/var/lib_prev.so
  timeout -k 10 200 python bench.py --no-cpu --config $cfg --steps 30 > gpurun_out/ab2_${cfg}_$V.json 2> gpurun_out/ab2.err || { echo BENCH_FAIL; tail -30 gpurun_out/ab2.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab2_${cfg}_$V.json').read().strip().splitlines()[-1])
print('$cfg', '$V', 'ms_per_step', d['ms_per_step'], 'scan_ms', d['roofline']['kernel_ms'])"
done
done
done
