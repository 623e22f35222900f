# Session 4: position claims in link2 -- GPU tests, then same-box A/B of the library call (tools/ab_scan.py: new vs HEAD)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_s4i.log 2>&1 || { echo PYTEST_FAIL; grep -E "^E|FAILED" gpurun_out/pytest_gpu_s4i.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu_s4i.log
ROUNDS=14 timeout -k 10 300 python tools/ab_scan.py rust-simd-r-drive_amd/build/libsrd_amd.so@1 rust-simd-r-drive_amd/build/var/lib_prev.so@1 > gpurun_out/ab_s4i.json 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_s4i.json; exit 1; }
cat gpurun_out/ab_s4i.json
rm -rf gpurun_out/prof_i
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_i -o run -- python3 bench.py --no-cpu --steps 20 > gpurun_out/bench_prof_i.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/bench_prof_i.log; exit 1; }
f=$(find gpurun_out/prof_i -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -12
ROUNDS=12 timeout -k 10 300 python tools/ab_ctx.py 'def:@1' 'w6:SRD_SCAN_WEIGHTS=1,0.94,0.88,0.82@1' 'even:SRD_SCAN_WEIGHTS=1,1,1,1@1' 'w7:SRD_SCAN_WEIGHTS=1,0.96,0.91,0.86@1' 'w8:SRD_SCAN_WEIGHTS=1,0.92,0.85,0.79@1' 'def2:@1' > gpurun_out/ab_s4i_w.json 2> gpurun_out/ab_s4i_w.err || { echo ABW_FAIL; tail -20 gpurun_out/ab_s4i_w.err; exit 1; }
cat gpurun_out/ab_s4i_w.json | tr -d '\n'; echo
