# Session 4: per-slot scan weights -- GPU tests, then same-process A/B with three contexts per setting
# def = the age-group default; s16 = per-slot shares from this build's wave stamps; s16d = the same, damped
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_s4x.log 2>&1 || { echo PYTEST_FAIL; grep -E "^E|FAILED" gpurun_out/pytest_gpu_s4x.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu_s4x.log
S16=1.0000,0.9858,0.9864,0.9858,0.9171,0.9165,0.9166,0.9059,0.8582,0.8508,0.8517,0.8502,0.7970,0.7953,0.7960,0.7876
S16D=1.0000,0.9929,0.9932,0.9929,0.9262,0.9259,0.9260,0.9206,0.8734,0.8696,0.8701,0.8693,0.8222,0.8213,0.8217,0.8173
ROUNDS=8 REPS=6 timeout -k 10 400 python tools/ab_ctx.py def1:@1 s16a:SRD_SCAN_WEIGHTS=$S16@1 s16da:SRD_SCAN_WEIGHTS=$S16D@1 def2:@1 s16b:SRD_SCAN_WEIGHTS=$S16@1 s16db:SRD_SCAN_WEIGHTS=$S16D@1 def3:@1 s16c:SRD_SCAN_WEIGHTS=$S16@1 s16dc:SRD_SCAN_WEIGHTS=$S16D@1 > gpurun_out/ab_s4x.json 2> gpurun_out/ab_s4x.err || { echo AB_FAIL; tail -20 gpurun_out/ab_s4x.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab_s4x.json')); print({k: (v['scan_ms_med'], v['wall_ms_med']) for k, v in d.items()})"
