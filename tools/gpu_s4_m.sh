# Session 4: slow vs fast contexts from inside the scan (tools/stamps_ctx.py, SRD_WAVE_STAMPS build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
NCTX=5 timeout -k 10 120 python tools/stamps_ctx.py > gpurun_out/stamps_ctx.txt 2>gpurun_out/stamps_ctx.err || { echo ST_FAIL; tail gpurun_out/stamps_ctx.err; exit 1; }
cat gpurun_out/stamps_ctx.txt
