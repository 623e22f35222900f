# Session 4: control of the weights A/B -- identical contexts in both orders, more weight points.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_ctx.py 'w2:SRD_SCAN_WEIGHTS=1,0.924,0.861,0.801@1' 'def:@1' 'w5:SRD_SCAN_WEIGHTS=1,0.91,0.84,0.78@1' 'defB:@1' 'w6:SRD_SCAN_WEIGHTS=1,0.94,0.88,0.82@1' 'even:SRD_SCAN_WEIGHTS=1,1,1,1@1' 'w2B:SRD_SCAN_WEIGHTS=1,0.924,0.861,0.801@1' > gpurun_out/ab_s4b.json 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_s4b.json; exit 1; }
cat gpurun_out/ab_s4b.json
