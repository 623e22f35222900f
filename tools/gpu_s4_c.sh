# Session 4: 8 identical contexts in one process -- does the workspace placement change the scan time?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SRD_DEBUG_ALLOC=1 ROUNDS=12 timeout -k 10 300 python tools/ab_ctx.py c0:@1 c1:@1 c2:@1 c3:@1 c4:@1 c5:@1 c6:@1 c7:@1 > gpurun_out/ab_s4c.json 2> gpurun_out/ab_s4c.err || { echo AB_FAIL; tail -20 gpurun_out/ab_s4c.err; exit 1; }
cat gpurun_out/ab_s4c.json
