# Session 4: placement vs context order -- first calls (workspace allocations) in reverse order; then with 1 GiB pads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
FIRST_ORDER=reverse ROUNDS=10 timeout -k 10 300 python tools/ab_ctx.py c0:@1 c1:@1 c2:@1 c3:@1 c4:@1 c5:@1 > gpurun_out/ab_s4d1.json 2> gpurun_out/ab_s4d1.err || { echo AB_FAIL; tail -20 gpurun_out/ab_s4d1.err; exit 1; }
cat gpurun_out/ab_s4d1.json; tail -1 gpurun_out/ab_s4d1.err
PAD_MB=1024 ROUNDS=10 timeout -k 10 300 python tools/ab_ctx.py c0:@1 c1:@1 c2:@1 c3:@1 c4:@1 c5:@1 > gpurun_out/ab_s4d2.json 2> gpurun_out/ab_s4d2.err || { echo AB_FAIL; tail -20 gpurun_out/ab_s4d2.err; exit 1; }
cat gpurun_out/ab_s4d2.json; tail -1 gpurun_out/ab_s4d2.err
