# Session 4: is the slow placement of the first-allocated workspaces the record regions' page spread?
# A..F allocate in order; B, D, F start with 8 candidate slots per span (records 4096 x 17 KiB instead of x 135 KiB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUNDS=10 timeout -k 10 300 python tools/ab_ctx.py A64:@1 B8:SRD_INIT_CAP=8@1 C64:@1 D8:SRD_INIT_CAP=8@1 E64:@1 F8:SRD_INIT_CAP=8@1 > gpurun_out/ab_s4e.json 2> gpurun_out/ab_s4e.err || { echo AB_FAIL; tail -20 gpurun_out/ab_s4e.err; exit 1; }
cat gpurun_out/ab_s4e.json; tail -1 gpurun_out/ab_s4e.err
