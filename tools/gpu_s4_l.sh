# Session 4: slow first contexts -- HW queue assignment? (QUEUE_BURN streams launched before the contexts)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for qb in 0 4 0 4 8; do
QUEUE_BURN=$qb NCTX=6 CALLS=7 timeout -k 10 120 python tools/tlb_probe.py > gpurun_out/qb.json 2>gpurun_out/qb.err || { echo QB_FAIL; tail gpurun_out/qb.err; exit 1; }
echo "burn=$qb $(cat gpurun_out/qb.json)"
done
