set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/block_persist.py > gpurun_out/block_persist.json 2> gpurun_out/bp.err || { echo BP_FAIL; tail gpurun_out/bp.err; exit 1; }
cat gpurun_out/block_persist.json
timeout -k 10 120 python tools/block_persist.py > gpurun_out/block_persist2.json 2> gpurun_out/bp.err || { echo BP_FAIL; tail gpurun_out/bp.err; exit 1; }
cat gpurun_out/block_persist2.json
