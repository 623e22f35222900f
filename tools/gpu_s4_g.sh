# Session 4: which placement matters -- the store's or the workspace's? (tools/placement_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/placement_probe.py > gpurun_out/place_g1.json 2> gpurun_out/place_g1.err || { echo P1_FAIL; tail -20 gpurun_out/place_g1.err; exit 1; }
echo default-ws; cat gpurun_out/place_g1.json
SRD_WS_MALLOC_FLAGS=4 timeout -k 10 200 python tools/placement_probe.py > gpurun_out/place_g2.json 2> gpurun_out/place_g2.err || { echo P2_FAIL; tail -20 gpurun_out/place_g2.err; exit 1; }
echo contiguous-ws; cat gpurun_out/place_g2.json
S2_FLAGS=0 timeout -k 10 200 python tools/placement_probe.py > gpurun_out/place_g3.json 2> gpurun_out/place_g3.err || { echo P3_FAIL; tail -20 gpurun_out/place_g3.err; exit 1; }
echo default-ws-s2-default; cat gpurun_out/place_g3.json
