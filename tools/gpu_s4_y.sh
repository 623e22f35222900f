# Session 4: per-slot scan weights, A/B inside each context (tools/weights_ab.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
D=1,0.93545,0.88889,0.84818
S16=1.0000,0.9858,0.9864,0.9858,0.9171,0.9165,0.9166,0.9059,0.8582,0.8508,0.8517,0.8502,0.7970,0.7953,0.7960,0.7876
S16D=1.0000,0.9929,0.9932,0.9929,0.9262,0.9259,0.9260,0.9206,0.8734,0.8696,0.8701,0.8693,0.8222,0.8213,0.8217,0.8173
NCTX=3 timeout -k 10 400 python tools/weights_ab.py def=$D s16=$S16 s16d=$S16D even=1,1,1,1 > gpurun_out/wab.txt 2> gpurun_out/wab.err || { echo WAB_FAIL; tail -20 gpurun_out/wab.err; exit 1; }
cat gpurun_out/wab.txt
