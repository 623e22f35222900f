# Session 4: per-slot scan weights, second A/B inside each context: how far past the fixed point
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
D=1,0.93545,0.88889,0.84818
S16=1.0000,0.9858,0.9864,0.9858,0.9171,0.9165,0.9166,0.9059,0.8582,0.8508,0.8517,0.8502,0.7970,0.7953,0.7960,0.7876
S15=1.0000,0.9787,0.9796,0.9788,0.9081,0.9072,0.9074,0.8915,0.8432,0.8324,0.8337,0.8314,0.7726,0.7701,0.7712,0.7590
S20=1.0000,0.9717,0.9729,0.9718,0.8991,0.8979,0.8982,0.8773,0.8286,0.8144,0.8161,0.8131,0.7490,0.7457,0.7471,0.7314
NCTX=3 timeout -k 10 400 python tools/weights_ab.py def=$D s16=$S16 s15=$S15 s20=$S20 > gpurun_out/wab2.txt 2> gpurun_out/wab2.err || { echo WAB_FAIL; tail -20 gpurun_out/wab2.err; exit 1; }
cat gpurun_out/wab2.txt
