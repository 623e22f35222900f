# rehearsal of the N>1 bench path on a 1-GPU box: 2 ranks on cuda:0 over gloo
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SRD_BENCH_SAME_DEVICE=1 SRD_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --entries-per-gpu 262144 > gpurun_out/bench_n2.log 2> gpurun_out/bench_n2.err || { echo BENCH2_FAIL; tail -30 gpurun_out/bench_n2.err; exit 1; }
cat gpurun_out/bench_n2.log
