# Round 3 evidence, part 2: PMC passes of the C2 bench (traffic.json), the extra configs, the N=2 one-box rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_pmc.sh > gpurun_out/pmc_summary_r3final.txt 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/pmc_summary_r3final.txt; exit 1; }
head -30 gpurun_out/pmc_summary_r3final.txt
TAG=r3final CONFIGS="c2torn c2full c3 c5 e2e ops" bash tools/gpu_r3_extra.sh || exit 1
SRD_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_n2_r3final.json 2> gpurun_out/bench_n2_r3final.err || { echo N2_FAIL; tail -20 gpurun_out/bench_n2_r3final.err; exit 1; }
cut -c1-300 gpurun_out/bench_n2_r3final.json
