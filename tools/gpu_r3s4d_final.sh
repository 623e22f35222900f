# Round 3, session 4: final evidence -- PMC passes (traffic.json for these sources, so the bench line carries
# roofline.traffic), tests + smoke + default bench + rocprof (gpu_r3_full.sh), extra configs, the N=2 rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_pmc.sh > gpurun_out/pmc_summary_r3s4d.txt 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/pmc_summary_r3s4d.txt; exit 1; }
head -30 gpurun_out/pmc_summary_r3s4d.txt
python3 tools/traffic_json.py gpurun_out/pmc_c gpurun_out/pmc_d gpurun_out/traffic_r3s4d.json || { echo TRAFFIC_FAIL; exit 1; }
cp gpurun_out/traffic_r3s4d.json profiles/traffic.json
TAG=r3s4d bash tools/gpu_r3_full.sh || exit 1
TAG=r3s4d CONFIGS="c2torn c2full c3 c5 e2e ops" bash tools/gpu_r3_extra.sh || exit 1
SRD_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_n2_r3s4d.json 2> gpurun_out/bench_n2_r3s4d.err || { echo N2_FAIL; tail -20 gpurun_out/bench_n2_r3s4d.err; exit 1; }
cut -c1-300 gpurun_out/bench_n2_r3s4d.json
