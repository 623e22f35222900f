set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/bw_probe > gpurun_out/bw_probe.log 2>&1 || { echo BW_FAIL; tail gpurun_out/bw_probe.log; exit 1; }
cat gpurun_out/bw_probe.log
timeout -k 10 300 python bench.py --no-cpu --e2e --steps 10 > gpurun_out/bench_e2e.log 2> gpurun_out/bench_e2e.err || { echo E2E_FAIL; tail -20 gpurun_out/bench_e2e.err; exit 1; }
grep e2e gpurun_out/bench_e2e.err
bash tools/gpu_pmc.sh > gpurun_out/pmc_summary.log 2>&1 || { echo PMC_FAIL; tail -20 gpurun_out/pmc_summary.log; exit 1; }
cat gpurun_out/pmc_summary.log
