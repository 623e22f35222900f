set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { local n=$1; shift; rm -rf gpurun_out/pmc_$n
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_$n -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS} > gpurun_out/pmc_$n.log 2>&1 || { echo "PMC $n FAIL"; tail -5 gpurun_out/pmc_$n.log; exit 1; }; }
run a SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT
run b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
python3 tools/pmc_sum.py gpurun_out/pmc_a gpurun_out/pmc_b | sed -n '/scan_kernel/,/WRITE_SIZE\|^--/p' | head -24
