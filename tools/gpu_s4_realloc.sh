set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/realloc_probe.py > gpurun_out/realloc.txt 2> gpurun_out/realloc.err || { echo RA_FAIL; tail -20 gpurun_out/realloc.err; exit 1; }
cat gpurun_out/realloc.txt
