# Session 4: per-context scan rate -- does a fresh stream change it? (tools/renew_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 python tools/renew_probe.py > gpurun_out/renew.txt 2>gpurun_out/renew.err || { echo RENEW_FAIL; tail gpurun_out/renew.err; exit 1; }
cat gpurun_out/renew.txt
