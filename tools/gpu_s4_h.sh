# Session 4: does the scan time drift within a process (clock ramp) and differ between processes?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python tools/drift_probe.py > gpurun_out/drift_$i.json 2> gpurun_out/drift.err || { echo DRIFT_FAIL; tail -20 gpurun_out/drift.err; exit 1; }
cat gpurun_out/drift_$i.json
done
