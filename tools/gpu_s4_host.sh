# Session 4: host overhead per call -- C loop vs the Python call path, timing level 0 vs 1 inside one context
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 120 ./tools/c_loop > gpurun_out/c_loop.json 2> gpurun_out/c_loop.err || { echo C_FAIL; tail gpurun_out/c_loop.err; exit 1; }
cat gpurun_out/c_loop.json
timeout -k 10 120 python tools/py_loop.py > gpurun_out/py_loop.json 2> gpurun_out/py_loop.err || { echo PY_FAIL; tail gpurun_out/py_loop.err; exit 1; }
cat gpurun_out/py_loop.json
done
