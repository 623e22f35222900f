# Session 4: GPU tests on the lazy scan-event readout; same-process A/B, three contexts per build (the
# per-context spread of the scan rate): new vs HEAD vs new with nontemporal glue stores
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_s4t.log 2>&1 || { echo PYTEST_FAIL; grep -E "^E|FAILED" gpurun_out/pytest_gpu_s4t.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu_s4t.log
N=rust-simd-r-drive_amd/build/libsrd_amd.so; P=rust-simd-r-drive_amd/build/var/lib_prev.so; G=rust-simd-r-drive_amd/build/var/lib_gluent.so
ROUNDS=10 timeout -k 10 400 python tools/ab_scan.py $N@1 $P@1 $G@1 $N@1 $P@1 $G@1 $N@1 $P@1 $G@1 > gpurun_out/ab_s4t.json 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_s4t.json; exit 1; }
python3 - <<'PY'
import json
txt = open("gpurun_out/ab_s4t.json").read()
d = json.loads(txt[txt.index("{"):])
print(json.dumps(d))
PY
