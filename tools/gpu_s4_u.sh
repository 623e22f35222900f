# Session 4: nontemporal scan stores (tile values + records) -- same-process A/B, three contexts per build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
N=rust-simd-r-drive_amd/build/libsrd_amd.so; V=rust-simd-r-drive_amd/build/var/lib_scannt.so
ROUNDS=10 timeout -k 10 400 python tools/ab_scan.py $N@1 $V@1 $N@1 $V@1 $N@1 $V@1 $N@1 $V@1 > gpurun_out/ab_s4u.json 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_s4u.json; exit 1; }
python3 - <<'PY'
import json
txt = open("gpurun_out/ab_s4u.json").read()
print(json.dumps(json.loads(txt[txt.index("{"):])))
PY
