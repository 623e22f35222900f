# Session 4: per-context spread -- the previous call's dirty glue outputs written back during the scan?
# gluent: timing variant whose glue stores its per-entry outputs nontemporally
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in prod gluent prod gluent; do
  if [ $v = prod ]; then unset SRD_LIB_PATH; else export SRD_LIB_PATH=$PWD/rust-simd-r-drive_amd/build/var/lib_$v.so; fi
  ROUNDS=8 REPS=6 timeout -k 10 150 python tools/ab_ctx.py a:@1 b:@1 c:@1 d:@1 e:@1 f:@1 > gpurun_out/gnt.json 2>gpurun_out/gnt.err || { echo GNT_FAIL; tail gpurun_out/gnt.err; exit 1; }
  echo "$v $(python3 -c "import json; d=json.load(open('gpurun_out/gnt.json')); print({k: (v['scan_ms_med'], v['wall_ms_med']) for k, v in d.items()})")"
done
