# Session 4: slow first contexts -- HW queue binding order vs workspace allocation order
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "BIND_ORDER=reverse" "BIND_ORDER=forward" "BIND_ORDER=reverse FIRST_ORDER=reverse" "BIND_ORDER=reverse"; do
  env $cfg ROUNDS=8 REPS=6 timeout -k 10 150 python tools/ab_ctx.py a:@1 b:@1 c:@1 d:@1 e:@1 f:@1 > gpurun_out/bind.json 2>gpurun_out/bind.err || { echo BIND_FAIL; tail gpurun_out/bind.err; exit 1; }
  echo "$cfg $(python3 -c "import json; d=json.load(open('gpurun_out/bind.json')); print({k: v['scan_ms_med'] for k, v in d.items()})")"
done
