# Session 4: per-context spread vs creation order -- the store allocated before the contexts (STORE_FIRST)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for sf in 1 0 1 0 1; do
  if [ $sf = 1 ]; then export STORE_FIRST=1; else unset STORE_FIRST; fi
  ROUNDS=8 REPS=6 timeout -k 10 150 python tools/ab_ctx.py a:@1 b:@1 c:@1 d:@1 e:@1 f:@1 > gpurun_out/sf.json 2>gpurun_out/sf.err || { echo SF_FAIL; tail gpurun_out/sf.err; exit 1; }
  echo "store_first=$sf $(python3 -c "import json; d=json.load(open('gpurun_out/sf.json')); print({k: v['scan_ms_med'] for k, v in d.items()})")"
done
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --no-cpu --steps 30 > gpurun_out/sf_bench.json 2>gpurun_out/sf.err || { echo SFB_FAIL; tail gpurun_out/sf.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sf_bench.json').read().strip().splitlines()[-1]); print('bench', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
