# Session 4: link2 one block per scan wave + precomputed wave shares -- GPU tests, C2 and C3 kernel breakdowns
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_s4l2.log 2>&1 || { echo PYTEST_FAIL; grep -E "^E|FAILED" gpurun_out/pytest_gpu_s4l2.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu_s4l2.log
for cfg in c2 c3; do
  steps=20; [ $cfg = c3 ] && steps=5
  rm -rf gpurun_out/prof_l2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_l2 -o run -- python3 bench.py --no-cpu --config $cfg --steps $steps --warmup 1 > gpurun_out/prof_l2.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_l2.log; exit 1; }
  f=$(find gpurun_out/prof_l2 -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/kernel_stats_${cfg}_l2.csv
  echo "== $cfg"; grep '^{' gpurun_out/prof_l2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])"
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/kernel_stats_${cfg}_l2.csv')):
    print(f\"{r['Name'][:58]:58s} {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us\")
" | head -14
done
