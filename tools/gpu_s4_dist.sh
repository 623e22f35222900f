# Session 4: the distribution of the default bench over separate processes on one box (the per-context spread)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 python bench.py --no-cpu --steps 50 > gpurun_out/dist_$i.json 2> gpurun_out/dist.err || { echo BENCH_FAIL; tail -20 gpurun_out/dist.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/dist_$i.json').read().strip().splitlines()[-1]); print('run $i', d['ms_per_step'], d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
