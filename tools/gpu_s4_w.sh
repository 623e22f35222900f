# Session 4: per-slot wave end times with the current build (tools/wave_stamps.py), for per-slot scan weights
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/wave_stamps.py > gpurun_out/stamps_w.txt 2>gpurun_out/stamps_w.err || { echo ST_FAIL; tail gpurun_out/stamps_w.err; exit 1; }
python3 -c "
import json
rows=[json.loads(l) for l in open('gpurun_out/stamps_w.txt')]
for r in rows[-3:]: print(r['mean_end_by_wave_slot'], r['wave_end_us_pct_0_1_10_50_90_99_100'], r['within_block_range_mean'])
"
