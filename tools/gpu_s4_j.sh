# Session 4: the PMC counter list of gfx950 (looking for address-translation counters)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/counters_list.txt 2>&1 || true
grep -i -E "utcl|tlb|translat|UTC" gpurun_out/counters_list.txt | head -60
wc -l gpurun_out/counters_list.txt
