# Session 4: slow first contexts -- are the per-tile value stores (4 KiB-strided wave regions) the cause?
# NOTILE: timing-only build whose scan drops those stores; 6 contexts allocated in order, interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in prod notile prod notile; do
  if [ $v = notile ]; then export SRD_LIB_PATH=$PWD/rust-simd-r-drive_amd/build/var/lib_notile.so AB_NOCRC=1; else unset SRD_LIB_PATH AB_NOCRC; fi
  NCTX=6 CALLS=7 timeout -k 10 120 python tools/tlb_probe.py > gpurun_out/nt.json 2>gpurun_out/nt.err || { echo NT_FAIL; tail gpurun_out/nt.err; exit 1; }
  echo "$v $(cat gpurun_out/nt.json)"
done
