cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
V=rust-simd-r-drive_amd/build/var
for L in e1 e2 e3 t3abl r4abl; do
  echo -n "$L "; SRD_LIB_PATH=$PWD/$V/lib_$L.so ABL=256,257,259,272,273,275 timeout -k 10 120 python tools/scan_ablate.py 2>/dev/null | tail -1 || exit 1
done
