# timing-only: scan-kernel ablation matrix for library variants (LIBS="name ..." in build/var)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
V=rust-simd-r-drive_amd/build/var
for L in ${LIBS:-batabl}; do
  echo -n "$L "; SRD_LIB_PATH=$PWD/$V/lib_$L.so ABL=${ABL:-256,257,258,259,260,272,273,274,275} timeout -k 10 120 python tools/scan_ablate.py 2>/dev/null | tail -1 || exit 1
done
