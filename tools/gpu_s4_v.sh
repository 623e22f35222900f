# Session 4: bucket-fill counter stride (device-scope claim atomics) -- glue kernel durations by rocprof, per build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in prod bf16 bf32 prod bf16 bf32; do
  if [ $v = prod ]; then unset SRD_LIB_PATH; else export SRD_LIB_PATH=$PWD/rust-simd-r-drive_amd/build/var/lib_$v.so; fi
  rm -rf gpurun_out/prof_v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_v -o run -- python3 bench.py --no-cpu --steps 20 > gpurun_out/prof_v.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_v.log; exit 1; }
  f=$(find gpurun_out/prof_v -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
d = {r["Name"].split("(")[0].replace("void ", "").replace("srd::", ""): round(float(r["AverageNs"]) / 1e3, 1) for r in csv.DictReader(open(sys.argv[1]))}
print(sys.argv[2], {k: d[k] for k in d if "synth" not in k and "fill" not in k})
PY
done
