# Session 4: address-translation counters of slow (first-allocated) vs fast contexts (tools/tlb_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/tlb_probe.py > gpurun_out/tlb_plain.json 2>gpurun_out/tlb.err || { echo PLAIN_FAIL; tail gpurun_out/tlb.err; exit 1; }
cat gpurun_out/tlb_plain.json
rm -rf gpurun_out/pmc_tlb1 gpurun_out/pmc_tlb2
timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_SERIALIZATION_STALL_sum --output-format csv -d gpurun_out/pmc_tlb1 -o run -- python3 tools/tlb_probe.py > gpurun_out/tlb_pmc1.log 2>&1 || { echo PMC1_FAIL; tail gpurun_out/tlb_pmc1.log; exit 1; }
tail -1 gpurun_out/tlb_pmc1.log
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_tlb2 -o run -- python3 tools/tlb_probe.py > gpurun_out/tlb_pmc2.log 2>&1 || { echo PMC2_FAIL; tail gpurun_out/tlb_pmc2.log; exit 1; }
tail -1 gpurun_out/tlb_pmc2.log
python3 - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/pmc_tlb1", "gpurun_out/pmc_tlb2"):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f: print(d, "no csv"); continue
    rows = [r for r in csv.DictReader(open(f[0])) if "scan_kernel" in r.get("Kernel_Name", "")]
    per = collections.OrderedDict()
    for r in rows:
        per.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    ids = list(per)
    print(d, len(ids), "scan dispatches")
    for i in ids:
        print(i, {k: int(v) for k, v in per[i].items()})
PY
