"""Write profiles/traffic.json from two rocprofv3 --pmc passes of the C2 bench
(tools/gpu_pmc.sh: pmc_c = FETCH_SIZE, pmc_d = WRITE_SIZE), tagged with the
sha256 of the kernel sources it measured (bench.py reports `traffic` only for
those sources).  FETCH_SIZE x2 per MI355X_MICROARCH.md (gfx950 counts half
the bytes of a 16 B/lane streaming read); WRITE_SIZE as is (KB -> x1024).

usage: python tools/traffic_json.py gpurun_out/pmc_c gpurun_out/pmc_d [out.json]"""
import collections
import csv
import datetime
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import kernel_sources_hash  # noqa: E402


def per_kernel(d, counter):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter:
                acc[row["Kernel_Name"].split("(")[0]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in acc.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles", "traffic.json")
    k = next(n for n in fetch if "scan_kernel" in n)
    fb = int(fetch[k] * 1024 * 2)
    wb = int(write.get(k, 0) * 1024)
    glue = {n: {"read_bytes": int(fetch[n] * 1024 * 2), "write_bytes": int(write.get(n, 0) * 1024)}
            for n in fetch if n != k}
    json.dump({
        "kernel": k,
        "workload": "C2 (1M x 4 KiB, 4362076116 B store)",
        "measured": datetime.date.today().isoformat(),
        "kernel_sources_sha256": kernel_sources_hash(),
        "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/gpu_pmc.sh), mean over dispatches",
        "note_fetch": "gfx950: FETCH_SIZE reports 1/2 of the bytes of a 16 B/lane streaming read -> x2",
        "fetch_bytes_corrected": fb,
        "write_bytes": wb,
        "scan_kernel_hbm_bytes_per_launch": fb + wb,
        "other_kernels": glue,
    }, open(out, "w"), indent=1)
    print(open(out).read())


if __name__ == "__main__":
    main()
