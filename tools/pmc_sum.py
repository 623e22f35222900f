"""Summarise rocprofv3 --pmc CSVs per kernel (mean over dispatches); scan
kernel metrics also per 4 KiB tile of the C2 store."""
import csv, glob, sys, collections
TILES = (4362076116 + 4095) // 4096
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0]
            acc[k][(row["Counter_Name"], row["Dispatch_Id"])].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    per = collections.defaultdict(list)
    for (name, disp), vals in cs.items():
        per[name].append(sum(vals))
    mean = {n: sum(v) / len(v) for n, v in per.items()}
    if "scan_kernel" in k:
        print("==", k)
        for n, v in sorted(mean.items()):
            extra = f"  per_tile={v / TILES:.1f}" if n.startswith("SQ_") else ""
            if n in ("FETCH_SIZE", "WRITE_SIZE"):
                extra = f"  (KB) -> x1024 = {v * 1024 / 1e9:.3f} GB"
            print(f"  {n:24s} {v:16.1f}{extra}")
    elif any(n in mean for n in ("FETCH_SIZE", "WRITE_SIZE")):
        print(f"-- {k[:60]:60s} " + " ".join(f"{n}={mean[n]:.0f}" for n in ("FETCH_SIZE", "WRITE_SIZE") if n in mean))
