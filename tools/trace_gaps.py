"""Per-step kernel timeline from a rocprofv3 kernel trace (timing tool only):
python tools/trace_gaps.py <run_kernel_trace.csv> [n_steps]"""
import csv, sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
seqs, cur = [], None
for r in rows:
    n = r['Kernel_Name']
    if 'scan_kernel' in n:
        cur = []
        seqs.append(cur)
    if cur is not None:
        cur.append((n.split('(')[0].replace('void ', '').replace('srd::', '')[:28], int(r['Start_Timestamp']),
                    int(r['End_Timestamp'])))
for s in seqs[-int(sys.argv[2]) if len(sys.argv) > 2 else -2:]:
    t0, prev = s[0][1], None
    for n, a, b in s:
        print(f"{n:30s} start {(a - t0) / 1e3:8.1f} dur {(b - a) / 1e3:7.1f} gap {((a - prev) / 1e3 if prev else 0):6.1f}")
        prev = b
    print('--')
st = [s[0][1] for s in seqs]
en = [s[-1][2] for s in seqs]
print('scan-to-scan us:', [round((st[i + 1] - st[i]) / 1e3, 1) for i in range(len(st) - 1)])
print('end-to-next-scan us:', [round((st[i + 1] - en[i]) / 1e3, 1) for i in range(len(st) - 1)])
