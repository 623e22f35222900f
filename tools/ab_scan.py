"""A/B timing of scan-kernel variants in ONE process (timing tool only).
usage: python tools/ab_scan.py lib1.so lib2.so[@level] ...   (interleaved rounds;
@level = srd_ctx_set_timing level, default 2: scan + whole-call events)"""
import ctypes as C, json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-simd-r-drive_amd"))
import torch
import srd_amd as S

libs = sys.argv[1:]
handles = []
for p in libs:
    path, _, lvl = p.partition("@")
    L = C.CDLL(os.path.abspath(path))
    L.srd_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.srd_validate_index_device.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.POINTER(S.DeviceResult)]
    L.srd_ctx_timings.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_double)]
    h = C.c_void_p()
    assert L.srd_ctx_create(0, C.byref(h)) == 0
    if hasattr(L, "srd_ctx_set_timing"):
        L.srd_ctx_set_timing.argtypes = [C.c_void_p, C.c_int]
        assert L.srd_ctx_set_timing(h, int(lvl or 2)) == 0
    handles.append((L, h))
ctx = S.Context(0)
c3 = os.environ.get("CONFIG") == "c3"  # C3: 10M Zipf-sized entries
n = int(os.environ.get("N_ENTRIES", 10_000_000 if c3 else 1 << 20))
lens = S.zipf_lens(n) if c3 else None
size = S.synth_store_len(n, 4096, lens)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, lens, seed=0x5EED0004 if c3 else 0x5EED0001, ctx=ctx)
torch.cuda.synchronize()
res = {p: [] for p in libs}
tot = {p: [] for p in libs}
wall = {p: [] for p in libs}
for rnd in range(int(os.environ.get('ROUNDS', 12))):
    for p, (L, h) in zip(libs, handles):
        r = S.DeviceResult()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            rc = L.srd_validate_index_device(h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r))
        wl = (time.perf_counter() - t0) / reps * 1e3
        a, k, b = C.c_double(), C.c_int(), C.c_double()
        L.srd_ctx_timings(h, C.byref(a), C.byref(k), C.byref(b))
        if not os.environ.get("AB_NOCHECK") or "noslow" not in p:  # timing-only variants may be wrong
            assert rc == 0 and r.final_len == size and r.n_crc_bad == 0 and r.n_chain == n, (p, rc, r.final_len, r.n_crc_bad)
        if rnd >= 2:
            res[p].append(a.value / max(k.value, 1))
            tot[p].append(b.value)
            wall[p].append(wl)
out = {os.path.basename(p.partition("@")[0]) + (("@" + p.partition("@")[2]) if "@" in p else ""): {"scan_ms_min": round(min(v), 4), "scan_ms_med": round(sorted(v)[len(v) // 2], 4),
                             "total_ms_med": round(sorted(tot[p])[len(v) // 2], 4),
                             "wall_ms_med": round(sorted(wall[p])[len(v) // 2], 4),
                             "wall_ms_min": round(min(wall[p]), 4)} for p, v in res.items()}
print(json.dumps(out, indent=0))
