"""Two or more builds of the library A/B'd in ONE process on the same device-resident
store (timing tool): NCTX contexts per build, the builds' calls interleaved
round by round, so the per-context spread shows up as spread
within each build instead of as a difference between them.  Every call's
result is checked against the store's closed form.
usage: python tools/lib_ab.py A.so B.so [C.so ...]     env: NCTX (3), ROUNDS (10), REPS (10), CONFIG=c2|c3"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import torch  # noqa: E402
import srd_amd as S  # noqa: E402


def bind(path):
    L = C.CDLL(path)
    L.srd_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.srd_ctx_set_timing.argtypes = [C.c_void_p, C.c_int]
    L.srd_ctx_timings.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_double)]
    L.srd_validate_index_device.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.POINTER(S.DeviceResult)]
    return L


libs = [bind(p) for p in sys.argv[1:]]
names = [os.path.basename(p) for p in sys.argv[1:]]
nctx, rounds, reps = int(os.environ.get("NCTX", 3)), int(os.environ.get("ROUNDS", 10)), int(os.environ.get("REPS", 10))
cfg = os.environ.get("CONFIG", "c2")
if cfg == "c3":
    n, lens, seed = 10_000_000, None, 0x5EED0004
    lens = S.zipf_lens(n)
else:
    n, lens, seed = 1 << 20, None, 0x5EED0001
size = S.synth_store_len(n, 4096, lens)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, lens, seed=seed)
torch.cuda.synchronize()
ctxs = []
# contexts created round-robin over the builds (contexts created first have
# run slower in some processes: no build gets all the early ones)
for _ in range(nctx):
    for b, L in enumerate(libs):
        h = C.c_void_p()
        assert L.srd_ctx_create(0, C.byref(h)) == 0
        assert L.srd_ctx_set_timing(h, S.TIMING_SCAN) == 0
        ctxs.append((b, L, h))
r = S.DeviceResult()
wall = {i: [] for i in range(len(ctxs))}
scan = {i: [] for i in range(len(ctxs))}
for rnd in range(rounds):
    for i, (b, L, h) in enumerate(ctxs):
        sm, k, tot = C.c_double(), C.c_int(), C.c_double()
        L.srd_ctx_timings(h, C.byref(sm), C.byref(k), C.byref(tot))
        t0 = time.perf_counter()
        for _ in range(reps):
            assert L.srd_validate_index_device(h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r)) == 0
        dt = (time.perf_counter() - t0) / reps * 1e3
        assert (r.final_len, r.n_chain, r.n_index, r.n_crc_bad, r.mode) == (size, n, n, 0, 0), (names[b], r.n_chain, r.mode)
        L.srd_ctx_timings(h, C.byref(sm), C.byref(k), C.byref(tot))
        if rnd:
            wall[i].append(dt)
            scan[i].append(sm.value / max(k.value, 1))
med = lambda x: sorted(x)[len(x) // 2]
out = {"config": cfg, "builds": names, "per_ctx": []}
for i, (b, L, h) in enumerate(ctxs):
    out["per_ctx"].append({"build": names[b], "call_med": round(med(wall[i]), 4), "call_min": round(min(wall[i]), 4),
                           "scan_med": round(med(scan[i]), 4), "glue_med": round(med(wall[i]) - med(scan[i]), 4)})
for b in range(len(libs)):
    rows = [x for x in out["per_ctx"] if x["build"] == names[b]]
    out[names[b]] = {k: round(sum(x[k] for x in rows) / len(rows), 4) for k in ("call_med", "scan_med", "glue_med")}
print(json.dumps(out, indent=1))
