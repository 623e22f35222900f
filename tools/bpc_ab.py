"""Scan blocks per CU (1 or 2, one resident at a time: the dispatcher hands a free CU the next block of its XCD) inside each context (timing tool; the
SRD_DEBUG_API build, `make -C rust-simd-r-drive_amd variant V=dbg
DEFS=-DSRD_DEBUG_API`): every context alternates REPS calls with the shares
(srd_debug_set_scan_bpc 2) and REPS with 1, ROUNDS rounds, the order flipped
every round, so the per-context spread of the scan cancels.
Every call's result is checked against the store's closed form.
usage: python tools/bpc_ab.py     env: NCTX (4), ROUNDS (8), REPS (10), CONFIG=c2|c3"""
import ctypes as C, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRD_LIB_PATH"] = os.path.join(ROOT, "rust-simd-r-drive_amd", "build", "var", "lib_dbg.so")
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import time
import torch
import srd_amd as S
L = S.lib()
L.srd_debug_set_scan_bpc.argtypes = [C.c_void_p, C.c_int]
nctx, rounds, reps = int(os.environ.get("NCTX", 4)), int(os.environ.get("ROUNDS", 8)), int(os.environ.get("REPS", 10))
cfg = os.environ.get("CONFIG", "c2")
if cfg == "c3":
    n, lens, seed = 10_000_000, S.zipf_lens(10_000_000), 0x5EED0004
else:
    n, lens, seed = 1 << 20, None, 0x5EED0001
size = S.synth_store_len(n, 4096, lens)
ctxs = [S.Context(0) for _ in range(nctx)]
for c in ctxs:
    c.set_timing(S.TIMING_SCAN)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, lens, seed=seed, ctx=ctxs[0])
torch.cuda.synchronize()
res = {(i, on): {"scan": [], "call": []} for i in range(nctx) for on in (0, 1)}
for rnd in range(rounds):
    for i, c in enumerate(ctxs):
        for on in ((1, 0) if rnd % 2 else (0, 1)):
            L.srd_debug_set_scan_bpc(c.h, 2 if on else 1)
            c.timings()
            t0 = time.perf_counter()
            for _ in range(reps):
                r = S.validate_index_device(t.data_ptr(), size, 0, c)
            dt = (time.perf_counter() - t0) / reps * 1e3
            assert (r.final_len, r.n_chain, r.n_index, r.n_crc_bad, r.mode) == (size, n, n, 0, 0)
            a, m, _ = c.timings()
            if rnd:
                res[(i, on)]["scan"].append(a / max(m, 1))
                res[(i, on)]["call"].append(dt)
med = lambda x: sorted(x)[len(x) // 2]
out = {"config": cfg, "per_ctx": []}
for i in range(nctx):
    r0, r1 = res[(i, 0)], res[(i, 1)]
    out["per_ctx"].append({"off_scan": round(med(r0["scan"]), 4), "on_scan": round(med(r1["scan"]), 4),
                           "scan_pct": round(100 * (med(r1["scan"]) / med(r0["scan"]) - 1), 2),
                           "off_call": round(med(r0["call"]), 4), "on_call": round(med(r1["call"]), 4),
                           "call_pct": round(100 * (med(r1["call"]) / med(r0["call"]) - 1), 2)})
print(json.dumps(out, indent=1))
