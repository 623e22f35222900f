"""Scan-variant A/B inside each context (timing tool; the SRD_DEBUG_API build,
`make -C rust-simd-r-drive_amd variant V=dbg DEFS=-DSRD_DEBUG_API`): every
context runs every variant (srd_debug_set_scan_variant) in interleaved rounds,
so the per-context spread of the scan rate cancels out.  Each
variant's results are checked against the store's closed form every batch.
usage: python tools/variant_ab.py [variants: 0 (product), 34 (line-per-lane loads), 7! / 8! (memory-only / compute-only ablations); default 0,34]   env: NCTX, ROUNDS, CONFIG=c2|c3|c2torn, N (entries)"""
import ctypes as C, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRD_LIB_PATH"] = os.path.join(ROOT, "rust-simd-r-drive_amd", "build", "var", "lib_dbg.so")
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import torch
import srd_amd as S
L = S.lib()
L.srd_debug_set_scan_variant.argtypes = [C.c_void_p, C.c_int]
# "7!": a timing-only ablation -- the optimistic scan alone (the library's
# debug scan-only flag), results not checked
spec = (sys.argv[1] if len(sys.argv) > 1 else "0,34").split(",")
variants = [int(v.rstrip("!")) for v in spec]
timing_only = {int(v.rstrip("!")) for v in spec if v.endswith("!")}
SCAN_ONLY = 1 << 30
cfg = os.environ.get("CONFIG", "c2")
ctxs = [S.Context(0) for _ in range(int(os.environ.get("NCTX", 3)))]
for c in ctxs:
    c.set_timing(S.TIMING_SCAN)
if cfg == "c3":
    n = int(os.environ.get("N", 10_000_000))  # N: a smaller / larger C3-shaped store
    lens = S.zipf_lens(n)
    seed = 0x5EED0004
else:
    n, lens, seed = int(os.environ.get("N", 1 << 20)), None, 0x5EED0001  # N: C2-shaped stores of other sizes
size = S.synth_store_len(n, 4096, lens)
flen = size + (7 if cfg == "c2torn" else 0)
t = torch.empty(S.padded_size(flen), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, lens, seed=seed, ctx=ctxs[0])
if cfg == "c2torn":
    t[size:flen].copy_(torch.frombuffer(bytearray(b"CORRUPT"), dtype=torch.uint8))
torch.cuda.synchronize()
r = S.DeviceResult()
scan = {(i, v): [] for i in range(len(ctxs)) for v in variants}
wall = {(i, v): [] for i in range(len(ctxs)) for v in variants}
reps = 5
for rnd in range(int(os.environ.get("ROUNDS", 8))):
    for i, c in enumerate(ctxs):
        for v in variants:
            assert L.srd_debug_set_scan_variant(c.h, v) == 0
            c.timings()
            t0 = time.perf_counter()
            fl = SCAN_ONLY if v in timing_only else 0
            for _ in range(reps):
                assert L.srd_validate_index_device(c.h, C.c_void_p(t.data_ptr()), flen, fl, C.byref(r)) == 0
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps * 1e3
            if v not in timing_only:
                assert (r.final_len, r.n_chain, r.n_index, r.n_crc_bad, r.mode) == (size, n, n, 0, 0), (v, r.final_len, r.n_chain, r.mode)
            a, k, _ = c.timings()
            if rnd:
                scan[(i, v)].append(a / k)
                wall[(i, v)].append(dt)
med = lambda x: sorted(x)[len(x) // 2]
out = {"config": cfg, "per_ctx": []}
for i in range(len(ctxs)):
    out["per_ctx"].append({f"v{v}": {"scan_med": round(med(scan[(i, v)]), 4), "scan_min": round(min(scan[(i, v)]), 4),
                                     "call_med": round(med(wall[(i, v)]), 4)} for v in variants})
base = variants[0]
for v in variants[1:]:
    rel = [med(scan[(i, v)]) / med(scan[(i, base)]) - 1 for i in range(len(ctxs))]
    relw = [med(wall[(i, v)]) / med(wall[(i, base)]) - 1 for i in range(len(ctxs))]
    out[f"v{v}_vs_v{base}"] = {"scan_pct": [round(100 * x, 2) for x in rel], "call_pct": [round(100 * x, 2) for x in relw]}
print(json.dumps(out, indent=1))
