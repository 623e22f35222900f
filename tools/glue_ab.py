"""Glue A/B inside each context (timing tool; the SRD_DEBUG_API build): round 0
of the optimistic pass with the shape check fused into chain_finalize_kernel
(look-back ranks, srd_debug_set_glue_fused 1) against check_kernel +
chain_finalize_kernel (0), interleaved per context so the per-context spread
 cancels.  Results are checked against the store's closed form.
usage: python tools/glue_ab.py          env: NCTX, ROUNDS, REPS, CONFIG=c2|c3"""
import ctypes as C, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRD_LIB_PATH"] = os.path.join(ROOT, "rust-simd-r-drive_amd", "build", "var", "lib_dbg.so")
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import torch
import srd_amd as S
L = S.lib()
L.srd_debug_set_glue_fused.argtypes = [C.c_void_p, C.c_int]
cfg = os.environ.get("CONFIG", "c2")
ctxs = [S.Context(0) for _ in range(int(os.environ.get("NCTX", 3)))]
for c in ctxs:
    c.set_timing(S.TIMING_SCAN)
if cfg == "c3":
    n, lens, seed = 10_000_000, S.zipf_lens(10_000_000), 0x5EED0004
else:
    n, lens, seed = 1 << 20, None, 0x5EED0001
size = S.synth_store_len(n, 4096, lens)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, lens, seed=seed, ctx=ctxs[0])
torch.cuda.synchronize()
r = S.DeviceResult()
modes = [0, 1]
reps = int(os.environ.get("REPS", 20))
call = {(i, m): [] for i in range(len(ctxs)) for m in modes}
glue = {(i, m): [] for i in range(len(ctxs)) for m in modes}
for rnd in range(int(os.environ.get("ROUNDS", 8))):
    for i, c in enumerate(ctxs):
        for m in modes:
            assert L.srd_debug_set_glue_fused(c.h, m) == 0
            c.timings()
            t0 = time.perf_counter()
            for _ in range(reps):
                assert L.srd_validate_index_device(c.h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r)) == 0
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps * 1e3
            assert (r.final_len, r.n_chain, r.n_index, r.n_crc_bad, r.mode) == (size, n, n, 0, 0), (m, r.n_chain, r.mode)
            a, k, _ = c.timings()
            if rnd:
                call[(i, m)].append(dt)
                glue[(i, m)].append(dt - a / k)  # call wall time - the scan kernel
med = lambda x: sorted(x)[len(x) // 2]
out = {"config": cfg, "reps": reps, "per_ctx": [{f"fused{m}": {"call_med": round(med(call[(i, m)]), 4),
                                                               "call_min": round(min(call[(i, m)]), 4),
                                                               "call_minus_scan_med": round(med(glue[(i, m)]), 4)}
                                                  for m in modes} for i in range(len(ctxs))]}
out["fused_vs_unfused_us"] = {"call": [round(1e3 * (med(call[(i, 1)]) - med(call[(i, 0)])), 1) for i in range(len(ctxs))],
                              "call_minus_scan": [round(1e3 * (med(glue[(i, 1)]) - med(glue[(i, 0)])), 1)
                                                  for i in range(len(ctxs))]}
print(json.dumps(out, indent=1))
