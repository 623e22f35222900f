"""Scan partition A/B inside each context (timing tool; the SRD_DEBUG_API build): every context runs every
weight set in interleaved rounds, so the per-context spread of the scan rate cancels out.
usage: python tools/weights_ab.py name=w0,w1,..  (4 or 16 relative shares) ..."""
import ctypes as C, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRD_LIB_PATH"] = os.path.join(ROOT, "rust-simd-r-drive_amd", "build", "var", "lib_dbg.so")
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import torch
import srd_amd as S
L = S.lib()
L.srd_debug_set_scan_weights.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int]
sets = []
for a in sys.argv[1:]:
    name, _, ws = a.partition("=")
    w = [float(x) for x in ws.split(",")]
    sets.append((name, (C.c_double * len(w))(*w), len(w)))
ctxs = [S.Context(0) for _ in range(int(os.environ.get("NCTX", 3)))]
for c in ctxs:
    c.set_timing(1)
n = 1 << 20
size = S.synth_store_len(n)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, ctx=ctxs[0])
torch.cuda.synchronize()
r = S.DeviceResult()
res = {(i, nm): [] for i in range(len(ctxs)) for nm, _, _ in sets}
for rnd in range(int(os.environ.get("ROUNDS", 8))):
    for i, c in enumerate(ctxs):
        for nm, w, k in sets:
            assert L.srd_debug_set_scan_weights(c.h, w, k) == 0
            for _ in range(5):
                assert L.srd_validate_index_device(c.h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r)) == 0
            assert r.final_len == size and r.n_chain == n and r.n_crc_bad == 0
            a, k2, _ = c.timings()
            if rnd:
                res[(i, nm)].append(a / k2)
for i in range(len(ctxs)):
    print(json.dumps({nm: round(sorted(res[(i, nm)])[len(res[(i, nm)]) // 2], 4) for nm, _, _ in sets}))
