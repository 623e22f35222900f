"""Does re-allocating the buffers the scan writes change a context's scan rate? (timing tool; SRD_DEBUG_API
build) NCTX contexts; measure each; give every context new scan buffers (old ones held, so the new ones land
elsewhere); measure again; repeat."""
import ctypes as C, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRD_LIB_PATH"] = os.path.join(ROOT, "rust-simd-r-drive_amd", "build", "var", "lib_dbg.so")
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import torch
import srd_amd as S
L = S.lib()
L.srd_debug_realloc_scan_bufs.argtypes = [C.c_void_p, C.c_int]
ctxs = [S.Context(0) for _ in range(int(os.environ.get("NCTX", 4)))]
for c in ctxs:
    c.set_timing(1)
n = 1 << 20
size = S.synth_store_len(n)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, ctx=ctxs[0])
torch.cuda.synchronize()
r = S.DeviceResult()


def measure():
    res = {i: [] for i in range(len(ctxs))}
    for rnd in range(5):
        for i, c in enumerate(ctxs):
            for _ in range(5):
                assert L.srd_validate_index_device(c.h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r)) == 0
            assert r.final_len == size and r.n_chain == n and r.n_crc_bad == 0
            a, k, _ = c.timings()
            if rnd:
                res[i].append(a / k)
    return [round(sorted(v)[len(v) // 2], 4) for v in res.values()]


print("initial", measure())
for it in range(3):
    for c in ctxs:
        assert L.srd_debug_realloc_scan_bufs(c.h, 1) == 0
    print("realloc", it + 1, measure())
