"""Scan time over a long run of C2 calls in one process (timing tool only): mean of each window of W calls."""
import ctypes as C, json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-simd-r-drive_amd"))
import torch
import srd_amd as S

L = S.lib()
n = 1 << 20
size = S.synth_store_len(n, 4096, None)
ctx = S.Context(0)
ctx.set_timing(1)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, None, seed=0x5EED0001, ctx=ctx)
torch.cuda.synchronize()
W, N = int(os.environ.get("W", 100)), int(os.environ.get("N", 2000))
out, acc, wall0 = [], [], time.perf_counter()
r = S.DeviceResult()
for i in range(N):
    assert L.srd_validate_index_device(ctx.h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r)) == 0
    acc.append(ctx.timings()[0])
    if len(acc) == W:
        out.append(round(sum(acc) / W, 4))
        acc = []
print(json.dumps({"window_means_ms": out, "wall_s": round(time.perf_counter() - wall0, 2)}))
