"""Contexts allocated one after another on one C2 store, then each timed in a block of calls
(timing / PMC tool only): run under rocprofv3 --pmc to compare address-translation counters of a slow
(first-allocated) and a fast context.  Prints each context's median scan ms (HIP events)."""
import ctypes as C, json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-simd-r-drive_amd"))
import torch
import srd_amd as S

L = S.lib()
# QUEUE_BURN=k: k torch streams each run a kernel before the contexts' first launches (HW queue assignment)
burn = []
for _ in range(int(os.environ.get("QUEUE_BURN", 0))):
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        burn.append(torch.zeros(1024, device="cuda") + 1)
    burn.append(st)
torch.cuda.synchronize()
nctx = int(os.environ.get("NCTX", 5))
ctxs = [S.Context(0) for _ in range(nctx)]
for c in ctxs:
    c.set_timing(1)
n = 1 << 20
size = S.synth_store_len(n, 4096, None)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, None, seed=0x5EED0001, ctx=ctxs[0])
torch.cuda.synchronize()
r = S.DeviceResult()
for c in ctxs:  # first calls: workspace allocations in order
    assert L.srd_validate_index_device(c.h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r)) == 0
out = {}
for i, c in enumerate(ctxs):
    v = []
    for _ in range(int(os.environ.get("CALLS", 5))):
        assert L.srd_validate_index_device(c.h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r)) == 0
        assert r.final_len == size and r.n_chain == n and (r.n_crc_bad == 0 or os.environ.get('AB_NOCRC'))
        v.append(c.timings()[0])
    out[f"ctx{i}"] = round(sorted(v)[len(v) // 2], 4)
print(json.dumps(out))
