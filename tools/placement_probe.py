"""Scan time vs memory placement (timing tool only): stores and contexts allocated at different points of one
process; every (context, store) pair timed in interleaved rounds.
  S1: torch.empty (the bench's store), S2: hipExtMallocWithFlags(hipDeviceMallocContiguous)
  A, B: first calls (workspace allocations) right after S1; C, D after S2"""
import ctypes as C, json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-simd-r-drive_amd"))
import torch
import srd_amd as S

L = S.lib()
hip = C.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
n = 1 << 20
size = S.synth_store_len(n, 4096, None)
nbytes = S.padded_size(size)


def first_call(ctx, ptr):
    r = S.DeviceResult()
    assert L.srd_validate_index_device(ctx.h, C.c_void_p(ptr), size, 0, C.byref(r)) == 0 and r.final_len == size


ctxs = {}
t1 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
s1 = t1.data_ptr()
for k in ("A", "B"):
    ctxs[k] = S.Context(0)
    ctxs[k].set_timing(1)
S.synth_store_device(s1, n, 4096, None, seed=0x5EED0001, ctx=ctxs["A"])
torch.cuda.synchronize()
for k in ("A", "B"):
    first_call(ctxs[k], s1)
p2 = C.c_void_p()
assert hip.hipExtMallocWithFlags(C.byref(p2), nbytes, int(os.environ.get("S2_FLAGS", 4))) == 0
s2 = p2.value
S.synth_store_device(s2, n, 4096, None, seed=0x5EED0001, ctx=ctxs["A"])
torch.cuda.synchronize()
for k in ("C", "D"):
    ctxs[k] = S.Context(0)
    ctxs[k].set_timing(1)
    first_call(ctxs[k], s2)
stores = {"S1": s1, "S2": s2}
res = {f"{c}{s}": [] for c in ctxs for s in stores}
for rnd in range(int(os.environ.get("ROUNDS", 8))):
    for c, ctx in ctxs.items():
        for s, ptr in stores.items():
            r = S.DeviceResult()
            for _ in range(6):
                assert L.srd_validate_index_device(ctx.h, C.c_void_p(ptr), size, 0, C.byref(r)) == 0
            assert r.final_len == size and r.n_chain == n and r.n_crc_bad == 0
            if rnd >= 1:
                res[f"{c}{s}"].append(ctx.timings()[0])
print(json.dumps({k: round(sorted(v)[len(v) // 2], 4) for k, v in res.items()}))
