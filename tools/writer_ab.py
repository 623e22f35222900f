"""write_kernel variants A/B'd inside each context (timing tool; the
SRD_DEBUG_API build, `make -C rust-simd-r-drive_amd variant V=dbg
DEFS=-DSRD_DEBUG_API`): the C5 batch (1M x 4 KiB entries, keys
bench-key-{i}) with payloads, keys and entries resident in HBM, as bench.py's
device_resident leg.  Variants 0 (the product kernel, coalesced lanes) and 29 (round 3's lane =
line layout) are checked against the C2 store; 21 (copy alone) and 22 (CRC
alone) are timing-only ablations.  Also times the runtime's
device-to-device copy of the same bytes.
usage: python tools/writer_ab.py [variants, default 0,21,22,29]   env: NCTX (2), ROUNDS (6), REPS (5)"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRD_LIB_PATH"] = os.path.join(ROOT, "rust-simd-r-drive_amd", "build", "var", "lib_dbg.so")
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import torch  # noqa: E402
import srd_amd as S  # noqa: E402

L = S.lib()
L.srd_debug_set_scan_variant.argtypes = [C.c_void_p, C.c_int]
variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,21,22,29").split(",")]
nctx, rounds, reps = int(os.environ.get("NCTX", 2)), int(os.environ.get("ROUNDS", 6)), int(os.environ.get("REPS", 5))
n, PL = 1 << 20, 4096
size = S.synth_store_len(n, PL)
dev = "cuda:0"
ctxs = [S.Context(0) for _ in range(nctx)]
store = torch.empty(S.padded_size(size), dtype=torch.uint8, device=dev)
S.synth_store_device(store.data_ptr(), n, PL, ctx=ctxs[0])
pays = store[: 4160 * n].view(n, 4160)[:, :PL].contiguous()
keys = [b"bench-key-%d" % i for i in range(n)]
kl = np.array([len(k) for k in keys], np.uint64)
ko = np.zeros(n, np.uint64)
ko[1:] = np.cumsum(kl)[:-1]
kbytes = torch.frombuffer(bytearray(b"".join(keys)), dtype=torch.uint8)
lens = np.full(n, PL, np.uint64)
offs = np.arange(n, dtype=np.uint64) * PL
ents = (S.WriteEntry * n)()
nt = C.c_uint64()
S._check(L.srd_batch_layout(0, None, S._ptr(ko), S._ptr(kl), S._ptr(offs), S._ptr(lens), n, 0,
                            C.cast(ents, C.c_void_p), C.byref(nt)))
d_ent = torch.frombuffer(bytearray(bytes(ents)), dtype=torch.uint8).to(dev)
d_keys = kbytes.to(dev)
d_kh = torch.empty(n, dtype=torch.int64, device=dev)
d_mo = torch.empty(n, dtype=torch.int64, device=dev)
out = torch.empty(size + 64, dtype=torch.uint8, device=dev)
torch.cuda.synchronize()


def run(c, k):
    for _ in range(k):
        S._check(L.srd_batch_write_device(c.h, C.c_void_p(d_keys.data_ptr()), C.c_void_p(pays.data_ptr()),
                                          C.c_void_p(d_ent.data_ptr()), n, C.c_void_p(out.data_ptr()), 0,
                                          C.c_void_p(d_kh.data_ptr()), C.c_void_p(d_mo.data_ptr()),
                                          C.c_void_p(c.stream)))


res = {(i, v): [] for i in range(nctx) for v in variants}
for rnd in range(rounds):
    for i, c in enumerate(ctxs):
        st = torch.cuda.ExternalStream(c.stream, device=dev)
        for v in variants:
            assert L.srd_debug_set_scan_variant(c.h, v) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                e0.record()
                run(c, reps)
                e1.record()
            torch.cuda.synchronize()
            if v in (0, 29):
                assert torch.equal(out[:size], store[:size]), "variant 0 output differs from the C2 store"
            if rnd:
                res[(i, v)].append(e0.elapsed_time(e1) / reps)
# reference: the same bytes moved by the runtime's device-to-device copy
# (torch copy_: read 4.36 GB + write 4.36 GB, no CRC, no layout)
cp = []
for rnd in range(rounds):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        out[:size].copy_(store[:size])
    e1.record()
    torch.cuda.synchronize()
    if rnd:
        cp.append(e0.elapsed_time(e1) / reps)
med = lambda x: sorted(x)[len(x) // 2]
o = {"workload": "C5 write_kernel, inputs in HBM (1M x 4 KiB)", "per_ctx": [],
     "d2d_copy_same_bytes_ms": {"ms_med": round(med(cp), 4), "ms_min": round(min(cp), 4)}}
for i in range(nctx):
    o["per_ctx"].append({f"v{v}": {"ms_med": round(med(res[(i, v)]), 4), "ms_min": round(min(res[(i, v)]), 4)}
                         for v in variants})
print(json.dumps(o, indent=1))
