"""(Experiment reverted: srd_debug_xcd is gone from the library; kept as the record of the measurement.)
Per-XCD block weights, A/B inside each context (timing tool; the SRD_DEBUG_API build): the weights learn
over LEARN calls (adaptive), then rounds alternate the learned weights and the even split, both held fixed."""
import ctypes as C, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRD_LIB_PATH"] = os.path.join(ROOT, "rust-simd-r-drive_amd", "build", "var", "lib_dbg.so")
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import torch
import srd_amd as S
L = S.lib()
D8 = C.c_double * 8
L.srd_debug_xcd.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
ctxs = [S.Context(0) for _ in range(int(os.environ.get("NCTX", 3)))]
for c in ctxs:
    c.set_timing(1)
n = 1 << 20
size = S.synth_store_len(n)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, ctx=ctxs[0])
torch.cuda.synchronize()
r = S.DeviceResult()


def run(c, k):
    for _ in range(k):
        assert L.srd_validate_index_device(c.h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r)) == 0
    assert r.final_len == size and r.n_chain == n and r.n_crc_bad == 0
    a, m, _ = c.timings()
    return a / m


learned, trace = [], []
for c in ctxs:
    tr = []
    for _ in range(int(os.environ.get("LEARN", 6))):
        tr.append(round(run(c, 5), 4))
    w = D8()
    L.srd_debug_xcd(c.h, C.addressof(w), None, 1)
    learned.append(D8(*w))
    trace.append(tr)
even = D8(*([1.0] * 8))
res = {(i, k): [] for i in range(len(ctxs)) for k in ("learned", "even")}
for rnd in range(int(os.environ.get("ROUNDS", 8))):
    for i, c in enumerate(ctxs):
        for k, w in (("learned", learned[i]), ("even", even)):
            L.srd_debug_xcd(c.h, None, C.addressof(w), 1)
            v = run(c, 5)
            if rnd:
                res[(i, k)].append(v)
for i in range(len(ctxs)):
    print(json.dumps({"ctx": i, "learn_trace": trace[i], "weights": [round(x, 3) for x in learned[i]],
                      **{k: round(sorted(res[(i, k)])[len(res[(i, k)]) // 2], 4) for k in ("learned", "even")}}))
