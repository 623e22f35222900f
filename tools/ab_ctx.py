"""A/B of per-context settings of ONE library build in one process (timing tool only).
usage: python tools/ab_ctx.py 'name:ENV=VAL,ENV2=VAL2@level' ...
Each variant gets its own srd_ctx created with the given environment (e.g.
SRD_SCAN_WEIGHTS, read at srd_ctx_create) and timing level (default 1: the
scan's events).  Rounds alternate the variants on the C2 store; prints the
median scan ms (HIP events), wall ms per call (Python loop, REPS calls) and
the minimum."""
import ctypes as C, json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-simd-r-drive_amd"))
import torch
import srd_amd as S

L = S.lib()
n = int(os.environ.get("N_ENTRIES", 1 << 20))
size = S.synth_store_len(n, 4096, None)
t = None
if os.environ.get("STORE_FIRST"):  # the store allocated before any context exists
    t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
variants = []
for spec in sys.argv[1:]:
    name, _, rest = spec.partition(":")
    envs, _, lvl = rest.partition("@")
    saved = {}
    for kv in filter(None, envs.split(",,")):
        k, _, v = kv.partition("=")
        saved[k] = os.environ.get(k)
        os.environ[k] = v
    ctx = S.Context(0)
    ctx.set_timing(int(lvl or 1))
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    variants.append((name, ctx))
if t is None:
    t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, None, seed=0x5EED0001, ctx=variants[0][1])
torch.cuda.synchronize()
print(f"store ptr {t.data_ptr():#x} bytes {t.numel()}", file=sys.stderr)
reps = int(os.environ.get("REPS", 10))
# BIND_ORDER=reverse|forward: a kernel on every context's stream (its HW queue binding) before any first call
if os.environ.get("BIND_ORDER"):
    keep = []
    for name, ctx in (variants[::-1] if os.environ["BIND_ORDER"] == "reverse" else variants):
        es = torch.cuda.ExternalStream(ctx.stream)
        with torch.cuda.stream(es):
            keep.append(torch.zeros(1024, device="cuda") + 1)
        es.synchronize()
# FIRST_ORDER=reverse: the contexts' first calls (their workspace allocations) in reverse order
first = variants[::-1] if os.environ.get("FIRST_ORDER") == "reverse" else variants
for name, ctx in first:
    if os.environ.get("PAD_MB"):  # a device allocation between the contexts' workspaces
        globals().setdefault("_pads", []).append(torch.empty(int(os.environ["PAD_MB"]) << 20, dtype=torch.uint8, device="cuda"))
    r = S.DeviceResult()
    assert L.srd_validate_index_device(ctx.h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r)) == 0
res = {v[0]: {"scan": [], "wall": []} for v in variants}
for rnd in range(int(os.environ.get("ROUNDS", 14))):
    for name, ctx in variants:
        r = S.DeviceResult()
        scan = 0.0
        t0 = time.perf_counter()
        for _ in range(reps):
            rc = L.srd_validate_index_device(ctx.h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r))
        wl = (time.perf_counter() - t0) / reps * 1e3
        a, k, _ = ctx.timings()
        assert rc == 0 and r.final_len == size and r.n_crc_bad == 0 and r.n_chain == n, (name, rc)
        if rnd >= 2:
            res[name]["scan"].append(a / max(k, 1))
            res[name]["wall"].append(wl)


def med(v):
    return round(sorted(v)[len(v) // 2], 4) if v else None


print(json.dumps({k: [round(x, 3) for x in v["scan"]] for k, v in res.items()}), file=sys.stderr)
print(json.dumps({k: {"scan_ms_med": med(v["scan"]), "scan_ms_min": round(min(v["scan"]), 4) if v["scan"] else None,
                      "wall_ms_med": med(v["wall"]), "wall_ms_min": round(min(v["wall"]), 4)}
                  for k, v in res.items()}, indent=0))
