"""Host overhead probe, Python side of tools/c_loop.c (timing tool): the bench's call path
(srd_amd.validate_index_device) in a loop, timing level 0 and 1 alternating inside one context."""
import json, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-simd-r-drive_amd"))
import torch
import srd_amd as S
ctx = S.Context(0)
n = 1 << 20
size = S.synth_store_len(n, 4096, None)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, None, seed=0x5EED0001, ctx=ctx)
torch.cuda.synchronize()
wall, cnt, scan, sl = [0.0, 0.0], [0, 0], 0.0, 0
ptr = t.data_ptr()
for rnd in range(12):
    for lvl in (0, 1):
        ctx.set_timing(lvl)
        for _ in range(3):
            S.validate_index_device(ptr, size, 0, ctx)
        ctx.timings()
        t0 = time.perf_counter()
        for _ in range(20):
            r = S.validate_index_device(ptr, size, 0, ctx)
            got = r.final_len, r.n_chain, r.n_crc_bad, r.n_index, r.mode  # what bench.py's step reads
        dt = (time.perf_counter() - t0) * 1e3
        assert got == (size, n, 0, n, 0)
        if rnd:
            wall[lvl] += dt
            cnt[lvl] += 20
        if lvl == 1:
            s, k, _ = ctx.timings()
            if rnd:
                scan += s
                sl += k
print(json.dumps({"py_wall_ms_per_call_level0": round(wall[0] / cnt[0], 4), "py_wall_ms_per_call_level1": round(wall[1] / cnt[1], 4),
                  "scan_ms_events": round(scan / sl, 4)}))
