"""Timing A/B of the C2 step (timing tool): steps with no events vs the
scan timed by hipExtLaunchKernel events vs marker events (SRD_SCAN_MARKER_EVENTS
is read once per process, so each mode runs in its own subprocess)."""
import json, os, subprocess, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
    import torch
    import srd_amd as S
    level = int(sys.argv[2])
    ctx = S.Context(0)
    ctx.set_timing(level)
    n = 1 << 20
    size = S.synth_store_len(n)
    store = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
    S.synth_store_device(store.data_ptr(), n, 4096, ctx=ctx)
    torch.cuda.synchronize()
    out = []
    for rep in range(4):
        for _ in range(5):
            S.validate_index_device(store.data_ptr(), size, 0, ctx)
        t0 = time.perf_counter()
        sm = 0.0
        for _ in range(40):
            r = S.validate_index_device(store.data_ptr(), size, 0, ctx)
            sm += ctx.timings()[0]
        dt = (time.perf_counter() - t0) / 40 * 1e3
        assert r.final_len == size
        out.append((round(dt, 4), round(sm / 40, 4)))
    print(json.dumps({"level": level, "marker": os.environ.get("SRD_SCAN_MARKER_EVENTS", ""), "ms_step_scan": out}))
else:
    for env, level in ((None, 0), (None, 1), ("1", 1), (None, 0), (None, 1)):
        e = dict(os.environ)
        if env:
            e["SRD_SCAN_MARKER_EVENTS"] = env
        print(subprocess.check_output([sys.executable, __file__, "child", str(level)], env=e, text=True).strip(), flush=True)
