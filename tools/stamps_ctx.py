"""Slow vs fast contexts from the inside (timing tool): the SRD_WAVE_STAMPS build on NCTX contexts allocated in
order; for each context's last call, the scan's event duration next to its in-kernel span (first block start ->
the last block's epilogue end, s_memrealtime) and wave-end percentiles."""
import ctypes as C, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRD_LIB_PATH"] = os.path.join(ROOT, "rust-simd-r-drive_amd", "build", "var", "lib_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import numpy as np
import torch
import srd_amd as S
L = S.lib()
nctx = int(os.environ.get("NCTX", 5))
ctxs = [S.Context(0) for _ in range(nctx)]
for c in ctxs:
    c.set_timing(1)
n = 1 << 20
size = S.synth_store_len(n)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, ctx=ctxs[0])
torch.cuda.synchronize()
r = S.DeviceResult()
for c in ctxs:
    assert L.srd_validate_index_device(c.h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r)) == 0
for rnd in range(3):
    for i, c in enumerate(ctxs):
        for _ in range(4):
            assert L.srd_validate_index_device(c.h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r)) == 0
        ev = c.timings()[0]
        st = np.zeros(8192 + 1024, np.uint64)
        assert L.srd_debug_wave_stamps(C.c_void_p(st.ctypes.data)) == 0
        t0 = st[8192:8192 + 256].astype(np.int64).min()
        we = (st[:4096].astype(np.int64) - t0) / 100.0
        epi = (int(st[8192 + 1023]) - t0) / 100.0
        ld = (st[8192 + 256:8192 + 512].astype(np.int64) - t0) / 100.0
        print(json.dumps({"round": rnd, "ctx": i, "event_ms": round(ev, 4), "in_kernel_us": round(epi, 1),
                          "tables_loaded_us_max": round(float(ld.max()), 1),
                          "wave_end_us_pct_0_50_100": [round(float(x), 1) for x in np.percentile(we, [0, 50, 100])]}))
