"""The shader clock during the C2 scan, per scan variant (timing tool): loads the
timing-only build made by `make -C rust-simd-r-drive_amd variant V=stamps
DEFS="-DSRD_WAVE_STAMPS -DSRD_DEBUG_API"`, runs each variant (0 product, 34
line-per-lane, 7 loads only, 8 body only on L2-resident tiles; 7 / 8 through
the scan-only flag, results not checked) and prints, per variant, the scan's
span and each wave's average shader clock: (s_memtime at the wave's end - at
its block's start) / (the same interval on s_memrealtime, 100 MHz).  Tells a
body that runs slower under the HBM stream because the clock drops from one
that stalls at a fixed clock.
usage: python tools/clock_stamps.py [variants, default 0,34,7,8]   env: REPS (5)"""
import ctypes as C, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRD_LIB_PATH"] = os.path.join(ROOT, "rust-simd-r-drive_amd", "build", "var", "lib_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import numpy as np
import torch
import srd_amd as S
L = S.lib()
L.srd_debug_set_scan_variant.argtypes = [C.c_void_p, C.c_int]
variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,34,7,8").split(",")]
SCAN_ONLY = 1 << 30
ctx = S.Context(0)
n = 1 << 20
size = S.synth_store_len(n)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, ctx=ctx)
torch.cuda.synchronize()
r = S.DeviceResult()
out = {}
for v in variants:
    assert L.srd_debug_set_scan_variant(ctx.h, v) == 0
    runs = []
    for rep in range(int(os.environ.get("REPS", 5))):
        fl = SCAN_ONLY if v in (7, 8) else 0
        assert L.srd_validate_index_device(ctx.h, C.c_void_p(t.data_ptr()), size, fl, C.byref(r)) == 0
        if v not in (7, 8):
            assert (r.final_len, r.n_chain, r.n_crc_bad) == (size, n, 0), (v, r.final_len, r.n_chain)
        st = np.zeros(8192 + 1024, np.uint64)
        ck = np.zeros(4096 + 256, np.uint64)
        assert L.srd_debug_wave_stamps(C.c_void_p(st.ctypes.data)) == 0
        assert L.srd_debug_wave_clk(C.c_void_p(ck.ctypes.data)) == 0
        rt_b = st[8192:8192 + 256].astype(np.int64)
        rt_w = st[:4096].astype(np.int64)
        ck_b = ck[4096:4096 + 256].astype(np.int64)
        ck_w = ck[:4096].astype(np.int64)
        blk = np.arange(4096) // 16
        drt = (rt_w - rt_b[blk]) / 100e6           # s
        dck = (ck_w - ck_b[blk]).astype(np.float64)  # shader clocks
        mhz = dck / drt / 1e6
        span_us = (rt_w.max() - rt_b.min()) / 100.0
        if rep:
            runs.append({"span_us": round(float(span_us), 1),
                         "wave_mhz_pct_10_50_90": [round(float(x), 0) for x in np.percentile(mhz, [10, 50, 90])]})
    out[f"v{v}"] = runs
print(json.dumps(out, indent=1))
