"""Per-wave finish spread of the C2 scan (timing tool): loads the timing-only
build made by `make -C rust-simd-r-drive_amd variant V=stamps DEFS=-DSRD_WAVE_STAMPS`,
runs validate calls and prints, for the last call's scan, the spread of block
start and wave end times (s_memrealtime, 10 ns ticks) relative to the first
block's start."""
import ctypes as C, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRD_LIB_PATH"] = os.path.join(ROOT, "rust-simd-r-drive_amd", "build", "var", "lib_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import numpy as np
import torch
import srd_amd as S
L = S.lib()
ctx = S.Context(0)
n = 1 << 20
size = S.synth_store_len(n)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, ctx=ctx)
out = []
for rep in range(5):
    r = S.validate_index_device(t.data_ptr(), size, 0, ctx)
    assert r.final_len == size
    st = np.zeros(8192 + 1024, np.uint64)
    assert L.srd_debug_wave_stamps(C.c_void_p(st.ctypes.data)) == 0
    blocks = st[8192:8192 + 256].astype(np.int64)
    waves = st[:4096].astype(np.int64)
    t0 = blocks.min()
    we = (waves - t0) / 100.0  # us
    bs = (blocks - t0) / 100.0
    q = np.percentile(we, [0, 1, 10, 50, 90, 99, 100])
    # per-block slowest wave, and per XCD (block % 8)
    bend = we.reshape(256, 16).max(1)
    xcd = [round(float(bend[i::8].mean()), 1) for i in range(8)]
    wv = we.reshape(256, 16)
    ld = (st[8192 + 256:8192 + 512].astype(np.int64) - t0) / 100.0
    bend_all = we.reshape(256, 16).max(1)
    epi = (int(st[8192 + 1023]) - t0) / 100.0
    dbg = None
    if hasattr(L, "srd_debug_wave_dbg"):
        dd = np.zeros(4096 * 4, np.uint64)
        assert L.srd_debug_wave_dbg(C.c_void_p(dd.ctypes.data)) == 0
        dd = dd.reshape(4096, 4).astype(np.int64)
        send = (dd[:, 0] - t0) / 100.0
        dbg = {"static_end_us_pct_0_50_100": [round(float(x), 1) for x in np.percentile(send, [0, 50, 100])],
               "chunks_per_wave_mean_max": [round(float(dd[:, 1].mean()), 2), int(dd[:, 1].max())],
               "claim_us_per_wave_mean_max": [round(float(dd[:, 2].mean() / 100.0), 2), round(float(dd[:, 2].max() / 100.0), 2)]}
    out.append({"dbg": dbg, "block_start_us_max": round(float(bs.max()), 2),
                "tables_loaded_us_pct_50_100": [round(float(np.percentile(ld, 50)), 2), round(float(ld.max()), 2)],
                "block_end_us_pct_0_10_50_90_100": [round(float(x), 1) for x in np.percentile(bend_all, [0, 10, 50, 90, 100])],
                "block_end_mean": round(float(bend_all.mean()), 1),
                "epilogue_end_us": round(epi, 1), "wave_end_us_pct_0_1_10_50_90_99_100": [round(float(x), 1) for x in q],
                "block_end_mean_per_xcd": xcd,
                "mean_end_by_wave_slot": [round(float(x), 1) for x in wv.mean(0)],
                "std_over_blocks_of_slot_mean": round(float(wv.mean(1).std()), 1),
                "within_block_range_mean": round(float((wv.max(1) - wv.min(1)).mean()), 1)})
for o in out:
    print(json.dumps(o))
