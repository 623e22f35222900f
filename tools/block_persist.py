"""Are the scan blocks' speeds persistent across launches? (timing tool; SRD_WAVE_STAMPS build) For K launches,
each block's end (its last wave, us from the first block start); prints the correlation of the per-block ends
between launches and the spread."""
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
ends = []
for rep in range(int(os.environ.get("K", 8))):
    r = S.validate_index_device(t.data_ptr(), size, 0, ctx)
    assert r.final_len == size
    st = np.zeros(8192 + 1024, np.uint64)
    assert L.srd_debug_wave_stamps(C.c_void_p(st.ctypes.data)) == 0
    t0 = st[8192:8192 + 256].astype(np.int64).min()
    we = (st[:4096].astype(np.int64) - t0) / 100.0
    ends.append(we.reshape(256, 16).max(1))
E = np.array(ends)
c = np.corrcoef(E)
off = c[~np.eye(len(E), dtype=bool)]
mean_end = E.mean(0)
print(json.dumps({"corr_between_launches_mean": round(float(off.mean()), 3), "corr_min": round(float(off.min()), 3),
                  "block_end_pct_0_50_100_each": [[round(float(x), 1) for x in np.percentile(e, [0, 50, 100])] for e in E],
                  "mean_over_launches_pct_0_50_100": [round(float(x), 1) for x in np.percentile(mean_end, [0, 50, 100])],
                  "per_xcd_mean": [round(float(mean_end[i::8].mean()), 1) for i in range(8)],
                  "slowest_blocks": [int(i) for i in np.argsort(mean_end)[-8:]]}))
