"""Per-XCD scan timing across contexts (timing tool; the stamps build,
`make -C rust-simd-r-drive_amd variant V=stamps DEFS=-DSRD_WAVE_STAMPS`).
Each scan block records its start, its waves' ends and the PHYSICAL XCD it
ran on (s_getreg HW_REG_XCC_ID).  For NCTX contexts x CALLS calls on one C2
store: the blockIdx -> XCD map (as the rotation of blockIdx % 8), the mean
block duration per physical XCD, and the scan time (first block start ->
last wave end) -- does a context's scan time follow the map, and is a
physical XCD's speed stable across contexts?"""
import ctypes as C, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRD_LIB_PATH"] = os.path.join(ROOT, "rust-simd-r-drive_amd", "build", "var", "lib_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import numpy as np
import torch
import srd_amd as S
L = S.lib()
nctx, calls = int(os.environ.get("NCTX", 4)), int(os.environ.get("CALLS", 6))
ctxs = [S.Context(0) for _ in range(nctx)]
n = 1 << 20
size = S.synth_store_len(n)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, ctx=ctxs[0])
torch.cuda.synchronize()
rows, blocks = [], []
for rnd in range(calls):
    for ci, c in enumerate(ctxs):
        r = S.validate_index_device(t.data_ptr(), size, 0, c)
        assert r.final_len == size and r.n_chain == n
        st = np.zeros(8192 + 1024, np.uint64)
        assert L.srd_debug_wave_stamps(C.c_void_p(st.ctypes.data)) == 0
        start = st[8192:8192 + 256].astype(np.int64)
        raw = st[8192 + 512:8192 + 768]
        xcc = (raw & np.uint64(0xFFFFFFFF)).astype(np.int64)
        hwid = (raw >> np.uint64(32)).astype(np.int64)
        wend = st[:4096].astype(np.int64).reshape(256, 16).max(1)
        blocks.append({"ctx": ci, "call": rnd, "xcc": xcc.tolist(), "hwid": hwid.tolist(),
                       "dur": ((wend - start) / 100.0).round(1).tolist(), "start": ((start - start.min()) / 100.0).round(1).tolist()})
        t0 = start.min()
        dur = (wend - start) / 100.0  # us
        end = (wend - t0) / 100.0
        rot = [int(x) for x in xcc[:8]]
        per_xcc = {int(x): round(float(dur[xcc == x].mean()), 1) for x in sorted(set(xcc.tolist()))}
        end_xcc = {int(x): round(float(end[xcc == x].max()), 1) for x in sorted(set(xcc.tolist()))}
        consistent = all(int(xcc[b]) == rot[b % 8] for b in range(256))
        rows.append({"ctx": ci, "call": rnd, "scan_us": round(float(end.max()), 1), "xcc_of_block_0_7": rot,
                     "map_is_rotation_mod8": consistent, "mean_block_us_per_xcc": per_xcc,
                     "last_end_us_per_xcc": end_xcc})
for rw in rows:
    print(json.dumps(rw))
if os.environ.get("DUMP"):
    json.dump(blocks, open(os.environ["DUMP"], "w"))
