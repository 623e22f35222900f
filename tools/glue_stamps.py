"""Where chain_finalize_kernel<true>'s time goes, per block (timing tool): the
SRD_GLUE_STAMPS build (`make -C rust-simd-r-drive_amd variant V=gstamps
DEFS="-DSRD_DEBUG_API -DSRD_GLUE_STAMPS"`) stamps each block's phase ends
with s_memrealtime (100 MHz): 0 start, 1 shape check done, 2 look-back done,
3 tables in LDS, 4 finalize loop done, 5 bucket ranges claimed, 6 end.
Prints, per phase, the median / max over blocks of the time since the
earliest block start (us), over REPS calls on the C2 store (CONFIG=c3: C3)."""
import ctypes as C, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SRD_LIB_PATH"] = os.path.join(ROOT, "rust-simd-r-drive_amd", "build", "var", "lib_gstamps.so")
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))
import numpy as np
import torch
import srd_amd as S
L = S.lib()
L.srd_debug_glue_stamps.argtypes = [C.c_void_p]
ctx = S.Context(0)
cfg = os.environ.get("CONFIG", "c2")  # c3: the 10 M Zipf-sized store
if cfg == "c3":
    n, lens, seed = 10_000_000, None, 0x5EED0004
    lens = S.zipf_lens(n)
else:
    n, lens, seed = 1 << 20, None, 0x5EED0001
size = S.synth_store_len(n, 4096, lens)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, lens, seed=seed, ctx=ctx)
torch.cuda.synchronize()
r = S.DeviceResult()
buf = np.zeros(256 * 8, np.uint64)
rows = []
for rep in range(int(os.environ.get("REPS", 12))):
    assert L.srd_validate_index_device(ctx.h, C.c_void_p(t.data_ptr()), size, 0, C.byref(r)) == 0
    assert (r.final_len, r.n_chain) == (size, n)
    assert L.srd_debug_glue_stamps(buf.ctypes.data_as(C.c_void_p)) == 0
    st = buf.reshape(256, 8).astype(np.int64)
    t0 = st[:, 0].min()
    rows.append((st[:, :7] - t0) / 100.0)  # 100 MHz -> us
a = np.stack(rows[2:])  # reps x blocks x phases
names = ["start", "check", "lookback", "tables", "finalize", "claims", "end"]
out = {nm: {"median_us": round(float(np.median(a[:, :, i])), 2), "max_us": round(float(np.median(a[:, :, i].max(axis=1))), 2)}
       for i, nm in enumerate(names)}
print(json.dumps(out, indent=1))
