# dump the bytes around given offsets of the C3 store (debug)
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-simd-r-drive_amd"))
import torch, srd_amd as S, numpy as np
ctx = S.Context(0)
n = int(os.environ.get("N", "10000000"))
lens = S.zipf_lens(n)
size = S.synth_store_len(n, 4096, lens)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, lens, seed=0x5EED0004, ctx=ctx)
torch.cuda.synchronize()
r = S.validate_index_device(t.data_ptr(), size, 0, ctx)
print("mode", r.mode)
mo = S.device_to_numpy(r.meta_off, r.n_chain, np.uint64)
for x in [int(v) for v in os.environ.get("OFFS", "").split(",") if v]:
    i = np.searchsorted(mo, x)
    print("m", x, "chain idx", i, "near chain m:", mo[max(i-2,0):i+2].tolist())
    b = t[x - 64: x + 84].cpu().numpy()
    print(" ".join(f"{v:02x}" for v in b[:64])); print(" ".join(f"{v:02x}" for v in b[64:]))
