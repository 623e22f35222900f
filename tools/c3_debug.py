import os, sys
sys.path.insert(0, "rust-simd-r-drive_amd")
import torch, srd_amd as S
n = 10_000_000
lens = S.zipf_lens(n)
size = S.synth_store_len(n, 4096, lens)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
ctx = S.Context(0)
S.synth_store_device(t.data_ptr(), n, 4096, lens, seed=0x5EED0004, ctx=ctx)
torch.cuda.synchronize()
for _ in range(2):
    r = S.validate_index_device(t.data_ptr(), size, 0, ctx)
    print(r.n_chain, r.mode, r.n_candidates, flush=True)
