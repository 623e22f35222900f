import os, sys
sys.path.insert(0, "rust-simd-r-drive_amd")
import torch, srd_amd as S
ctx = S.Context(0)
for n in (1 << 20, 1000):
    size = S.synth_store_len(n)
    t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
    S.synth_store_device(t.data_ptr(), n, 4096, ctx=ctx)
    torch.cuda.synchronize()
    os.environ["SRD_DEBUG"] = "1"
    r = S.validate_index_device(t.data_ptr(), size, 0, ctx)
    print(n, r.final_len, r.n_chain, flush=True)
