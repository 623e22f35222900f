# which pass (optimistic / full) handles a store; SRD_DEBUG=1 prints the plan,
# SRD_SYNC_DEBUG=1 names a faulting kernel
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-simd-r-drive_amd"))
import torch, srd_amd as S
ctx = S.Context(0)
for n in [int(x) for x in os.environ.get("NS", "3000,200000,2000000").split(",")]:
    lens = S.zipf_lens(n)
    size = S.synth_store_len(n, 4096, lens)
    t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
    S.synth_store_device(t.data_ptr(), n, 4096, lens, seed=0x5EED0004, ctx=ctx)
    torch.cuda.synchronize()
    r = S.validate_index_device(t.data_ptr(), size, 0, ctx)
    print(n, "mode", r.mode, "final", r.final_len == size, "chain", r.n_chain, "cand", r.n_candidates, flush=True)
    del t
