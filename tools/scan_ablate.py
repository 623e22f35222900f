# timing-only helper: scan-kernel time on the C2 store under SRD_SCAN_ABLATE variants
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-simd-r-drive_amd"))
import torch, srd_amd as S
ctx = S.Context(0)
n = 1 << 20
size = S.synth_store_len(n)
t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
S.synth_store_device(t.data_ptr(), n, 4096, ctx=ctx)
torch.cuda.synchronize()
res = {}
for ab in [int(x) for x in os.environ.get('ABL', '0,1,2,3,4').split(',')]:
    os.environ["SRD_SCAN_ABLATE"] = str(ab)
    ts = []
    for i in range(8):
        try:
            S.validate_index_device(t.data_ptr(), size, 0, ctx)
        except Exception as e:
            pass
        ts.append(ctx.timings()[0] / max(ctx.timings()[1], 1))
    res[ab] = round(min(ts[2:]), 4)
print(json.dumps(res))
