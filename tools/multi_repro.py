"""Debug aid: srd_validate_index_multi over each golden fixture with N contexts, printing progress."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-simd-r-drive_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np
import srd_amd as S
from conftest import load_cases
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
flags = int(sys.argv[2]) if len(sys.argv) > 2 else 0
cs = [S.Context(0) for _ in range(n)]
for name, (data, m) in load_cases().items():
    a = np.frombuffer(data, np.uint8) if data else np.zeros(0, np.uint8)
    print(name, a.size, S.shard_cuts(a, n), flush=True)
    r = S.validate_index_multi(a, cs, flags)
    print("  ->", r.final_len, r.n_chain, r.n_index, r.mode, "want", m["final_len"], flush=True)
print("repro ok", flush=True)
