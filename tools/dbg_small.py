import os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, "rust-simd-r-drive_amd"); sys.path.insert(0, "oracle")
import json, numpy as np
import srd_amd as S, oracle as O
os.environ["SRD_DEBUG"] = "1"
cases = json.load(open("tests/golden/cases.json"))
for m in cases[:8] if isinstance(cases, list) else list(cases.values())[:8]:
    data = open(os.path.join("tests/golden", m["file"]), "rb").read()
    r = S.validate_index(np.frombuffer(data, np.uint8))
    print(m["file"], r.final_len, m["final_len"], r.n_chain, r.n_index, len(m["index"]), flush=True)
