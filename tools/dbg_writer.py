# debugging aid: per-entry diff of the GPU batch writer against the oracle writer
import os, random, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rust-simd-r-drive_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import srd_amd as S, oracle as O
from test_writer import rand_batch, ref_layout, oracle_write

ctx = S.Context(0)
rng = random.Random(1)
keys, pays = rand_batch(rng, 300)
nt, out, kh, mo = S.batch_write(keys, pays, 0, False, ctx)
want_nt, want, want_kh = oracle_write(0, keys, pays, False)
tails, mos, _ = ref_layout(0, pays, False)
nbad = 0
for i in range(len(pays)):
    m = mos[i]
    st = m - len(pays[i])
    a, b = out[tails[i]:m + 20], want[tails[i]:m + 20]
    if a != b or kh[i] != want_kh[i]:
        nbad += 1
        if nbad <= 12:
            pay_ok = out[st:m] == want[st:m]
            print(f"entry {i}: len {len(pays[i])} klen {len(keys[i])} pay_ok {pay_ok} kh {kh[i]:x} want {want_kh[i]:x} "
                  f"crc got {out[m+16:m+20].hex()} want {want[m+16:m+20].hex()} pad_ok {out[tails[i]:st]==want[tails[i]:st]}")
print("bad", nbad, "of", len(pays))
