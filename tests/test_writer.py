"""Checksum-on-append batch writer (BASELINE config C5) --
DataStoreWriter::batch_write / batch_write_with_key_hashes
(data_store.rs:838-939) through the C ABI.

CPU tests: the host layout (srd_batch_layout) against an independent
restatement of the reference's tail arithmetic, and the reference's
InvalidInput errors.  GPU tests: the serialized bytes, key hashes and
metadata offsets bit-exact against the oracle writer (oracle/srd_oracle.c,
orc_write_entries + orc_xxh3_64), and the C5 shape (bench keys, 4 KiB
splitmix64 payloads) byte-identical to the C2 store."""
import random

import numpy as np
import pytest

import oracle as O
import srd_amd as S


def ref_layout(tail, payloads, allow_null):
    """data_store.rs:863-931: (prev tails, metadata offsets, new tail)."""
    tails, mos = [], []
    for p in payloads:
        tails.append(tail)
        if p == b"\x00":
            if not allow_null:
                raise ValueError("NULL-byte payloads cannot be written directly.")
            tail += 1 + 20
        else:
            if not p:
                raise ValueError("Payload cannot be empty.")
            tail += ((64 - tail % 64) & 63) + len(p) + 20
        mos.append(tail - 20)
    return tails, mos, tail


def rand_batch(rng, n, null_frac=0.0):
    keys, pays = [], []
    for i in range(n):
        keys.append(bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 3, 8, 11, 16, 17, 40, 128, 129, 240, 300]))))
        if rng.random() < null_frac:
            pays.append(b"\x00")
        else:
            L = rng.choice([1, 2, 3, 5, 7, 20, 63, 64, 65, 100, 127, 128, 1000, 4095, 4096, 4097, 8191, 12289, 20000])
            pays.append(bytes(rng.getrandbits(8) for _ in range(L)))
    return keys, pays


@pytest.mark.parametrize("tail", [0, 5, 64, 1000003])
def test_layout_matches_reference_arithmetic(tail):
    rng = random.Random(tail)
    keys, pays = rand_batch(rng, 60, null_frac=0.15)
    ents, nt = S.batch_layout(tail, keys, pays, allow_null=True)
    tails, _, want = ref_layout(tail, pays, True)
    assert nt == want
    for i, p in enumerate(pays):
        assert ents[i].tail == tails[i]
        assert ents[i].flags == (1 if p == b"\x00" else 0)
        assert ents[i].len == len(p) and ents[i].key_len == len(keys[i])


def test_layout_errors():
    with pytest.raises(S.SrdError, match="Payload cannot be empty"):
        S.batch_layout(0, [b"k1", b"k2"], [b"abc", b""])
    with pytest.raises(S.SrdError, match="NULL-byte payloads cannot be written directly"):
        S.batch_layout(0, [b"k"], [b"\x00"])
    # with allow_null (the delete path) the NULL byte is a tombstone
    ents, nt = S.batch_layout(0, [b"k"], [b"\x00"], allow_null=True)
    assert ents[0].flags == 1 and nt == 21
    # a zero byte inside a longer payload is data, not a tombstone
    ents, nt = S.batch_layout(0, [b"k"], [b"\x00\x00"])
    assert ents[0].flags == 0 and nt == 22


# ---------------------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def ctx():
    c = S.Context(0)
    yield c
    c.close()


def oracle_write(tail, keys, pays, allow_null, prefix=b""):
    kh = [O.xxh3_64(k) for k in keys]
    buf = bytearray(prefix)
    nt = O.write_entries(buf, tail, list(zip(kh, pays)), allow_null)
    return nt, bytes(buf[tail:nt]), kh


@pytest.mark.gpu
@pytest.mark.parametrize("tail,allow_null,seed", [(0, False, 1), (0, True, 2), (5, True, 3), (4096 + 17, False, 4),
                                                  (1000003, True, 5)])
def test_batch_write_matches_oracle(ctx, tail, allow_null, seed):
    rng = random.Random(seed)
    keys, pays = rand_batch(rng, 300, null_frac=0.1 if allow_null else 0.0)
    nt, out, kh, mo = S.batch_write(keys, pays, tail, allow_null, ctx)
    prefix = bytes(rng.getrandbits(8) for _ in range(tail)) if tail < 5000 else bytes(tail)
    want_nt, want, want_kh = oracle_write(tail, keys, pays, allow_null, prefix)
    assert nt == want_nt
    assert out == want
    assert kh == want_kh
    assert mo == ref_layout(tail, pays, allow_null)[1]


@pytest.mark.gpu
def test_batch_write_errors(ctx):
    with pytest.raises(S.SrdError, match="NULL-byte payloads"):
        S.batch_write([b"a", b"b"], [b"xy", b"\x00"], 0, False, ctx)
    with pytest.raises(S.SrdError, match="Payload cannot be empty"):
        S.batch_write([b"a"], [b""], 0, True, ctx)


@pytest.mark.gpu
def test_batch_write_multi_chunk_unaligned_sources(ctx):
    # > 64 MiB of payload (several chunks through the double-buffered staging),
    # sources at odd offsets inside one blob (the byte path of the kernel)
    import torch
    rng = np.random.default_rng(7)
    n = 9000
    lens = rng.integers(1, 16384, n).astype(np.uint64)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(lens + 3)[:-1]  # 3-byte gaps: unaligned sources
    blob = rng.integers(0, 256, int(offs[-1] + lens[-1]), dtype=np.uint8)
    keys = [b"bench-key-%d" % i for i in range(n)]
    kb = np.frombuffer(b"".join(keys), np.uint8)
    kl = np.array([len(k) for k in keys], np.uint64)
    ko = np.zeros(n, np.uint64)
    ko[1:] = np.cumsum(kl)[:-1]
    tail = 130
    nt0 = tail
    for L in lens:
        nt0 += ((64 - nt0 % 64) & 63) + int(L) + 20
    cap = nt0 - (tail & ~63)
    dev = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    nt, kh, mo = S.batch_write_raw(dev.data_ptr(), cap, tail, kb.ctypes.data, ko, kl, blob.ctypes.data, offs, lens,
                                   0, ctx)
    assert nt == nt0
    pays = [blob[int(o):int(o + L)].tobytes() for o, L in zip(offs, lens)]
    want_nt, want, want_kh = oracle_write(tail, keys, pays, False, bytes(tail))
    got = dev.cpu().numpy().tobytes()[tail - (tail & ~63):]
    assert want_nt == nt and got == want
    assert [int(x) for x in kh] == want_kh


@pytest.mark.gpu
def test_batch_write_c5_shape_equals_c2_store(ctx):
    # C5: bench keys + 4 KiB splitmix64 payloads -> byte-identical to the C2
    # store of the same seeds, checked on a 20000-entry prefix
    import torch
    n = 20000
    size = S.synth_store_len(n)
    store = torch.zeros(S.padded_size(size), dtype=torch.uint8, device="cuda")
    S.synth_store_device(store.data_ptr(), n, 4096, ctx=ctx)
    pays = store[: 4160 * n].view(n, 4160)[:, :4096].contiguous().cpu()
    pin = torch.empty(pays.numel(), dtype=torch.uint8, pin_memory=True)
    pin.copy_(pays.reshape(-1))
    keys = [b"bench-key-%d" % i for i in range(n)]
    kb = np.frombuffer(b"".join(keys), np.uint8)
    kl = np.array([len(k) for k in keys], np.uint64)
    ko = np.zeros(n, np.uint64)
    ko[1:] = np.cumsum(kl)[:-1]
    lens = np.full(n, 4096, np.uint64)
    offs = np.arange(n, dtype=np.uint64) * 4096
    out = torch.zeros(size + 64, dtype=torch.uint8, device="cuda")
    nt, kh, mo = S.batch_write_raw(out.data_ptr(), size + 64, 0, kb.ctypes.data, ko, kl, pin.data_ptr(), offs, lens,
                                   0, ctx)
    torch.cuda.synchronize()
    assert nt == size
    assert torch.equal(out[:size], store[:size])
    assert int(mo[-1]) == size - 20 and int(kh[0]) == O.xxh3_64(b"bench-key-0")


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["gap", "reversed"])
def test_batch_write_device_gapped_and_reordered_tables(ctx, order):
    """srd_batch_write_device on a caller-built entry table whose entries do
    not follow one another: two batches laid out by
    srd_batch_layout at tails 0 and ntA + 1013, the table [A, B] (a gap
    between A's last metadata and B's first tail) or [B, A] (tails out of
    order).  Each entry writes exactly its own bytes -- the prepad of an entry
    whose table predecessor does not end at its tail is written by its own
    wave -- so the bytes between the batches keep the buffer's fill and the
    bytes of each batch equal the oracle writer's (data_store.rs:847-939)."""
    import ctypes as C
    import torch
    rng = random.Random(11 if order == "gap" else 12)
    keys_a, pays_a = rand_batch(rng, 40)
    keys_b, pays_b = rand_batch(rng, 40)
    ents_a, nt_a = S.batch_layout(0, keys_a, pays_a)
    t_b = nt_a + 1013
    ents_b, nt_b = S.batch_layout(t_b, keys_b, pays_b)
    pay_a, key_a = b"".join(pays_a), b"".join(keys_a)
    for e in ents_b:  # B's sources follow A's in the shared blobs
        e.src += len(pay_a)
        e.key_src += len(key_a)
    table = list(ents_a) + list(ents_b) if order == "gap" else list(ents_b) + list(ents_a)
    n = len(table)
    arr = (S.WriteEntry * n)(*table)
    d_ent = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).cuda()
    d_pay = torch.frombuffer(bytearray(pay_a + b"".join(pays_b)), dtype=torch.uint8).cuda()
    d_key = torch.frombuffer(bytearray(key_a + b"".join(keys_b)), dtype=torch.uint8).cuda()
    fill = 0xAB
    d_out = torch.full((nt_b + 128,), fill, dtype=torch.uint8, device="cuda")
    d_kh = torch.zeros(n, dtype=torch.int64, device="cuda")
    d_mo = torch.zeros(n, dtype=torch.int64, device="cuda")
    S._check(S.lib().srd_batch_write_device(ctx.h, C.c_void_p(d_key.data_ptr()), C.c_void_p(d_pay.data_ptr()),
                                            C.c_void_p(d_ent.data_ptr()), n, C.c_void_p(d_out.data_ptr()), 0,
                                            C.c_void_p(d_kh.data_ptr()), C.c_void_p(d_mo.data_ptr()), None))
    torch.cuda.synchronize()
    want_a_nt, want_a, kh_a = oracle_write(0, keys_a, pays_a, False)
    want_b_nt, want_b, kh_b = oracle_write(t_b, keys_b, pays_b, False, bytes(t_b))
    assert (want_a_nt, want_b_nt) == (nt_a, nt_b)
    want = want_a + bytes([fill]) * (t_b - nt_a) + want_b + bytes([fill]) * 128
    got = d_out.cpu().numpy().tobytes()
    assert got == want
    mos_a = ref_layout(0, pays_a, False)[1]
    mos_b = ref_layout(t_b, pays_b, False)[1]
    kh = [int(x) & (2**64 - 1) for x in d_kh.cpu().tolist()]
    mo = [int(x) for x in d_mo.cpu().tolist()]
    if order == "gap":
        assert kh == kh_a + kh_b and mo == mos_a + mos_b
    else:
        assert kh == kh_b + kh_a and mo == mos_b + mos_a
