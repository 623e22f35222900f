"""Device KeyIndexer + batched keyed reads:
KeyIndexer::get_packed (key_indexer.rs:164-167), batch_read /
batch_read_hashed_keys (data_store.rs:1111-1158) over read_entry_with_context
(:502-565), through the C ABI, on the index a GPU validate pass built.

Checked against the oracle's KeyIndexer::build map and a Python restatement of
read_entry_with_context, on a store written by the oracle writer with
overwrites and deletes (tombstones), and the reference's own batch_ops_tests.rs
cases (missing keys, hashed reads with and without verification, the
collision check)."""
import random

import numpy as np
import pytest

import oracle as O
import srd_amd as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = S.Context(0)
    yield c
    c.close()


def read_entry_with_context(f: bytes, index: dict, key_hash: int, verify_hash=None):
    """data_store.rs:502-565 on the oracle index."""
    packed = index.get(key_hash)
    if packed is None:
        return None
    tag, off = packed >> 48, packed & ((1 << 48) - 1)
    if verify_hash is not None and tag != verify_hash >> 48:
        return None
    if off + 20 > len(f):
        return None
    prev = int.from_bytes(f[off + 8:off + 16], "little")
    start = prev + ((64 - prev % 64) & 63)
    if off > prev and off - prev == 1 and f[prev:off] == b"\x00":
        start = prev
    if start >= off:
        return None
    if off - start == 1 and f[start:off] == b"\x00":
        return None
    return (start, off)


def build_store(seed):
    rng = random.Random(seed)
    buf = bytearray()
    tail = 0
    latest = {}
    keys = [b"key-%d" % i for i in range(300)] + [b"a", b"b", b"c", b"d"]
    for rnd in range(4):
        batch = []
        for k in rng.sample(keys, 120):
            if rnd and rng.random() < 0.25:
                batch.append((k, b"\x00"))  # delete -> tombstone (batch_delete writes NULL payloads)
            else:
                p = bytes(rng.getrandbits(8) for _ in range(rng.choice([1, 3, 7, 64, 100, 4096, 5000])))
                if p == b"\x00":
                    p = b"\x01"
                batch.append((k, p))
        for k, p in batch:
            latest[k] = p
        tail = O.write_entries(buf, tail, [(O.xxh3_64(k), p) for k, p in batch], allow_null=True)
    return bytes(buf), keys, latest


def device_index(ctx, f):
    import torch
    dev = torch.zeros(S.padded_size(len(f)), dtype=torch.uint8, device="cuda")
    dev[: len(f)] = torch.frombuffer(bytearray(f), dtype=torch.uint8).cuda()
    r = S.validate_index_device(dev.data_ptr(), len(f), 0, ctx)
    assert r.final_len == len(f)
    idx = S.DeviceIndex(r.index_key_hash, r.index_packed, r.n_index, ctx)
    return dev, idx


def test_get_packed_matches_key_indexer(ctx):
    f, keys, _ = build_store(1)
    want = O.key_indexer_build(np.frombuffer(f, np.uint8), len(f))
    dev, idx = device_index(ctx, f)
    hashes = list(want.keys()) + [12345, 0, (1 << 64) - 1, O.xxh3_64(b"never written")]
    got = idx.get_packed(np.array(hashes, np.uint64))
    for h, g in zip(hashes, got):
        assert int(g) == want.get(h, S.INDEX_NONE), hex(h)


@pytest.mark.parametrize("seed", [2, 3])
def test_batch_read_matches_read_entry_with_context(ctx, seed):
    f, keys, latest = build_store(seed)
    index = O.key_indexer_build(np.frombuffer(f, np.uint8), len(f))
    dev, idx = device_index(ctx, f)
    query = keys + [b"missing_key", b"fake_key"]
    rng = random.Random(seed)
    rng.shuffle(query)
    got = idx.batch_read(dev.data_ptr(), len(f), query)
    for k, g in zip(query, got):
        h = O.xxh3_64(k)
        assert g == read_entry_with_context(f, index, h, h), k
        if g is not None:
            assert f[g[0]:g[1]] == latest[k], k  # the latest non-deleted payload
        else:
            assert latest.get(k) in (None, b"\x00"), k
    # hashed reads without verification: same answers
    hashes = [O.xxh3_64(k) for k in query]
    assert idx.batch_read_hashed_keys(dev.data_ptr(), len(f), hashes) == got


def test_reference_batch_ops_cases(ctx):
    # batch_ops_tests.rs:46-72, :132-167, :197-281 on one store
    buf = bytearray()
    entries = [(b"a", b"AAA"), (b"b", b"BBB"), (b"c", b"CCC"), (b"d", b"DDD"), (b"exists_1", b"payload one"),
               (b"exists_2", b"payload two"), (b"key1", b"val1"), (b"key2", b"val2"), (b"real_key", b"some data")]
    tail = O.write_entries(buf, 0, [(O.xxh3_64(k), p) for k, p in entries])
    f = bytes(buf)
    dev, idx = device_index(ctx, f)
    res = idx.batch_read(dev.data_ptr(), len(f), [b"a", b"b", b"c", b"d"])
    assert [f[s:e] for s, e in res] == [b"AAA", b"BBB", b"CCC", b"DDD"]
    res = idx.batch_read(dev.data_ptr(), len(f), [b"exists_1", b"missing_key", b"exists_2"])
    assert f[res[0][0]:res[0][1]] == b"payload one" and res[1] is None and f[res[2][0]:res[2][1]] == b"payload two"
    hashes = S.compute_hash_batch([b"key1", b"key2"], ctx)
    res = idx.batch_read_hashed_keys(dev.data_ptr(), len(f), hashes, [b"key1", b"key2"])
    assert [f[s:e] for s, e in res] == [b"val1", b"val2"]
    res = idx.batch_read_hashed_keys(dev.data_ptr(), len(f), [S.compute_hash(b"exists"), 12345])
    assert res == [None, None]  # "exists" was never written here; 12345 never is
    real = S.compute_hash(b"real_key")
    assert idx.batch_read_hashed_keys(dev.data_ptr(), len(f), [real], [b"fake_key"]) == [None]  # tag mismatch
    assert f[slice(*idx.batch_read_hashed_keys(dev.data_ptr(), len(f), [real])[0])] == b"some data"
    with pytest.raises(ValueError, match="Mismatched lengths"):
        idx.batch_read_hashed_keys(dev.data_ptr(), len(f), [real], [b"a", b"b"])
