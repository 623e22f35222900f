"""Iteration and compaction over the device index:
EntryIterator / par_iter_entries (entry_iterator.rs:69-126,
data_store.rs:297-361), estimate_compaction_savings (data_store.rs:605-616)
and compact (data_store.rs:706-749), through the C ABI on the index a GPU
validate pass built.  Checked against Python restatements of the reference
loops on stores written by the oracle writer (overwrites, deletes), the
scenarios of parallel_iterator_tests.rs and compaction_tests.rs, and the
write_stream NULL-only rejection compact() inherits."""
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


def entry_iterator(f: bytes, tail: int):
    """EntryIterator::next (entry_iterator.rs:69-126): (start, end, meta_off, key_hash), newest first."""
    out, seen, cursor = [], set(), tail
    while cursor >= 20:
        mo = cursor - 20
        kh = int.from_bytes(f[mo:mo + 8], "little")
        prev = int.from_bytes(f[mo + 8:mo + 16], "little")
        start = prev + ((64 - prev % 64) & 63)
        if mo > prev and mo - prev == 1 and f[prev:mo] == b"\x00":
            start = prev
        if start >= mo or mo > len(f):
            break
        cursor = prev
        if kh in seen:
            continue
        seen.add(kh)
        if mo - start == 1 and f[start:mo] == b"\x00":
            continue
        out.append((start, mo, mo, kh))
    return out


def build_store(seed, n_keys=200, rounds=4):
    rng = random.Random(seed)
    buf, tail = bytearray(), 0
    keys = [b"k%d" % i for i in range(n_keys)]
    for rnd in range(rounds):
        batch = []
        for k in rng.sample(keys, n_keys // 2):
            if rnd and rng.random() < 0.2:
                batch.append((O.xxh3_64(k), b"\x00"))
            else:
                p = bytes(rng.getrandbits(8) | 1 for _ in range(rng.choice([1, 5, 64, 100, 4096, 6000])))
                batch.append((O.xxh3_64(k), p))
        tail = O.write_entries(buf, tail, batch, allow_null=True)
    return bytes(buf)


def validated(ctx, f):
    import torch
    dev = torch.zeros(S.padded_size(len(f)), dtype=torch.uint8, device="cuda")
    dev[: len(f)] = torch.frombuffer(bytearray(f), dtype=torch.uint8).cuda()
    r = S.validate_index_device(dev.data_ptr(), len(f), 0, ctx)
    assert r.final_len == len(f)
    return dev, r


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_iter_entries_matches_entry_iterator(ctx, seed):
    f = build_store(seed)
    dev, r = validated(ctx, f)
    st, en, mo, kh = S.iter_entries_device(dev.data_ptr(), len(f), r.index_packed, r.n_index, ctx)
    want = entry_iterator(f, len(f))
    assert len(st) == len(want)
    assert [(int(a), int(b), int(c), int(d)) for a, b, c, d in zip(st, en, mo, kh)] == want
    savings = S.estimate_compaction_savings_device(dev.data_ptr(), len(f), r.index_packed, r.n_index, ctx)
    assert savings == max(len(f) - sum(e - s + 20 for s, e, _, _ in want), 0)


def test_compact_matches_reference(ctx):
    f = build_store(4)
    dev, r = validated(ctx, f)
    out = S.compact_device(dev.data_ptr(), len(f), r.index_packed, r.n_index, ctx).cpu().numpy().tobytes()
    # compact(): write_stream_with_key_hash of each iter_entries entry, in order, into an empty store
    want_buf = bytearray()
    O.write_entries(want_buf, 0, [(kh, f[s:e]) for s, e, _, kh in entry_iterator(f, len(f))])
    assert out == bytes(want_buf)
    assert len(out) < len(f)
    # the compacted store opens to the same live key set with the same payloads
    a = np.frombuffer(out, np.uint8)
    assert O.recover_valid_chain(a) == len(out)
    live = {kh: f[s:e] for s, e, _, kh in entry_iterator(f, len(f))}
    assert {kh: out[s:e] for s, e, _, kh in entry_iterator(out, len(out))} == live


def test_reference_iterator_and_compaction_scenarios(ctx):
    # parallel_iterator_tests.rs: deleted / updated-then-deleted / latest version only;
    # compaction_tests.rs: 7 keys written, overwritten, one deleted -> smaller file
    buf, tail = bytearray(), 0
    h = O.xxh3_64
    ks = [b"text_key", b"binary_key", b"struct_key", b"integer_key", b"float_key", b"mixed_key", b"temp_key"]
    tail = O.write_entries(buf, tail, [(h(k), b"v1-" + k) for k in ks])
    tail = O.write_entries(buf, tail, [(h(k), b"v2-" + k) for k in ks])
    tail = O.write_entries(buf, tail, [(h(b"temp_key"), b"\x00")], allow_null=True)
    f = bytes(buf)
    dev, r = validated(ctx, f)
    st, en, _, kh = S.iter_entries_device(dev.data_ptr(), len(f), r.index_packed, r.n_index, ctx)
    got = {int(k): f[int(s):int(e)] for s, e, k in zip(st, en, kh)}
    assert got == {h(k): b"v2-" + k for k in ks[:-1]}
    out = S.compact_device(dev.data_ptr(), len(f), r.index_packed, r.n_index, ctx).cpu().numpy().tobytes()
    assert len(out) < len(f)
    assert S.estimate_compaction_savings_device(dev.data_ptr(), len(f), r.index_packed, r.n_index, ctx) > 0


def test_compact_rejects_null_only_payload(ctx):
    # write_stream (which compact() uses) rejects all-NULL payloads of any length
    buf = bytearray()
    O.write_entries(buf, 0, [(O.xxh3_64(b"a"), b"abc"), (O.xxh3_64(b"z"), b"\x00\x00\x00")])
    f = bytes(buf)
    dev, r = validated(ctx, f)
    with pytest.raises(S.SrdError, match="NULL-byte-only streams"):
        S.compact_device(dev.data_ptr(), len(f), r.index_packed, r.n_index, ctx)
