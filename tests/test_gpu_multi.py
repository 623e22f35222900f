"""srd_validate_index_multi: DataStore::open of one host store on several
GPUs in ONE process, no RCCL (data_store.rs:84-117).  On this
1-GPU box the "devices" are 2 / 3 contexts on the same GPU (each its own
stream and workspace, driven by its own host thread).  Every result must be
identical to the whole-file oracle's: final_len, the chain, every CRC, the
latest-wins index -- also when the store does not compose (torn tail, forged
cut) and the whole-file path decides.  Plus the host-input staging modes and
DataStore.open on an mmap'd file."""
import random

import numpy as np
import pytest
import xxhash

import oracle as O
import srd_amd as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs():
    cs = [S.Context(0) for _ in range(3)]
    yield cs
    for c in cs:
        c.close()


def same_as_oracle(r, data, name):
    a = O.as_u8(data)
    want_len = O.recover_valid_chain(a)
    assert r.final_len == want_len, (name, r.final_len, want_len)
    ch = O.chain(a, want_len)
    assert r.n_chain == len(ch), (name, r.n_chain, len(ch))
    for k in ("meta_off", "key_hash", "prev_offset", "payload_start", "payload_len", "crc_stored", "crc_computed",
              "crc_ok"):
        got = getattr(r, k).astype(np.uint64)
        exp = np.array([e[k] for e in ch], np.uint64)
        assert np.array_equal(got, exp), (name, k)
    idx = O.key_indexer_build(a, want_len)
    assert r.index() == idx, name
    # the index order is the chain order of each key's latest entry
    assert list(r.index_packed & np.uint64((1 << 48) - 1)) == sorted(v & ((1 << 48) - 1) for v in idx.values())
    assert r.n_crc_bad == sum(1 - e["crc_ok"] for e in ch)


def _mixed_store(n=1500, seed=3):
    lens = np.minimum(S.zipf_lens(n, seed=seed), 1 << 18)
    return O.synth_store(n, lens=lens)


def _overwrite_store(seed=11, n=600):
    rnd = random.Random(seed)
    buf, t = bytearray(), 0
    for _ in range(n):
        kh = xxhash.xxh3_64_intdigest(b"key%d" % rnd.randrange(90))
        if rnd.random() < 0.15:
            t = O.write_entries(buf, t, [(kh, b"\x00")], allow_null=True)
        else:
            pl = rnd.randbytes(rnd.choice([1, 8, 20, 64, 100, 700, 4096, 5000]))
            t = O.write_entries(buf, t, [(kh, b"\x01" if pl == b"\x00" else pl)])
    return np.frombuffer(bytes(buf), np.uint8)


@pytest.mark.parametrize("nd", [2, 3])
def test_multi_matches_oracle(ctxs, nd):
    stores = {"c1": O.synth_store(1000), "mixed": _mixed_store(), "overwrites": _overwrite_store()}
    for name, st in stores.items():
        r = S.validate_index_multi(st, ctxs[:nd])
        same_as_oracle(r, st, f"{name}/{nd}")
        assert r.mode == S.SRD_MODE_OPTIMISTIC, name


@pytest.mark.parametrize("nd", [2, 3])
def test_multi_golden_fixtures(golden_cases, ctxs, nd):
    for name, (data, m) in golden_cases.items():
        r = S.validate_index_multi(np.frombuffer(data, np.uint8) if data else np.zeros(0, np.uint8), ctxs[:nd])
        assert r.final_len == m["final_len"], name
        assert r.n_chain == len(m["chain"]), name
        assert r.index() == {int(k, 16): int(v, 16) for k, v in m["index"].items()}, name
        assert [int(x) for x in r.crc_computed] == [e["crc_computed"] for e in m["chain"]], name


def test_multi_not_composed_goes_whole_file(ctxs):
    base = _mixed_store(800, seed=5)
    rnd = random.Random(2)
    # torn tails, flipped bytes, trailing garbage: the whole-file path decides
    for cut in [base.size - 7, base.size - 100, rnd.randrange(base.size // 2, base.size)]:
        same_as_oracle(S.validate_index_multi(base[:cut], ctxs[:3]), base[:cut], f"cut{cut}")
    b = base.copy()
    b[rnd.randrange(b.size)] ^= 0x10
    same_as_oracle(S.validate_index_multi(b, ctxs[:2]), b, "flip")
    g = np.concatenate([base, np.frombuffer(b"CORRUPT", np.uint8)])
    same_as_oracle(S.validate_index_multi(g, ctxs[:2]), g, "corrupt")


def test_multi_forged_cut_is_refuted(ctxs):
    from test_shard_gloo import fake_cut_store
    store, fake = fake_cut_store()
    assert S.shard_cuts(store, 2)[1] == fake
    r = S.validate_index_multi(store, ctxs[:2])
    same_as_oracle(r, store, "forged")


def test_staging_modes_agree(ctxs):
    st = _mixed_store(600, seed=8)
    want = S.validate_index(st, 0, ctxs[0])
    assert ctxs[0].stage_mode() == "bounce buffers"  # the default for unpinned host memory
    for flags, mode in ((S.SRD_FLAG_STAGE_PAGEABLE, "pageable copy"), (S.SRD_FLAG_STAGE_REGISTER, "registered mapping")):
        r = S.validate_index(st, flags, ctxs[0])
        assert ctxs[0].stage_mode() == mode
        assert (r.final_len, r.n_chain, r.n_index) == (want.final_len, want.n_chain, want.n_index)
        assert np.array_equal(r.crc_computed, want.crc_computed) and r.index() == want.index()
    r = S.validate_index_multi(st, ctxs[:3], S.SRD_FLAG_STAGE_REGISTER)
    same_as_oracle(r, st, "register-multi")


@pytest.mark.parametrize("nd", [1, 2, 3])
def test_datastore_open_mmap(tmp_path, ctxs, nd):
    """DataStore::open of a file: the mapping goes to the library as is
    (registered or bounce-staged), on 1-3 contexts."""
    p = tmp_path / "store.bin"
    st = _mixed_store(700, seed=13)
    p.write_bytes(st.tobytes())
    ds = S.DataStore.open(str(p), ctxs=ctxs[:nd])
    assert ds.tail_offset == st.size and ds.len() == len(O.key_indexer_build(st, st.size))
    e = ds.read(b"bench-key-42")
    assert e is not None and e.is_valid_checksum()
    assert ctxs[0].stage_mode() in ("registered mapping", "bounce buffers")
    # torn tail on several contexts: truncated exactly like data_store.rs:91-104
    p.write_bytes(st.tobytes() + b"CORRUPT")
    with pytest.warns(UserWarning):
        ds = S.DataStore.open(str(p), ctxs=ctxs[:nd])
    assert ds.tail_offset == st.size and p.stat().st_size == st.size


@pytest.mark.parametrize("nd", [3, 4, 6])
def test_multi_forged_cut_merges_with_lower_neighbour(nd):
    """A forged cut inside the store (not the top shard's): the shard above it
    is unproven and is re-validated together with its lower neighbour (the
    first non-empty one below); the result is still the oracle's."""
    from test_shard_gloo import fake_cut_store
    store, fake = fake_cut_store()
    cuts = list(S.shard_cuts(store, nd))
    assert fake in cuts and cuts.index(fake) >= 1
    cs = [S.Context(0) for _ in range(nd)]
    try:
        r = S.validate_index_multi(store, cs)
        same_as_oracle(r, store, f"forged-{nd}")
    finally:
        for c in cs:
            c.close()
