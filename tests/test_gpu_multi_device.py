"""srd_validate_index_multi_device: DataStore::open (data_store.rs:84-117) of a
store already resident in the HBM of several GPUs, one entry-range shard per
context, no RCCL.  On this 1-GPU box the "GPUs" are several
contexts on cuda:0 (each its own stream, workspace and host thread; the
copies between them are the same hipMemcpyPeerAsync calls, device-local).

Small stores: every output against the whole-file oracle -- the chain
segments concatenated in shard order, every CRC, and the index both by owner
(the union of the owners' parts, each key at its owner) and merged on
ctxs[0] (identical to the single-GPU order) -- also when a forged cut sends a
run of shards to its lower neighbour and when a torn tail / corruption sends
the store to the whole-file path; `summary.path` says which decided.

Full C4 (BASELINE configs[3]: 16M x 4 KiB = 69,793,218,516 B, 8 shards of 2^21
entries): by size-independent properties -- final_len, counts, the chain's
offsets, every CRC against the oracle's host CRC (plus sampled zlib), one
flipped byte = one bad CRC, the
index's key set = the chain's key set = the bench-key-{i} hashes sampled, every
key at its owner, merged == union of the owners' parts.
"""
import random
import zlib

import numpy as np
import pytest
import xxhash

import oracle as O
import srd_amd as S

pytestmark = pytest.mark.gpu
M48 = (1 << 48) - 1


def _owner(k: int, world: int) -> int:
    return ((k >> 32) * world) >> 32


def _place(ctxs, store: np.ndarray, cuts):
    """Each context's span [floor16K(lo), hi) of the host store in its HBM."""
    import torch
    spans, soffs, keep = [], [], []
    for i in range(len(ctxs)):
        lo, hi = cuts[i], cuts[i + 1]
        if lo == hi:
            spans.append(0)
            soffs.append(0)
            continue
        so = lo - lo % S.SPAN_ALIGN
        t = torch.zeros(S.padded_size(hi - so), dtype=torch.uint8, device="cuda")
        t[: hi - so].copy_(torch.from_numpy(np.ascontiguousarray(store[so:hi])))
        keep.append(t)
        spans.append(t.data_ptr())
        soffs.append(so)
    torch.cuda.synchronize()
    return spans, soffs, keep


_CHAIN = (("meta_off", np.uint64), ("key_hash", np.uint64), ("prev_offset", np.uint64),
          ("payload_start", np.uint64), ("payload_len", np.uint64), ("crc_stored", np.uint32),
          ("crc_computed", np.uint32), ("crc_ok", np.uint8))


def _chain(shards):
    out = {}
    for k, dt in _CHAIN:
        parts = [S.device_to_numpy(getattr(r, k), r.n_chain, dt) for r in shards if r.n_chain]
        out[k] = np.concatenate(parts) if parts else np.zeros(0, dt)
    return out


def _check(ctxs, store, cuts, name, want_path=None):
    a = O.as_u8(store)
    want_len = O.recover_valid_chain(a)
    ch = O.chain_arrays(a, want_len)
    want_idx = O.key_indexer_build(a, want_len)
    spans, soffs, keep = _place(ctxs, a, cuts)
    n = len(ctxs)
    for flags in (0, S.SRD_FLAG_MERGE_INDEX):
        shards, sm = S.validate_index_multi_device(ctxs, spans, soffs, cuts, flags)
        assert sm.final_len == want_len, (name, flags, sm.final_len, want_len)
        assert sm.n_chain == len(ch["meta_off"]) == sum(r.n_chain for r in shards), name
        got = _chain(shards)
        for k, _ in _CHAIN:
            assert np.array_equal(got[k].astype(np.uint64), ch[k].astype(np.uint64)), (name, flags, k)
        assert sm.n_crc_bad == int((ch["crc_ok"] == 0).sum()), name
        if want_path is not None:
            assert sm.path == want_path, (name, flags, sm.path)
        if flags:
            assert sm.merged == 1
            keys = S.device_to_numpy(sm.index_key_hash, sm.n_index)
            packed = S.device_to_numpy(sm.index_packed, sm.n_index)
            assert dict(zip(keys.tolist(), packed.tolist())) == want_idx, name
            # the single-GPU order: chain order of each key's latest entry
            assert (packed & np.uint64(M48)).tolist() == sorted(v & M48 for v in want_idx.values()), name
        else:
            assert sm.merged == (1 if n == 1 else 0)
            union = {}
            for p, r in enumerate(shards):
                ks = S.device_to_numpy(r.index_key_hash, r.n_index).tolist()
                vs = S.device_to_numpy(r.index_packed, r.n_index).tolist()
                if n > 1:
                    assert all(_owner(k, n) == p for k in ks), (name, p)
                    # each owner's part is in chain order too
                    assert [v & M48 for v in vs] == sorted(v & M48 for v in vs), (name, p)
                for k, v in zip(ks, vs):
                    assert k not in union
                    union[k] = v
            assert sm.n_index == len(union) and union == want_idx, name
    del keep


@pytest.fixture(scope="module")
def ctxs():
    cs = [S.Context(0) for _ in range(6)]
    yield cs
    for c in cs:
        c.close()


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


@pytest.mark.parametrize("nd", [1, 2, 3, 5])
def test_multi_device_matches_oracle(ctxs, nd):
    for name, st in {"c1": O.synth_store(1000), "mixed": _mixed_store(), "overwrites": _overwrite_store()}.items():
        _check(ctxs[:nd], st, S.shard_cuts(st, nd), f"{name}/{nd}", S.SRD_MULTI_COMPOSED)


def test_multi_device_empty_shards(ctxs):
    st = O.synth_store(300)
    cuts = S.shard_cuts(st, 3)
    # the middle shard empty, and a store on one shard out of four
    _check(ctxs[:3], st, [0, cuts[1], cuts[1], st.size], "empty-middle", S.SRD_MULTI_COMPOSED)
    _check(ctxs[:4], st, [0, st.size, st.size, st.size, st.size], "one-shard", S.SRD_MULTI_COMPOSED)
    _check(ctxs[:2], np.zeros(0, np.uint8), [0, 0, 0], "empty-store", S.SRD_MULTI_COMPOSED)


@pytest.mark.parametrize("nd", [3, 4, 6])
def test_multi_device_forged_cut_takes_neighbour(ctxs, nd):
    """A cut on a forged metadata record inside a payload: the shard above it
    is unproven; it is re-validated with its lower neighbour (bytes gathered
    onto the neighbour's GPU), not by the whole-file path."""
    from test_shard_gloo import fake_cut_store
    store, fake = fake_cut_store()
    cuts = S.shard_cuts(store, nd)
    assert fake in cuts[1:-1]
    _check(ctxs[:nd], store, cuts, f"forged-{nd}", S.SRD_MULTI_NEIGHBOUR)


def test_multi_device_torn_and_corrupt_go_whole_file(ctxs):
    base = _mixed_store(800, seed=5)
    rnd = random.Random(2)
    for cut in [base.size - 7, base.size - 100, rnd.randrange(base.size // 2, base.size)]:
        st = base[:cut]
        # cuts of the intact prefix: the top shard ends at the torn file_len
        cuts = S.shard_cuts(st, 3)
        _check(ctxs[:3], st, cuts, f"cut{cut}")
        assert ctxs[0].multi_summary().path == S.SRD_MULTI_WHOLE_FILE or O.recover_valid_chain(st) == st.size
    g = np.concatenate([base, np.frombuffer(b"CORRUPT", np.uint8)])
    _check(ctxs[:2], g, S.shard_cuts(g, 2), "corrupt", S.SRD_MULTI_WHOLE_FILE)
    # a flipped payload byte: the chain composes, exactly one CRC is bad
    b = base.copy()
    ch = O.chain_arrays(base, base.size)
    i = len(ch["meta_off"]) // 2
    b[int(ch["payload_start"][i]) + int(ch["payload_len"][i]) // 2] ^= 0x10
    _check(ctxs[:3], b, S.shard_cuts(b, 3), "flip", S.SRD_MULTI_COMPOSED)


def test_multi_duplicate_context_is_an_error(ctxs):
    st = O.synth_store(100)
    with pytest.raises(S.SrdError, match="distinct"):
        S.validate_index_multi(st, [ctxs[0], ctxs[1], ctxs[0]])
    cuts = S.shard_cuts(st, 2)
    spans, soffs, keep = _place(ctxs[:2], st, cuts)
    with pytest.raises(S.SrdError, match="distinct"):
        S.validate_index_multi_device([ctxs[1], ctxs[1]], spans, soffs, cuts)
    with pytest.raises(S.SrdError):  # a span that does not start at a 16 KiB boundary
        S.validate_index_multi_device(ctxs[:2], spans, [0, soffs[1] + 64], cuts)


def test_host_multi_reports_its_path(ctxs):
    """srd_validate_index_multi (host input) now runs the device
    implementation; srd_ctx_multi_summary names the path that decided."""
    from test_shard_gloo import fake_cut_store
    st = _mixed_store(700, seed=9)
    r = S.validate_index_multi(st, ctxs[:3])
    assert r.final_len == st.size and ctxs[0].multi_summary().path == S.SRD_MULTI_COMPOSED
    store, fake = fake_cut_store()
    cuts = S.shard_cuts(store, 4)
    assert fake in cuts
    r = S.validate_index_multi(store, ctxs[:4])
    assert r.final_len == store.size and ctxs[0].multi_summary().path == S.SRD_MULTI_NEIGHBOUR
    torn = np.concatenate([st, np.frombuffer(b"CORRUPT", np.uint8)])
    r = S.validate_index_multi(torn, ctxs[:2])
    assert r.final_len == st.size and ctxs[0].multi_summary().path == S.SRD_MULTI_WHOLE_FILE


# ---------------------------------------------------------------------------
# Full C4 on one GPU: 8 contexts, 2^21 entries each, 65 GiB resident

C4_N, C4_W, C4_LEN = 1 << 24, 8, 69_793_218_516


def test_full_c4_eight_shards():
    import torch
    import srd_shard as SH
    assert S.synth_store_len(C4_N, 4096) == C4_LEN
    cs = [S.Context(0) for _ in range(C4_W)]
    spans, soffs, cuts, keep = [], [], [0], []
    try:
        for first, cnt in SH.plan_entry_shards(C4_N, C4_W):
            lo, hi = S.synth_span(None, 0, first, cnt, 4096)
            so = lo - lo % S.SPAN_ALIGN
            t = torch.empty(S.padded_size(hi - so), dtype=torch.uint8, device="cuda")
            S.synth_span(t.data_ptr(), so, first, cnt, 4096, ctx=cs[len(keep)])
            keep.append(t)
            spans.append(t.data_ptr())
            soffs.append(so)
            assert lo == cuts[-1]
            cuts.append(hi)
        torch.cuda.synchronize()
        assert cuts[-1] == C4_LEN
        shards, sm = S.validate_index_multi_device(cs, spans, soffs, cuts)
        assert (sm.path, sm.mode, sm.final_len, sm.n_chain, sm.n_index, sm.n_crc_bad) == \
            (S.SRD_MULTI_COMPOSED, 0, C4_LEN, C4_N, C4_N, 0)
        assert [r.n_chain for r in shards] == [C4_N // C4_W] * C4_W
        # chain offsets: entry i's metadata at 4160 i + 4096, strictly in file order
        mo = torch.cat([S.device_view(r.meta_off, r.n_chain) for r in shards])
        assert torch.equal(mo, torch.arange(C4_N, device="cuda", dtype=torch.int64) * 4160 + 4096)
        ln = torch.cat([S.device_view(r.payload_len, r.n_chain) for r in shards])
        assert int(ln.min()) == int(ln.max()) == 4096
        crc = torch.cat([S.device_view(r.crc_computed, r.n_chain, np.uint32) for r in shards])
        st = torch.cat([S.device_view(r.crc_stored, r.n_chain, np.uint32) for r in shards])
        assert torch.equal(crc, st)
        kh = torch.cat([S.device_view(r.key_hash, r.n_chain) for r in shards])
        per = C4_N // C4_W
        # every one of the 2^24 computed CRCs against the oracle's independent
        # PCLMUL CRC (entry_handle.rs:260-275 / compute_checksum.rs:15-20) over
        # each shard's bytes streamed D2H in ~2 GiB groups of whole entries:
        # crc_stored was written by the device's synth kernel, which shares the
        # scan's CRC machinery, so crc == st alone could hide a common bug
        grp = 1 << 19
        host = torch.empty(4160 * grp, dtype=torch.uint8, pin_memory=True)
        hn = host.numpy()
        crc_h = crc.cpu().numpy().view(np.uint32)
        checked = 0
        for s_i in range(C4_W):
            for i0 in range(s_i * per, (s_i + 1) * per, grp):
                i1 = min(i0 + grp, (s_i + 1) * per)
                b0 = 4160 * i0 - soffs[s_i]
                nb = 4160 * (i1 - i0) - 64  # through the last entry's payload
                host[:nb].copy_(keep[s_i][b0:b0 + nb])
                starts = np.arange(i1 - i0, dtype=np.uint64) * np.uint64(4160)
                got = O.crc32_ranges(hn[:nb], starts, np.full(i1 - i0, 4096, np.uint64), threads=16)
                bad = np.nonzero(got != crc_h[i0:i1])[0]
                assert bad.size == 0, ("crc_computed differs from the host CRC", s_i, int(i0 + bad[0]), bad.size)
                checked += i1 - i0
        assert checked == C4_N
        del host, hn, crc_h
        # sampled CRCs against zlib, straight from the shards' HBM
        for i in np.random.default_rng(4).integers(0, C4_N, 200).tolist():
            s = i // per
            off = 4160 * i - soffs[s]
            assert int(crc[i]) & 0xFFFFFFFF == zlib.crc32(keep[s][off:off + 4096].cpu().numpy().tobytes()), i
        for i in np.random.default_rng(6).integers(0, C4_N, 2000).tolist() + [0, C4_N - 1]:
            assert int(kh[i]) & (2**64 - 1) == xxhash.xxh3_64_intdigest(b"bench-key-%d" % i), i
        # the index: every key at its owner, the key set = the chain's key set
        ik = []
        for p, r in enumerate(shards):
            k = S.device_view(r.index_key_hash, r.n_index)
            hi32 = (k >> 32) & 0xFFFFFFFF
            assert bool(((hi32 * C4_W) >> 32 == p).all()), p
            v = S.device_view(r.index_packed, r.n_index)
            assert bool(((v & M48) - 4096).remainder(4160).eq(0).all())
            ik.append(k)
        ik = torch.cat(ik)
        assert torch.equal(torch.sort(ik).values, torch.sort(kh).values)
        owner_sorted = torch.sort(ik).values
        del ik
        # the merged index on ctxs[0] equals the union of the owners' parts
        shards2, sm2 = S.validate_index_multi_device(cs, spans, soffs, cuts, S.SRD_FLAG_MERGE_INDEX)
        assert (sm2.path, sm2.final_len, sm2.n_index, sm2.merged) == (S.SRD_MULTI_COMPOSED, C4_LEN, C4_N, 1)
        mk = S.device_view(sm2.index_key_hash, sm2.n_index)
        mv = S.device_view(sm2.index_packed, sm2.n_index)
        assert torch.equal(torch.sort(mk).values, owner_sorted)
        assert torch.equal(mv & M48, torch.arange(C4_N, device="cuda", dtype=torch.int64) * 4160 + 4096)
        del mk, mv, owner_sorted, mo, ln, crc, st, kh
        # one flipped payload byte in shard 5 -> exactly one bad CRC, still composed
        i = 5 * per + 12345
        pos = 4160 * i + 777 - soffs[5]
        keep[5][pos] ^= 0x40
        shards, sm = S.validate_index_multi_device(cs, spans, soffs, cuts)
        assert (sm.path, sm.final_len, sm.n_chain, sm.n_crc_bad) == (S.SRD_MULTI_COMPOSED, C4_LEN, C4_N, 1)
        ok = S.device_view(shards[5].crc_ok, shards[5].n_chain, np.uint8)
        assert torch.nonzero(ok == 0).flatten().tolist() == [12345]
        keep[5][pos] ^= 0x40
    finally:
        del keep
        for c in cs:
            c.close()
        torch.cuda.empty_cache()
