"""GPU parity of the entry-range shard path (srd_validate_span_device) and the
index exchange (srd_index_partition_device + srd_index_build_device) against
the CPU oracle: every shard's chain segment, CRCs and local index, and the
merged global index, bit-exact with the whole-file result
(data_store.rs:383-482, key_indexer.rs:98-124)."""
import random

import numpy as np
import pytest
import xxhash

import oracle as O
import srd_amd as S

pytestmark = pytest.mark.gpu

FIELDS = ("meta_off", "key_hash", "prev_offset", "payload_start", "payload_len", "crc_stored",
          "crc_computed", "crc_ok")


@pytest.fixture(scope="module")
def ctx():
    c = S.Context(0)
    yield c
    c.close()


def _dev(host: np.ndarray, span_off: int, hi: int):
    import torch
    n = hi - span_off
    t = torch.zeros(S.padded_size(n), dtype=torch.uint8, device="cuda")
    t[:n] = torch.from_numpy(np.ascontiguousarray(host[span_off:hi]))
    torch.cuda.synchronize()
    return t


def _arr(ptr, n, dt):
    return S.device_to_numpy(ptr, n, dt)


def shard_chain(r):
    return {k: _arr(getattr(r, k), r.n_chain, np.uint32 if k.startswith("crc_") and k != "crc_ok" else
                    (np.uint8 if k == "crc_ok" else np.uint64)) for k in FIELDS}


def check_shards(store: np.ndarray, cuts, ctx, name):
    """cuts: chain entry indices where shards start (first must be 0)."""
    flen = O.recover_valid_chain(store)
    assert flen == store.size, name
    ch = O.chain(store, flen)
    tails = [0] + [e["meta_off"] + 20 for e in ch]
    bounds = list(zip(cuts, cuts[1:] + [len(ch)]))
    all_pairs = []
    import torch
    for (a, b) in bounds:
        lo, hi = tails[a], tails[b]
        span_off = lo - lo % S.SPAN_ALIGN
        t = _dev(store, span_off, hi)
        r = S.validate_span_device(t.data_ptr(), span_off, lo, hi, 0, ctx)
        assert r.mode == 0 and r.final_len == hi and r.n_chain == b - a, (name, a, b, r.mode, r.final_len, r.n_chain)
        got = shard_chain(r)
        for k in FIELDS:
            exp = np.array([e[k] for e in ch[a:b]], np.uint64)
            assert np.array_equal(got[k].astype(np.uint64), exp), (name, a, b, k)
        # shard-local KeyIndexer: latest entry per key inside the shard
        want = {}
        for e in ch[a:b]:
            want[e["key_hash"]] = ((e["key_hash"] >> 48) << 48) | e["meta_off"]
        keys = _arr(r.index_key_hash, r.n_index, np.uint64)
        packed = _arr(r.index_packed, r.n_index, np.uint64)
        assert dict(zip(map(int, keys), map(int, packed))) == want, (name, a, b)
        assert r.n_crc_bad == sum(1 - e["crc_ok"] for e in ch[a:b])
        all_pairs.append((torch.from_numpy(keys.view(np.int64)).cuda(), torch.from_numpy(packed.view(np.int64)).cuda()))
    # index exchange over W owners (all shards on this one GPU): partition,
    # concatenate each owner's runs in shard order, build, union == full index
    W = 4
    runs = [[] for _ in range(W)]
    for k, v in all_pairs:
        n = k.numel()
        out = torch.empty(2 * max(n, 1), dtype=torch.int64, device="cuda")
        counts = S.index_partition_device(k.data_ptr(), v.data_ptr(), n, W, out.data_ptr(), ctx)
        assert sum(counts) == n
        o = 0
        for w, c in enumerate(counts):
            runs[w].append(out[2 * o: 2 * (o + c)])
            for kk in out[2 * o: 2 * (o + c): 2].cpu().numpy().view(np.uint64):
                assert ((int(kk) >> 32) * W) >> 32 == w
            o += c
    merged = {}
    for w in range(W):
        pairs = torch.cat(runs[w]) if runs[w] else torch.empty(0, dtype=torch.int64, device="cuda")
        n = pairs.numel() // 2
        ok = torch.empty(max(n, 1), dtype=torch.int64, device="cuda")
        op = torch.empty(max(n, 1), dtype=torch.int64, device="cuda")
        ni = S.index_build_device(pairs.data_ptr(), n, ok.data_ptr(), op.data_ptr(), ctx)
        kk = ok[:ni].cpu().numpy().view(np.uint64)
        pp = op[:ni].cpu().numpy().view(np.uint64)
        for a_, b_ in zip(kk, pp):
            assert int(a_) not in merged
            merged[int(a_)] = int(b_)
    assert merged == O.key_indexer_build(store, flen), name


def test_shards_c1(ctx):
    check_shards(O.synth_store(1000), [0, 1, 333, 700, 999], ctx, "c1")


def test_shards_mixed(ctx):
    rng = np.random.default_rng(0x5EED0003)
    r = np.arange(1, 16)
    p = 1.0 / r ** 2.0
    k = rng.choice(np.arange(6, 21), size=400, p=p / p.sum())
    lens = ((1 << k) - np.where(k >= 7, rng.integers(0, 64, size=400), 0)).astype(np.uint64)
    check_shards(O.synth_store(len(lens), lens=lens), [0, 50, 51, 200, 390], ctx, "zipf")


def test_shards_overwrites_tombstones(ctx):
    rnd = random.Random(23)
    buf = bytearray()
    t = 0
    for step in range(600):
        kh = xxhash.xxh3_64_intdigest(b"key%d" % rnd.randrange(80))
        if rnd.random() < 0.15:
            t = O.write_entries(buf, t, [(kh, b"\x00")], allow_null=True)
        else:
            n = rnd.choice([1, 5, 20, 64, 100, 3000, 4096, 9000])
            t = O.write_entries(buf, t, [(kh, rnd.randbytes(n))])
    store = np.frombuffer(bytes(buf), np.uint8)
    check_shards(store, [0, 100, 101, 102, 350, 599], ctx, "tomb")


def test_unproven_span_reports_mode(ctx):
    store = O.synth_store(300)
    ch = O.chain(store, store.size)
    lo = ch[99]["meta_off"] + 20
    cut = store.size - 7  # torn tail inside the last shard
    span_off = lo - lo % S.SPAN_ALIGN
    t = _dev(store, span_off, cut)
    r = S.validate_span_device(t.data_ptr(), span_off, lo, cut, 0, ctx)
    assert r.mode == S.SRD_MODE_SPAN_UNPROVEN and r.final_len == 0
    # a wrong lower tail is not proven either
    t = _dev(store, span_off, store.size)
    r = S.validate_span_device(t.data_ptr(), span_off, lo + 64, store.size, 0, ctx)
    assert r.mode == S.SRD_MODE_SPAN_UNPROVEN


def test_synth_span_matches_whole_store(ctx):
    import torch
    n = 2000
    size = S.synth_store_len(n)
    whole = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
    S.synth_store_device(whole.data_ptr(), n, 4096, ctx=ctx)
    for first, cnt in ((0, 700), (700, 600), (1300, 700), (1999, 1)):
        lo, hi = S.synth_span(None, 0, first, cnt)
        span_off = lo - lo % S.SPAN_ALIGN
        t = torch.zeros(S.padded_size(hi - span_off), dtype=torch.uint8, device="cuda")
        assert S.synth_span(t.data_ptr(), span_off, first, cnt, ctx=ctx) == (lo, hi)
        assert torch.equal(t[: hi - span_off], whole[span_off:hi]), (first, cnt)
        r = S.validate_span_device(t.data_ptr(), span_off, lo, hi, 0, ctx)
        assert (r.mode, r.final_len, r.n_chain, r.n_crc_bad, r.n_index) == (0, hi, cnt, 0, cnt), (first, r.mode)


def test_backend_build_waits_for_torch_stream(ctx):
    """The index exchange hands the library pairs produced on torch's stream
    (the RCCL all_to_all); HipBackend.build must order its own stream after
    it.  torch's stream is held back by a sleep kernel before the copy that
    produces the pairs: a build that does not wait reads zeros."""
    import torch
    import srd_shard as SH
    store = O.synth_store(300)
    ch = O.chain(store, store.size)
    host = np.array([[e["key_hash"], ((e["key_hash"] >> 48) << 48) | e["meta_off"]] for e in ch],
                    np.uint64).reshape(-1)
    src = torch.from_numpy(host.view(np.int64)).cuda()
    dst = torch.zeros_like(src)
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000_000)  # ~0.1 s of GPU time on torch's current stream
    dst.copy_(src)
    ok, op = SH.HipBackend(ctx, 0).build(dst)
    got = dict(zip(ok.cpu().numpy().view(np.uint64).tolist(), op.cpu().numpy().view(np.uint64).tolist()))
    assert got == O.key_indexer_build(store, store.size)
