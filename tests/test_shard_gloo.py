"""The multi-GPU exchange protocol of srd_shard (boundary composition +
owner-partitioned index all_to_all) on CPU: world_size 2 and 3 over gloo.
The per-shard device work is replaced by the CPU oracle (test checker only);
the product HipBackend is covered by tests/test_gpu_shards.py on the GPU."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class OracleBackend:
    """Stand-in for HipBackend: same outputs, computed by the oracle."""

    def __init__(self, store):
        import oracle as O
        self.O, self.store = O, store
        self.flen = O.recover_valid_chain(store)
        self.chain = O.chain(store, self.flen)
        self.tails = {e["meta_off"] + 20: i for i, e in enumerate(self.chain)}

    def validate_span(self, buf, span_off, lo, hi, flags=0):
        ch = self.chain
        a = 0 if lo == 0 else self.tails.get(lo, -1) + 1
        b = self.tails.get(hi, -2) + 1
        proven = a >= 0 and b > a and (lo == 0 or ch[a]["prev_offset"] == lo)
        seg = ch[a:b] if proven else []
        latest = {}
        for e in seg:
            latest[e["key_hash"]] = ((e["key_hash"] >> 48) << 48) | e["meta_off"]
        from srd_shard import ShardStatus
        st = ShardStatus(bool(proven), lo, hi, len(seg), sum(1 - e["crc_ok"] for e in seg))
        k = torch.tensor(np.array(list(latest.keys()), np.uint64).view(np.int64))
        v = torch.tensor(np.array(list(latest.values()), np.uint64).view(np.int64))
        return st, k, v, seg

    def partition(self, keys, packed, world):
        ku = keys.numpy().view(np.uint64)
        own = ((ku >> np.uint64(32)) * np.uint64(world)) >> np.uint64(32)
        order = np.argsort(own, kind="stable")
        pairs = np.stack([keys.numpy()[order], packed.numpy()[order]], 1).reshape(-1)
        return torch.from_numpy(pairs.copy()), [int((own == w).sum()) for w in range(world)]

    def build(self, pairs):
        p = pairs.numpy().reshape(-1, 2)
        latest = {}
        for k, v in p:
            latest.pop(int(k), None)  # latest position wins; order = file order of the latest entry
            latest[int(k)] = int(v)
        return torch.tensor(list(latest.keys()), dtype=torch.int64), torch.tensor(list(latest.values()), dtype=torch.int64)


def _worker(rank, world, port, store_bytes, cuts, torn, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rust-simd-r-drive_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import srd_shard as SH
        store = np.frombuffer(store_bytes, np.uint8)
        be = OracleBackend(np.frombuffer(store_bytes[:len(store_bytes) - torn], np.uint8) if torn else store)
        full = OracleBackend(store)
        tails = [0] + [e["meta_off"] + 20 for e in full.chain]
        a, b = cuts[rank], cuts[rank + 1]
        lo, hi = tails[a], tails[b]
        file_len = store.size - torn
        if rank == world - 1:
            hi = file_len
        span_off = lo - lo % 16384
        buf = torch.from_numpy(store[span_off:hi].copy())
        res = SH.sharded_validate_index(be, buf, span_off, lo, hi, file_len)
        q.put((rank, res.composed, res.final_len, res.n_chain, res.n_index,
               dict(zip(res.owner_keys.numpy().view(np.uint64).tolist(), res.owner_packed.numpy().view(np.uint64).tolist()))))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, store, cuts, torn=0):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, store.tobytes(), cuts, torn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return sorted(out)


def _store():
    import random
    import xxhash
    import oracle as O
    rnd = random.Random(41)
    buf = bytearray()
    t = 0
    for _ in range(300):
        kh = xxhash.xxh3_64_intdigest(b"k%d" % rnd.randrange(70))
        if rnd.random() < 0.1:
            t = O.write_entries(buf, t, [(kh, b"\x00")], allow_null=True)
        else:
            t = O.write_entries(buf, t, [(kh, rnd.randbytes(rnd.choice([1, 9, 64, 500, 4096])))])
    return np.frombuffer(bytes(buf), np.uint8)


@pytest.mark.parametrize("world,cuts", [(2, [0, 150, 300]), (3, [0, 1, 200, 300])])
def test_sharded_exchange_matches_whole_file(world, cuts):
    import oracle as O
    store = _store()
    out = _run(world, store, cuts)
    want = O.key_indexer_build(store, store.size)
    merged = {}
    for rank, composed, final_len, n_chain, n_index, idx in out:
        assert composed and final_len == store.size and n_chain == 300 and n_index == len(want)
        for k, v in idx.items():
            assert k not in merged
            assert ((k >> 32) * world) >> 32 == rank  # owner partition
            merged[k] = v
    assert merged == want


def test_sharded_torn_tail_is_not_composed():
    store = _store()
    out = _run(2, store, [0, 150, 300], torn=9)
    assert all(not composed for _, composed, *_ in out)


# ---- shard boundaries of an arbitrary store (srd_shard_cuts host pre-pass)

def _zipf_store(n=400):
    import srd_amd as S
    import oracle as O
    lens = S.zipf_lens(n, s=2.0)
    lens = np.minimum(lens, 1 << 16)  # keep the CPU oracle fast; still 64 B .. 64 KiB, unaligned tails
    return O.synth_store(n, lens=lens)


def _true_tails(store):
    import oracle as O
    t = O.recover_valid_chain(store)
    return {0} | {e["meta_off"] + 20 for e in O.chain(store, t, compute_crc=False)}


@pytest.mark.parametrize("name", ["mixed", "zipf", "alignment", "tombstones", "overwrite_delete", "nested"])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_shard_cuts_are_chain_tails(name, world):
    sys.path[:0] = [os.path.join(ROOT, "rust-simd-r-drive_amd")]
    import srd_amd as S
    if name == "mixed":
        store = _store()
    elif name == "zipf":
        store = _zipf_store()
    else:
        store = np.fromfile(os.path.join(ROOT, "tests", "golden", name + ".bin"), np.uint8)
    cuts = S.shard_cuts(store, world)
    assert len(cuts) == world + 1 and cuts[0] == 0 and cuts[-1] == store.size
    assert cuts == sorted(cuts)
    tails = _true_tails(store)
    assert set(cuts[:-1]) <= tails, (cuts, sorted(tails)[:20])
    if store.size > 1 << 20:  # large stores: every target has a tail within one entry below it
        assert len(set(cuts)) == world + 1


def test_shard_cuts_edge_cases():
    sys.path[:0] = [os.path.join(ROOT, "rust-simd-r-drive_amd")]
    import srd_amd as S
    assert S.shard_cuts(np.zeros(0, np.uint8), 4) == [0, 0, 0, 0, 0]
    z = np.zeros(100000, np.uint8)  # zero bytes look like p == 0 nodes everywhere: never a cut
    assert S.shard_cuts(z, 3) == [0, 0, 0, z.size]
    g = np.fromfile(os.path.join(ROOT, "tests", "golden", "garbage_1k.bin"), np.uint8)
    c = S.shard_cuts(g, 2)
    assert c[0] == 0 and c[-1] == g.size


def _host_worker(rank, world, port, store_bytes, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rust-simd-r-drive_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import srd_shard as SH
        store = np.frombuffer(store_bytes, np.uint8)
        res = SH.sharded_open_host(OracleBackend(store), store)
        q.put((rank, res.composed, res.final_len, res.n_chain, res.n_index,
               dict(zip(res.owner_keys.numpy().view(np.uint64).tolist(), res.owner_packed.numpy().view(np.uint64).tolist())),
               res.retried))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_open_host_byte_cuts(world):
    """Arbitrary store (Zipf sizes, unaligned tails): cuts from the pre-pass,
    spans copied from the host store, index equal to the whole-file build."""
    import oracle as O
    store = _zipf_store()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_worker, args=(r, world, port, store.tobytes(), q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    want = O.key_indexer_build(store, store.size)
    merged = {}
    for rank, composed, final_len, n_chain, n_index, idx, retried in out:
        assert composed and not retried and final_len == store.size and n_chain == 400 and n_index == len(want)
        assert not (merged.keys() & idx.keys())
        merged.update(idx)
    assert merged == want


def fake_cut_store():
    """A store whose byte-balanced cut lands in a 200 KB payload that holds a
    forged metadata record (prev = the real previous tail) below the target:
    srd_shard_cuts picks the forged tail, and composition must refute it."""
    import oracle as O
    rnd = np.random.default_rng(7)

    def build(fake_off):
        buf, t = bytearray(), 0
        for i in range(30):
            t = O.write_entries(buf, t, [(1000 + i, rnd.bytes(4096))])
        t_prev = t
        big = bytearray(rnd.bytes(200000))
        if fake_off is not None:
            big[fake_off:fake_off + 20] = (77).to_bytes(8, "little") + t_prev.to_bytes(8, "little") + b"\x01\x02\x03\x04"
        t = O.write_entries(buf, t, [(2000, bytes(big))])
        for i in range(30):
            t = O.write_entries(buf, t, [(3000 + i, rnd.bytes(4096))])
        return np.frombuffer(bytes(buf), np.uint8), t_prev

    s, t_prev = build(None)
    start = t_prev + ((64 - t_prev % 64) % 64)
    off = s.size // 2 - start - 520
    s, _ = build(off)
    return s, start + off + 20


def test_fake_tail_cut_is_refuted():
    sys.path[:0] = [os.path.join(ROOT, "rust-simd-r-drive_amd")]
    import srd_amd as S
    store, fake = fake_cut_store()
    assert S.shard_cuts(store, 2)[1] == fake
    assert fake not in _true_tails(store)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_worker, args=(r, 2, port, store.tobytes(), q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    # the forged cut leaves a shard unproven; the retry with its lower
    # neighbour composes, and the index is the whole-file one
    import oracle as O
    want = O.key_indexer_build(store, store.size)
    merged = {}
    for rank, composed, final_len, n_chain, n_index, idx, retried in out:
        assert composed and retried and final_len == store.size and n_index == len(want)
        merged.update(idx)
    assert merged == want


@pytest.mark.parametrize("proven,cuts,want", [
    ([True, False], [0, 5, 9], [(0, 1)]),
    ([False, True], [0, 5, 9], [(0, 0)]),
    ([True, True, False, False, True], [0, 1, 2, 3, 4, 5], [(1, 3)]),
    ([True, True, False], [0, 4, 4, 9], [(0, 2)]),  # the empty shard 1 is skipped
    ([False, True, False], [0, 4, 4, 9], [(0, 2)]),  # only an empty shard between two runs: they merge
    ([False, True, False], [0, 4, 6, 9], [(0, 0), (1, 2)]),  # a non-empty proven shard between: two runs
])
def test_neighbour_runs(proven, cuts, want):
    sys.path[:0] = [os.path.join(ROOT, "rust-simd-r-drive_amd")]
    import srd_shard as SH
    assert SH.neighbour_runs(proven, cuts) == want


def _forged_worker(rank, world, port, store_bytes, q, lower, members):
    """sharded_validate_index on the forged-cut store over the ranks `members`
    (a subgroup of the world; the others only join new_group), each member's
    span starting `lower` alignment steps below span_of(lo)."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "rust-simd-r-drive_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = dist.new_group(members)
        if rank in members:
            import srd_amd as S
            import srd_shard as SH
            store = np.frombuffer(store_bytes, np.uint8)
            gr = dist.get_rank(g)
            lo, hi = SH.plan_byte_shards(store, len(members))[gr]
            span_off = max(0, SH.span_of(lo) - lower * S.SPAN_ALIGN)
            buf = torch.zeros(S.padded_size(hi - span_off) if hi > lo else 1, dtype=torch.uint8)
            if hi > lo:
                buf[: hi - span_off].copy_(torch.from_numpy(store[span_off:hi].copy()))
            res = SH.sharded_validate_index(OracleBackend(store), buf, span_off, lo, hi, int(store.size), g)
            q.put((gr, res.composed, res.retried, res.final_len, res.n_index,
                   dict(zip(res.owner_keys.numpy().view(np.uint64).tolist(),
                            res.owner_packed.numpy().view(np.uint64).tolist()))))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,members,lower", [(6, [0, 1, 2, 3, 4, 5], 1), (3, [1, 2], 0)])
def test_neighbour_retry_lower_span_and_subgroup(world, members, lower):
    """The retry with the lower neighbour (a forged cut) when the neighbour's
    span starts below span_of(lo) (any 16 KiB multiple <= lo is allowed), and
    inside a process subgroup (send / recv address global ranks).  Six
    shards: the forged cut is cut 3, shards 2 and 3 (ending / starting at it)
    are unproven, and the neighbour is shard 1, whose span lies above 0."""
    import oracle as O
    store, _ = fake_cut_store()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_forged_worker, args=(r, world, port, store.tobytes(), q, lower, members))
             for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in members)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    want = O.key_indexer_build(store, store.size)
    merged = {}
    for gr, composed, retried, final_len, n_index, idx in out:
        assert composed and retried and final_len == store.size and n_index == len(want)
        assert not (merged.keys() & idx.keys())
        merged.update(idx)
    assert merged == want
