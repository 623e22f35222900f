"""The product multi-GPU path (srd_shard.sharded_validate_index + HipBackend)
with 2 and 3 ranks in separate processes sharing this box's one GPU (gloo for
the exchange; the driver's 8-GPU run uses RCCL): the merged global index
equals the oracle's KeyIndexer::build of the same whole store."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, n_total, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-simd-r-drive_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import srd_amd as S
    import srd_shard as SH
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        ctx = S.Context(0)
        first, cnt = SH.plan_entry_shards(n_total, world)[rank]
        lo, hi = S.synth_span(None, 0, first, cnt, 1000)
        span_off = lo - lo % S.SPAN_ALIGN
        buf = torch.zeros(S.padded_size(hi - span_off), dtype=torch.uint8, device="cuda:0")
        S.synth_span(buf.data_ptr(), span_off, first, cnt, 1000, ctx=ctx)
        res = SH.sharded_validate_index(SH.HipBackend(ctx, 0), buf, span_off, lo, hi, S.synth_store_len(n_total, 1000))
        q.put((rank, res.composed, res.final_len, res.n_chain, res.n_crc_bad, res.n_index,
               dict(zip(res.owner_keys.cpu().numpy().view(np.uint64).tolist(),
                        res.owner_packed.cpu().numpy().view(np.uint64).tolist()))))
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_open_two_processes(world):
    import torch.multiprocessing as mp
    import oracle as O
    n = 3001
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    store = O.synth_store(n, 1000)
    want = O.key_indexer_build(store, store.size)
    merged = {}
    for rank, composed, final_len, n_chain, n_bad, n_index, idx in out:
        assert (composed, final_len, n_chain, n_bad, n_index) == (True, store.size, n, 0, len(want))
        assert not (merged.keys() & idx.keys())
        merged.update(idx)
    assert merged == want


def _host_worker(rank, world, port, store_bytes, q):
    """sharded_open_host on the product path: cuts from srd_shard_cuts, the
    rank's span copied from the host store into HBM, HipBackend."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "rust-simd-r-drive_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import srd_amd as S
    import srd_shard as SH
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        ctx = S.Context(0)
        store = np.frombuffer(store_bytes, np.uint8)
        res = SH.sharded_open_host(SH.HipBackend(ctx, 0), store)
        q.put((rank, res.composed, res.final_len, res.n_chain, res.n_crc_bad, res.n_index,
               dict(zip(res.owner_keys.cpu().numpy().view(np.uint64).tolist(),
                        res.owner_packed.cpu().numpy().view(np.uint64).tolist())), res.retried))
        torch.cuda.synchronize()
        ctx.close()
    finally:
        dist.destroy_process_group()


def _run_host(world, store):
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_host_worker, args=(r, world, port, store.tobytes(), q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return out


def _zipf_host_store(n=1500):
    import srd_amd as S
    import oracle as O
    return O.synth_store(n, lens=S.zipf_lens(n, s=2.0))


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_open_host_zipf(world):
    """Arbitrary store (C3's Zipf sizes, 64 B .. 1 MiB, unaligned tails): byte
    cuts guessed by the host pre-pass, proven by the shards; the merged index
    equals the oracle's whole-file KeyIndexer::build."""
    import oracle as O
    store = _zipf_host_store()
    out = _run_host(world, store)
    want = O.key_indexer_build(store, store.size)
    merged = {}
    for rank, composed, final_len, n_chain, n_bad, n_index, idx, retried in out:
        assert (composed, final_len, n_chain, n_bad, n_index, retried) == (True, store.size, 1500, 0, len(want), False)
        assert not (merged.keys() & idx.keys())
        merged.update(idx)
    assert merged == want


def test_sharded_open_host_refutes_bad_cuts():
    """A forged tail under the cut target: the shard above it is unproven and
    is re-validated with its lower neighbour (the bytes sent rank to rank):
    composed, the index the oracle's.  A torn tail stays unproven after that
    retry, so the whole-file path decides (checked here against the oracle)."""
    import oracle as O
    import srd_amd as S
    from test_shard_gloo import fake_cut_store
    fake, _ = fake_cut_store()
    out = _run_host(2, fake)
    want = O.key_indexer_build(fake, fake.size)
    merged = {}
    for rank, composed, final_len, n_chain, n_bad, n_index, idx, retried in out:
        assert (composed, retried, final_len, n_index) == (True, True, fake.size, len(want))
        merged.update(idx)
    assert merged == want
    torn = np.concatenate([_zipf_host_store(600), np.frombuffer(b"CORRUPT", np.uint8)])
    out = _run_host(2, torn)
    assert all(not composed for _, composed, *_ in out)
    r = S.validate_index(torn)
    assert r.final_len == O.recover_valid_chain(torn)
    assert r.index() == O.key_indexer_build(torn, r.final_len)
