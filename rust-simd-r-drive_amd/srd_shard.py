"""Multi-GPU open of one store sharded by entry range --
the torch.distributed variant, NOT the product path of bench.py.

The product multi-GPU open is srd_validate_index_multi_device /
srd_validate_index_multi (include/srd_amd.h): ONE process drives every GPU of
the node (data_store.rs:84-117 is one call; north_star says "without RCCL"),
with persistent per-context host threads and xGMI peer reads for the index
exchange.  This module keeps the one-process-per-GPU formulation (gloo /
RCCL collectives for the composition check and the index all_to_all) for
callers that already run one rank per GPU; its protocol is tested on CPU with
gloo (tests/test_shard_gloo.py) and its HIP backend on one GPU
(tests/test_gpu_shard_dist.py).

One process per GPU.  Rank r holds the file bytes of entries
[first_r, first_r + n_r) in its HBM (plus < 16 KiB of the previous shard as a
halo, so the span starts on a 16 KiB boundary) and proves, with
srd_validate_span_device, that the backward chain from its upper tail hi_r
reaches an entry whose prev_offset is its lower tail lo_r.  No data-path
collective is needed for that: shards are independent.

The exchange step is small and real:
  1. boundaries: all_gather of (proven, lo, hi, n_chain, n_crc_bad) and the
     rank's per-owner index counts (so no separate count exchange) -- the
     shard chains compose into the whole file's chain iff every shard is
     proven, lo_0 == 0, hi_r == lo_{r+1} and hi_{W-1} == file_len.  That is
     recover_valid_chain's answer (data_store.rs:383-482) for a clean store:
     final_len = file_len.  Anything else (a torn tail, a corrupt shard) is
     decided by the whole-file path, whose byte-wise outer loop is global.
  2. index: KeyIndexer::build (key_indexer.rs:98-124) is latest-wins over the
     whole chain, so keys that live in several shards must meet.  Each rank
     partitions its shard-local index by owner = ((key_hash >> 32) * W) >> 32,
     an all_to_all moves the pairs to their owners (16 B per key), and each
     owner runs the bucketed build over the runs it received, which arrive in
     shard order = file order, so latest-wins-by-position stays exact.  The
     global index is the disjoint union of the owners' indexes; its size is
     an all_reduce(SUM).

The device work goes through a backend object so that the protocol can be
exercised on CPU with the gloo backend in the tests (tests/test_shard_gloo.py
plugs in the oracle there, as the checker); `HipBackend` is the product and
has no fallback.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

import srd_amd as S


def plan_entry_shards(n_entries: int, world: int) -> list[tuple[int, int]]:
    """Equal entry-count ranges (first, count), one per rank."""
    base, extra = divmod(n_entries, world)
    out, first = [], 0
    for r in range(world):
        n = base + (1 if r < extra else 0)
        out.append((first, n))
        first += n
    return out


@dataclass
class ShardStatus:
    proven: bool
    lo: int
    hi: int
    n_chain: int
    n_crc_bad: int


@dataclass
class ShardedResult:
    final_len: int          # whole-file recover_valid_chain result (file_len when all shards compose)
    composed: bool          # False -> the caller must run the whole-file path
    n_chain: int            # chain entries over all shards
    n_crc_bad: int
    n_index: int            # global KeyIndexer size (disjoint union of owner indexes)
    owner_keys: torch.Tensor    # this rank's part of the global index (key_hash as int64 bits)
    owner_packed: torch.Tensor  # pack(tag16, offset48) as int64 bits
    local: object = None        # backend's shard-local result (chain arrays in the context's device
                                # buffers: valid until the next call on that context), or the
                                # exception of a failed shard
    retried: bool = False       # a run of unproven shards was re-validated with its lower neighbour
    lo: int = 0                 # this rank's shard after that re-validation (lo == hi: emptied)
    hi: int = 0


class HipBackend:
    """Device work on this rank's GPU through the C ABI (libsrd_amd.so)."""

    def __init__(self, ctx: S.Context, device: int):
        self.ctx, self.device = ctx, device

    def _after_torch(self, t: torch.Tensor):
        # inputs written on torch's stream (copies, the RCCL collectives):
        # the library's own stream waits for them (an event, no host sync)
        torch.cuda.ExternalStream(self.ctx.stream, device=t.device).wait_stream(torch.cuda.current_stream(t.device))

    def validate_span(self, buf: torch.Tensor, span_off: int, lo: int, hi: int, flags: int = 0):
        self._after_torch(buf)
        r = S.validate_span_device(buf.data_ptr(), span_off, lo, hi, flags, self.ctx)
        # the chain reaches this shard's tail (lo == 0 is the whole-file rule:
        # a torn tail's chain may end below hi in either mode)
        proven = r.mode != S.SRD_MODE_SPAN_UNPROVEN and r.final_len == hi
        st = ShardStatus(bool(proven), lo, hi, int(r.n_chain), int(r.n_crc_bad))
        keys = S.device_view(r.index_key_hash, r.n_index, np.uint64, self.device)
        packed = S.device_view(r.index_packed, r.n_index, np.uint64, self.device)
        return st, keys, packed, r

    def partition(self, keys: torch.Tensor, packed: torch.Tensor, world: int):
        n = keys.numel()
        pairs = torch.empty(2 * max(n, 1), dtype=torch.int64, device=keys.device)
        counts = S.index_partition_device(keys.data_ptr(), packed.data_ptr(), n, world, pairs.data_ptr(), self.ctx)
        return pairs[: 2 * n], counts

    def build(self, pairs: torch.Tensor):
        n = pairs.numel() // 2
        ok = torch.empty(max(n, 1), dtype=torch.int64, device=pairs.device)
        op = torch.empty(max(n, 1), dtype=torch.int64, device=pairs.device)
        self._after_torch(pairs)  # the RCCL all_to_all wrote `pairs` on torch's stream
        ni = S.index_build_device(pairs.data_ptr(), n, ok.data_ptr(), op.data_ptr(), self.ctx)
        return ok[:ni], op[:ni]


def plan_byte_shards(file: np.ndarray, world: int) -> list[tuple[int, int]]:
    """(lo, hi) entry tails per rank for an arbitrary host store: the cuts of
    the host pre-pass srd_shard_cuts (byte-balanced guesses that the
    composition check below proves or refutes)."""
    c = S.shard_cuts(file, world)
    return [(c[r], c[r + 1]) for r in range(world)]


def span_of(lo: int) -> int:
    """First byte a rank holds: lo rounded down to the span alignment (16 KiB)."""
    return lo - lo % S.SPAN_ALIGN


def sharded_open_host(backend, file: np.ndarray, group=None) -> ShardedResult:
    """DataStore::open over a host store (the mmap) on W ranks: every rank
    computes the same cuts, copies its span [span_off, hi) into its HBM and
    joins sharded_validate_index.  `composed` False (a torn tail, corruption or
    a cut that is not a real chain tail) means the whole-file path decides."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = plan_byte_shards(file, world)[rank]
    span_off = span_of(lo)
    dev = backend_device(backend)
    buf = torch.zeros(S.padded_size(hi - span_off) if hi > lo else 1, dtype=torch.uint8, device=dev)
    if hi > lo:
        buf[: hi - span_off].copy_(torch.from_numpy(np.ascontiguousarray(file[span_off:hi])))
    return sharded_validate_index(backend, buf, span_off, lo, hi, int(file.size), group)


def backend_device(backend) -> torch.device:
    d = getattr(backend, "device", None)
    return torch.device("cpu") if d is None else torch.device("cuda", d) if isinstance(d, int) else torch.device(d)


def neighbour_runs(proven: list[bool], cuts: list[int]) -> list[tuple[int, int]]:
    """The re-validation plan when shards are unproven (srd_validate_index_multi's
    rule): each run [i, b] of consecutive unproven shards is taken over by its
    lower neighbour a -- the first non-empty shard below (an empty shard proves
    nothing; its cut may be the forged one), or the run itself at shard 0 --
    which re-validates [cuts[a], cuts[b+1]): both ends are tails the
    neighbours proved.  Returns [(a, b)]."""
    runs, floor, i, n = [], 0, 0, len(proven)
    while i < n:
        if proven[i]:
            i += 1
            continue
        b = i
        while b + 1 < n and not proven[b + 1]:
            b += 1
        a = i - 1 if i else 0
        while a > floor and cuts[a] == cuts[a + 1]:
            a -= 1
        if runs and a <= floor and cuts[a] == cuts[a + 1]:
            # only empty shards back to the previous run: no tail between them
            # is proven, so this run joins that one (both would otherwise end
            # or start at the suspect cut)
            runs[-1] = (runs[-1][0], b)
        else:
            runs.append((max(a, floor), b))
        floor = b + 1
        i = b + 1
    return runs


def sharded_validate_index(backend, buf: torch.Tensor, span_off: int, lo: int, hi: int, file_len: int,
                           group=None, retry: bool = True) -> ShardedResult:
    """One rank's part of the sharded open: validate its shard, check the
    composition, exchange the index.  Collective over `group`.

    Shards left unproven by a cut that is no chain tail are retried once with
    their lower neighbour (neighbour_runs): the run's ranks send their bytes
    to the neighbour rank (point-to-point), which re-validates the merged
    span; the others keep their shards.  Only what is still unproven (a torn
    tail, corruption) returns composed = False for the whole-file path."""
    world = dist.get_world_size(group)
    dev = buf.device
    # collectives run where the backend lives: device memory for nccl (RCCL
    # over xGMI), host memory for gloo (CPU tests, several ranks on one GPU)
    cd = torch.device("cpu") if dist.get_backend(group) == "gloo" else dev
    keys = packed = torch.empty(0, dtype=torch.int64, device=dev)
    local = None
    if lo == hi:  # an empty shard (srd_shard_cuts found no tail in its range): composes trivially
        st = ShardStatus(True, lo, hi, 0, 0)
    else:
        # a rank whose shard fails (an argument, capacity or allocation error)
        # still joins every collective below with proven = False, so all
        # ranks reach the same "not composed" decision (no rank blocks)
        try:
            st, keys, packed, local = backend.validate_span(buf, span_off, lo, hi)
        except (S.SrdError, RuntimeError) as e:
            st = ShardStatus(False, lo, hi, 0, 0)
            local = e
    # owner partition of the shard-local index (needed only when the shards
    # compose, but done first so that one all_gather carries both the
    # boundary rows and every rank's per-owner send counts)
    if keys.numel():
        pairs, counts = backend.partition(keys, packed, world)
    else:
        pairs, counts = torch.empty(0, dtype=torch.int64, device=dev), [0] * world
    # 1. boundaries (+ the count matrix of the index all_to_all)
    w = 5 + world
    mine = torch.tensor([int(st.proven), st.lo, st.hi, st.n_chain, st.n_crc_bad] + list(counts),
                        dtype=torch.int64, device=cd)
    allst = torch.empty(world * w, dtype=torch.int64, device=cd)
    dist.all_gather_into_tensor(allst, mine, group=group)
    rows = allst.view(world, w).cpu().tolist()
    composed = all(r[0] for r in rows) and rows[0][1] == 0 and rows[-1][2] == file_len and all(
        rows[i][2] == rows[i + 1][1] for i in range(world - 1))
    n_chain = sum(r[3] for r in rows)
    n_bad = sum(r[4] for r in rows)
    cuts = [r[1] for r in rows] + [rows[-1][2]]
    hard = isinstance(local, Exception)
    errs = torch.tensor([int(hard)], dtype=torch.int64, device=cd)
    dist.all_reduce(errs, group=group)
    consistent = cuts[0] == 0 and cuts[-1] == file_len and all(rows[i][2] == rows[i + 1][1] for i in range(world - 1))
    if not composed and retry and not int(errs.item()) and consistent:
        return _retry_with_neighbours(backend, buf, span_off, lo, hi, file_len, group, [bool(r[0]) for r in rows],
                                      cuts)
    if not composed:
        empty = torch.empty(0, dtype=torch.int64, device=dev)
        return ShardedResult(0, False, 0, 0, 0, empty, empty, local, lo=lo, hi=hi)
    # 2. index exchange: pairs to their owners
    me = dist.get_rank(group)
    rc = [rows[r][5 + me] for r in range(world)]
    got = torch.empty(2 * sum(rc), dtype=torch.int64, device=cd)
    dist.all_to_all_single(got, pairs.to(cd), [2 * c for c in rc], [2 * c for c in counts], group=group)
    okeys, opacked = backend.build(got.to(dev))
    ni = torch.tensor([okeys.numel()], dtype=torch.int64, device=cd)
    dist.all_reduce(ni, group=group)
    return ShardedResult(file_len, True, n_chain, n_bad, int(ni.item()), okeys, opacked, local, lo=lo, hi=hi)


def _retry_with_neighbours(backend, buf, span_off, lo, hi, file_len, group, proven, cuts) -> ShardedResult:
    """Ranks a+1..b of a run send their bytes [lo_i, hi_i) to rank a, which
    appends them to its span: its new shard is [cuts[a], cuts[b+1]); the
    senders' shards become empty at cuts[b+1].  Then the normal protocol,
    without a second retry."""
    me = dist.get_rank(group)
    dev = buf.device
    cd = torch.device("cpu") if dist.get_backend(group) == "gloo" else dev
    runs = neighbour_runs(proven, cuts)
    # send / recv take GLOBAL ranks; the run plan speaks of ranks in `group`
    glob = (lambda r: r) if group is None or group is dist.group.WORLD else (
        lambda r: dist.get_global_rank(group, r))
    n_lo, n_hi, n_buf, n_off = lo, hi, buf, span_off
    for a, b in runs:
        if a < me <= b:  # a sender: its bytes go to rank a, its shard empties
            if hi > lo:
                dist.send(buf[lo - span_off: hi - span_off].contiguous().to(cd), glob(a), group=group)
            n_lo = n_hi = cuts[b + 1]
            n_buf = torch.empty(0, dtype=torch.uint8, device=dev)
            n_off = n_lo - n_lo % S.SPAN_ALIGN
        elif me == a:  # the neighbour: its span [span_off, hi) + the run's bytes
            parts = [buf[: hi - span_off] if hi > lo else torch.empty(0, dtype=torch.uint8, device=dev)]
            for i in range(a + 1, b + 1):
                if cuts[i + 1] > cuts[i]:
                    t = torch.empty(cuts[i + 1] - cuts[i], dtype=torch.uint8, device=cd)
                    dist.recv(t, glob(i), group=group)
                    parts.append(t.to(dev))
            n_lo = cuts[a]
            n_hi = cuts[b + 1]
            # the merged bytes start at the neighbour's span (any 16 KiB
            # multiple <= lo: the span keeps its offset), or -- an empty
            # neighbour -- at its cut (the bytes below a shard's lower tail
            # are never read as entries: zeros are fine there)
            n_off = span_off if hi > lo else n_lo - n_lo % S.SPAN_ALIGN
            start = span_off if hi > lo else cuts[a + 1]
            merged = torch.cat([p.reshape(-1) for p in parts])
            n_buf = torch.zeros(S.padded_size(n_hi - n_off) if n_hi > n_lo else 1, dtype=torch.uint8, device=dev)
            n_buf[start - n_off: start - n_off + merged.numel()].copy_(merged)
    res = sharded_validate_index(backend, n_buf, n_off, n_lo, n_hi, file_len, group, retry=False)
    res.retried = True
    return res
