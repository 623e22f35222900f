"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
golden fixtures.  Bit-exact for every integer output: final_len, the chain
(meta_off, key_hash, prev_offset, payload_start, payload_len, stored and
computed CRC, crc_ok) and the KeyIndexer map."""
import os
import random
import struct
import zlib

import numpy as np
import pytest
import xxhash

import oracle as O
import srd_amd as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = S.Context(0)
    yield c
    c.close()


def check_against_oracle(data, ctx, flags=0, name=""):
    a = O.as_u8(data)
    want_len = O.recover_valid_chain(a)
    r = S.validate_index(a, flags, ctx)
    assert r.final_len == want_len, (name, r.final_len, want_len)
    ch = O.chain(a, want_len)
    assert r.n_chain == len(ch), (name, r.n_chain, len(ch))
    if ch:
        for k in ("meta_off", "key_hash", "prev_offset", "payload_start", "payload_len", "crc_stored",
                  "crc_computed", "crc_ok"):
            got = getattr(r, k).astype(np.uint64)
            exp = np.array([e[k] for e in ch], np.uint64)
            bad = np.nonzero(got != exp)[0]
            assert bad.size == 0, (name, k, bad[:5], got[bad[:5]], exp[bad[:5]])
    assert r.index() == O.key_indexer_build(a, want_len), name
    assert r.n_crc_bad == sum(1 - e["crc_ok"] for e in ch)
    return r


@pytest.mark.parametrize("flags", [0, S.SRD_FLAG_FORCE_FULL])
def test_golden_fixtures(golden_cases, ctx, flags):
    for name, (data, m) in golden_cases.items():
        r = S.validate_index(data, flags, ctx)
        assert r.final_len == m["final_len"], name
        assert r.n_chain == len(m["chain"]), name
        for i, e in enumerate(m["chain"]):
            assert int(r.meta_off[i]) == e["meta_off"], name
            assert int(r.key_hash[i]) == int(e["key_hash"], 16), name
            assert int(r.payload_start[i]) == e["payload_start"], name
            assert int(r.payload_len[i]) == e["payload_len"], name
            assert int(r.crc_stored[i]) == e["crc_stored"], name
            assert int(r.crc_computed[i]) == e["crc_computed"], (name, i)
            assert int(r.crc_ok[i]) == e["crc_ok"], name
        assert r.index() == {int(k, 16): int(v, 16) for k, v in m["index"].items()}, name


def test_recover_and_key_indexer_api(golden_cases, ctx):
    for name, (data, m) in golden_cases.items():
        assert S.recover_valid_chain(data, ctx) == m["final_len"], name
        ki = S.KeyIndexer.build(data[: m["final_len"]], m["final_len"], ctx)
        assert ki.index == {int(k, 16): int(v, 16) for k, v in m["index"].items()}, name


def test_xxh3_reference_goldens(ref_goldens, ctx):
    # tests/hash_stability_tests.rs:16-72 through compute_hash_batch
    keys = [bytes.fromhex(k) for k in ref_goldens["xxh3_64"]]
    got = S.compute_hash_batch(keys, ctx)
    assert got == [int(v, 16) for v in ref_goldens["xxh3_64"].values()]
    for g in ref_goldens["namespace"]:  # hash_stability_tests.rs:76-100
        a, b = S.compute_hash_batch([g["prefix"].encode(), g["key"].encode()], ctx)
        assert struct.pack("<QQ", a, b).hex() == g["out"]


def test_xxh3_random_lengths(ctx):
    rnd = random.Random(7)
    keys = [rnd.randbytes(n) for n in list(range(0, 260)) + [300, 1000, 1024, 1025, 2048, 5000]]
    assert S.compute_hash_batch(keys, ctx) == [xxhash.xxh3_64_intdigest(k) for k in keys]


def test_crc32_batch(ref_goldens, ctx):
    rnd = random.Random(3)
    buf = rnd.randbytes(300_000)
    offs, lens = [], []
    for n in list(range(0, 130)) + [4095, 4096, 4097, 8192 + 5, 100_000]:
        o = rnd.randrange(0, len(buf) - n)
        offs.append(o)
        lens.append(n)
    got = S.crc32_batch(buf, offs, lens, ctx)
    assert [int(x) for x in got] == [zlib.crc32(buf[o:o + n]) for o, n in zip(offs, lens)]
    for hexd, want in ref_goldens["crc32"].items():
        assert S.compute_checksum(bytes.fromhex(hexd)) == int(want, 16).to_bytes(4, "little")


def _device_synth(n, payload_len=4096, lens=None):
    import torch
    size = S.synth_store_len(n, payload_len, lens)
    t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
    S.synth_store_device(t.data_ptr(), n, payload_len, lens)
    torch.cuda.synchronize()
    return t[:size].cpu().numpy()


def test_device_writer_matches_oracle():
    # checksum-on-append writer (data_store.rs:847-939) vs the oracle writer
    assert np.array_equal(_device_synth(300), O.synth_store(300))
    lens = np.array([1, 2, 3, 63, 64, 65, 100, 4095, 4096, 4097, 9000, 70000, 5, 1 << 17], np.uint64)
    assert np.array_equal(_device_synth(len(lens), lens=lens), O.synth_store(len(lens), lens=lens))


@pytest.mark.parametrize("flags", [0, S.SRD_FLAG_FORCE_FULL])
def test_c1_store(ctx, flags):
    check_against_oracle(O.synth_store(1000), ctx, flags, "c1")


def _zipf_lens(n, seed=0x5EED0003, s=2.0):
    # C3 shape: 2^k, k=6..20, Zipf over r=k-5; L = 2^k - j for k>=7
    rng = np.random.default_rng(seed)
    r = np.arange(1, 16)
    p = 1.0 / r ** s
    p /= p.sum()
    k = rng.choice(np.arange(6, 21), size=n, p=p)
    j = rng.integers(0, 64, size=n)
    L = (1 << k) - np.where(k >= 7, j, 0)
    return L.astype(np.uint64)


def test_full_reason_codes(ctx):
    """srd_device_result.full_reason: why the optimistic pass did not decide
    (the full-pass fallback, ~1.8x a call, is visible).  An intact
    store decides (NONE); SRD_FLAG_FORCE_FULL; a cut deep inside an entry (no
    strong node at the start tail, data_store.rs:388-420); and the slot-space
    bound (capK >= 2^31 for a store above ~1 TiB) forced on a C1 store by a
    context created under SRD_SLOT_LIMIT_LOG2=10 -- the outputs stay the
    oracle's in every case."""
    st = O.synth_store(1000)
    r = check_against_oracle(st, ctx, 0, "intact")
    assert (r.mode, r.full_reason) == (S.SRD_MODE_OPTIMISTIC, S.SRD_FULL_NONE)
    r = check_against_oracle(st, ctx, S.SRD_FLAG_FORCE_FULL, "forced")
    assert (r.mode, r.full_reason) == (S.SRD_MODE_FULL, S.SRD_FULL_FORCED)
    r = check_against_oracle(st[: st.size - 1500], ctx, 0, "cut")
    assert r.mode == S.SRD_MODE_FULL and r.full_reason in (S.SRD_FULL_NO_START, S.SRD_FULL_UNPROVEN)
    os.environ["SRD_SLOT_LIMIT_LOG2"] = "10"
    try:
        c2 = S.Context(0)
    finally:
        del os.environ["SRD_SLOT_LIMIT_LOG2"]
    try:
        r = check_against_oracle(st, c2, 0, "slot limit")
        assert (r.mode, r.full_reason) == (S.SRD_MODE_FULL, S.SRD_FULL_SLOT_SPACE)
    finally:
        c2.close()


def _ctx_with_env(**env):
    """A context created under the given SRD_* environment knobs (read once at
    srd_ctx_create)."""
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return S.Context(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("block", [0, 100, 255])
def test_lookback_fallback(ctx, block):
    """The fused shape check's decoupled look-back (chain_finalize_kernel<true>)
    falls back safely when a chain block's spin bound runs out:
    SRD_LB_FAIL_BLOCK=b treats block b's look-back as timed out.  The block
    publishes a poisoned prefix, every later block's look-back fails on it, and
    the plan carries ST_LOOKBACK, so the call goes to the full pass
    (SRD_FULL_LOOKBACK) and still returns the oracle's outputs
    (data_store.rs:383-482, key_indexer.rs:98-124).  A normal context's next
    call decides optimistically again (stale granules carry another tag)."""
    lens = _zipf_lens(1500, seed=77)
    stores = {"c1": O.synth_store(1000), "zipf": O.synth_store(len(lens), lens=lens)}
    c = _ctx_with_env(SRD_LB_FAIL_BLOCK=block)
    try:
        for name, st in stores.items():
            r = check_against_oracle(st, c, 0, f"lb{block}:{name}")
            assert (r.mode, r.full_reason) == (S.SRD_MODE_FULL, S.SRD_FULL_LOOKBACK), (name, r.mode, r.full_reason)
    finally:
        c.close()
    r = check_against_oracle(stores["c1"], ctx, 0, "after")
    assert (r.mode, r.full_reason) == (S.SRD_MODE_OPTIMISTIC, S.SRD_FULL_NONE)


def test_unfused_glue_agrees(golden_cases):
    """Round 0 of the optimistic pass runs the shape check fused into
    chain_finalize_kernel<true> (neighbour-lane parent words, lazy start node,
    per-block root tail); SRD_GLUE_FUSED=0 runs check_kernel +
    chain_finalize_kernel<false>, the shape the retry rounds use.  Both must
    give the oracle's outputs on the golden, torn, flipped, tombstone and
    false-chain stores."""
    rnd = random.Random(31)
    lens = _zipf_lens(2000, seed=43)
    mixed = O.synth_store(len(lens), lens=lens)
    stores = {name: data for name, (data, m) in golden_cases.items()}
    stores["zipf"] = mixed
    for i in range(6):
        stores[f"cut{i}"] = mixed[: rnd.randrange(1, mixed.size)]
        flip = mixed.copy()
        flip[rnd.randrange(flip.size)] ^= 1 << rnd.randrange(8)
        stores[f"flip{i}"] = flip
    stores["corrupt"] = np.concatenate([mixed, np.frombuffer(b"CORRUPT", np.uint8)])
    buf = bytearray()
    t = 0
    for step in range(300):
        kh = xxhash.xxh3_64_intdigest(b"key%d" % rnd.randrange(40))
        if rnd.random() < 0.2:
            t = O.write_entries(buf, t, [(kh, b"\x00")], allow_null=True)
        else:
            t = O.write_entries(buf, t, [(kh, rnd.randbytes(rnd.choice([1, 20, 64, 700, 4096])) or b"\x01")])
    stores["tomb"] = bytes(buf)
    for fused in ("1", "0"):
        c = _ctx_with_env(SRD_GLUE_FUSED=fused)
        try:
            for name, data in stores.items():
                check_against_oracle(data, c, 0, f"fused{fused}:{name}")
            for rv in (False, True):
                data = _false_chain_store(rv)
                r = check_against_oracle(data, c, 0, f"fused{fused}:false{rv}")
                assert r.mode == S.SRD_MODE_OPTIMISTIC, (fused, rv, r.mode)
        finally:
            c.close()


def test_xcd_block_shares_repeated_calls():
    """The optimistic scan sizes its blocks by the measured speed of the XCD
    each one ran on in the previous call (XPart, srd_kernels.hip): the table
    is used from the second call on a store of the same span count and grid.
    Repeated calls -- small grids (C1: 16 blocks) and the full 256-block grid
    (20,000 x 4 KiB), a Zipf store, and a flipped byte between calls -- must
    give the oracle's outputs every time, and equal a context with the shares
    off (SRD_XPART=0).  The same calls run the per-store choice of the tile-load
    pattern (scan_variant_tune): both patterns, then the faster one."""
    rnd = random.Random(71)
    lens = _zipf_lens(3000, seed=5)
    stores = [O.synth_store(1000), O.synth_store(20_000), O.synth_store(len(lens), lens=lens)]
    on, off = S.Context(0), _ctx_with_env(SRD_XPART=0)
    try:
        for st in stores:
            loads = []
            for k in range(11):
                data = st
                if k == 9:  # (after the load-pattern trial: a store with a bad CRC may take the full pass)
                    data = st.copy()
                    data[rnd.randrange(data.size)] ^= 0x20
                r = check_against_oracle(data, on, 0, f"xpart{k}")
                loads.append(on.scan_loads())
                r2 = S.validate_index(data, 0, off)
                assert (r.final_len, r.n_chain, r.n_crc_bad) == (r2.final_len, r2.n_chain, r2.n_crc_bad)
                assert np.array_equal(r.crc_computed, r2.crc_computed) and r.index() == r2.index()
            # the tile-load pattern per store: a warm-up call, then calls
            # alternating the two patterns -- four, and up to eight while the
            # bests are within 2 % -- then the one with the faster best scan is kept (a
            # flipped byte keeps the store's span count: still the same
            # store); srd_ctx_scan_trial reports both bests
            ch, t_co, t_li = on.scan_trial()
            assert t_co > 0 and t_li > 0 and ch == (1 if t_li < t_co else 0), (ch, t_co, t_li)
            assert any(loads[: m + 1] == [0] + [k & 1 for k in range(m)] and set(loads[m + 1:]) == {ch}
                       for m in range(4, 9)), str((loads, ch, t_co, t_li))
    finally:
        on.close()
        off.close()


# key_hash pairs whose Xxh3BuildHasher hashes (XXH3-64 of the 8 LE bytes,
# key_indexer.rs:98-124) share the low 32 bits and the top 14 bits: the same
# index bucket at any bucket count and the same 32-bit partial key in the
# bucket records (found by a search over 2^25 keys; checked below)
PARTIAL_KEY_PAIRS = [(0x5A5A000000CC16BD, 0x5A5A000000E96736), (0x5A5A00000000992F, 0x5A5A0000003FE6D1),
                     (0x5A5A00000030969B, 0x5A5A000001ED8F14)]


@pytest.mark.parametrize("flags", [0, S.SRD_FLAG_FORCE_FULL])
def test_index_partial_key_collisions(ctx, flags):
    """The bucketed KeyIndexer::build keeps 8-byte bucket records (chain index
    + the low word of the key's hash) and deduplicates by that partial key;
    two different keys that share it must still both be indexed, each at its
    own latest entry (key_indexer.rs:98-124 is latest-wins per full key_hash):
    idx_dedup detects the mismatch against the full keys and redoes the
    bucket exactly.  Cases: a pair written once each, a pair with interleaved
    overwrites, a pair whose later key is a tombstone."""
    for a, b in PARTIAL_KEY_PAIRS:
        ha = xxhash.xxh3_64_intdigest(struct.pack("<Q", a))
        hb = xxhash.xxh3_64_intdigest(struct.pack("<Q", b))
        assert a != b and ha & 0xFFFFFFFF == hb & 0xFFFFFFFF and ha >> 50 == hb >> 50
    rnd = random.Random(61)
    (a1, b1), (a2, b2), (a3, b3) = PARTIAL_KEY_PAIRS
    seq = [(a1, 1), (b1, 1)]                                   # once each: b1 wins the partial key
    seq += [(a2, 1), (b2, 1), (a2, 1), (0x1234, 1), (b2, 1), (a2, 1)]  # overwrites interleaved
    seq += [(b3, 1), (a3, 1), (b3, 0)]                          # the later b3 a tombstone
    seq += [(rnd.getrandbits(64), 1) for _ in range(300)]
    rnd.shuffle(seq[11:])
    buf = bytearray()
    t = 0
    for kh, live in seq:
        if live:
            t = O.write_entries(buf, t, [(kh, rnd.randbytes(rnd.choice([5, 64, 700, 4096])) or b"\x01")])
        else:
            t = O.write_entries(buf, t, [(kh, b"\x00")], allow_null=True)
    r = check_against_oracle(bytes(buf), ctx, flags, "partial-key pairs")
    idx = r.index()
    for a, b in PARTIAL_KEY_PAIRS:
        assert a in idx and b in idx


def _ctx_with_loads(mode):
    os.environ["SRD_SCAN_LOADS"] = mode
    try:
        return S.Context(0)
    finally:
        del os.environ["SRD_SCAN_LOADS"]


@pytest.mark.parametrize("flags", [0, S.SRD_FLAG_FORCE_FULL])
def test_scan_load_patterns_agree(golden_cases, flags):
    """The scan loads a tile either coalesced + nontemporal with an in-register
    transpose to line-per-lane order or line per lane (the optimistic pass
    measures both per store and keeps the faster); SRD_SCAN_LOADS pins one
    pattern for a context.  Both must give
    the oracle's outputs on every golden fixture and on mixed-size, tombstone,
    torn and flipped stores, in both passes."""
    rnd = random.Random(23)
    lens = _zipf_lens(2500, seed=41)
    mixed = O.synth_store(len(lens), lens=lens)
    stores = {name: data for name, (data, m) in golden_cases.items()}
    stores["zipf"] = mixed
    stores["cut"] = mixed[: rnd.randrange(1, mixed.size)]
    flip = mixed.copy()
    flip[rnd.randrange(flip.size)] ^= 0x10
    stores["flip"] = flip
    stores["c1"] = O.synth_store(300)
    for mode in ("coal", "lines"):
        c = _ctx_with_loads(mode)
        try:
            for name, data in stores.items():
                check_against_oracle(data, c, flags, f"{mode}:{name}")
        finally:
            c.close()


@pytest.mark.parametrize("flags", [0, S.SRD_FLAG_FORCE_FULL])
def test_mixed_sizes(ctx, flags):
    lens = _zipf_lens(3000)
    check_against_oracle(O.synth_store(len(lens), lens=lens), ctx, flags, "zipf")


@pytest.mark.parametrize("flags", [0, S.SRD_FLAG_FORCE_FULL])
def test_root_entry_metadata_lines(ctx, flags):
    # the root entry (prev 0) has no candidate record: finalize takes its
    # metadata-line suffix from the per-tile values for lines 0 / 1 / 32 of a
    # tile, the slow kernel otherwise -- every first-entry length class
    for first in [4096, 8192, 64, 100, 127, 2048, 2100, 4160, 4200, 6144 + 40, 12288, 3000, 20, 63, 1 << 17]:
        lens = np.array([first] + [4096, 77, 2048, 5000] * 3, np.uint64)
        check_against_oracle(O.synth_store(len(lens), lens=lens), ctx, flags, f"root{first}")


@pytest.mark.parametrize("flags", [0, S.SRD_FLAG_FORCE_FULL])
def test_whole_tile_counts_around_the_inline_limit(ctx, flags):
    # a finalize lane combines up to LONG_TILES (16) whole tiles itself, a
    # longer entry takes the slow list (a wave each): entries of 1..22 whole
    # tiles between their start and metadata tiles, at shifting alignments
    # (the small entries between them move every start within its tile)
    rnd = random.Random(17)
    lens = []
    for w in range(1, 23):
        for d in (-70, -1, 0, 1, 63, 2100):
            lens += [w * 4096 + d, rnd.choice([20, 77, 1000, 4095, 2048 + 7])]
    lens = np.array(lens, np.uint64)
    check_against_oracle(O.synth_store(len(lens), lens=lens), ctx, flags, "tiles")


def test_tombstones_and_overwrites_random(ctx):
    rnd = random.Random(11)
    buf = bytearray()
    t = 0
    for step in range(400):
        k = rnd.randrange(60)
        kh = xxhash.xxh3_64_intdigest(b"key%d" % k)
        if rnd.random() < 0.2:
            t = O.write_entries(buf, t, [(kh, b"\x00")], allow_null=True)
        else:
            n = rnd.choice([1, 3, 8, 20, 64, 100, 700, 4096, 5000])
            pl = bytes(rnd.choice([0, 0, 0, 1, 2, 255]) for _ in range(n)) if rnd.random() < 0.5 else rnd.randbytes(n)
            if pl == b"\x00":
                pl = b"\x01"
            t = O.write_entries(buf, t, [(kh, pl)])
    for flags in (0, S.SRD_FLAG_FORCE_FULL):
        check_against_oracle(bytes(buf), ctx, flags, "tomb")


def test_torn_and_corrupted(ctx):
    rnd = random.Random(5)
    base = O.synth_store(40)
    lens = _zipf_lens(60, seed=9)
    mixed = O.synth_store(len(lens), lens=lens)
    for store in (base, mixed):
        for _ in range(12):
            cut = rnd.randrange(1, store.size)
            check_against_oracle(store[:cut], ctx, 0, "cut%d" % cut)
        for _ in range(6):
            b = store.copy()
            pos = rnd.randrange(b.size)
            b[pos] ^= 1 << rnd.randrange(8)
            check_against_oracle(b, ctx, 0, "flip%d" % pos)
        check_against_oracle(np.concatenate([store, np.frombuffer(b"CORRUPT", np.uint8)]), ctx, 0, "corrupt")


def _fuzz_store(rnd):
    """A random store built by batch_write_with_key_hashes (data_store.rs:847-939):
    overwrites from a small key pool, tombstones (a lone NULL byte,
    data_store.rs:995-1015), zero-heavy payloads, and payloads that embed a
    forged metadata record (key hash, a prev offset that is an earlier entry's
    end or junk, a nonzero checksum) at a random alignment -- false candidates
    for the scan's node filter (data_store.rs:404-470)."""
    buf = bytearray()
    t = 0
    ends = [0]
    for _ in range(rnd.randrange(1, 120)):
        batch = []
        for _ in range(rnd.choice([1, 1, 1, 2, 5])):
            kh = xxhash.xxh3_64_intdigest(b"fz%d" % rnd.randrange(40))
            kind = rnd.random()
            if kind < 0.12:
                batch.append((kh, b"\x00"))
                continue
            n = rnd.choice([1, 2, 7, 19, 20, 21, 63, 64, 65, 100, 500, 2047, 4096, 4100, 9000, rnd.randrange(1, 20000)])
            if kind < 0.35:
                pl = bytearray(n)  # zeros with a few set bytes: aligned zero halfwords everywhere
                for _ in range(max(1, n // 64)):
                    pl[rnd.randrange(n)] = rnd.randrange(1, 256)
            else:
                pl = bytearray(rnd.randbytes(n))
            if kind > 0.7 and n >= 40:
                prev = rnd.choice(ends) if rnd.random() < 0.8 else rnd.randrange(1 << 20)
                forged = struct.pack("<QQI", rnd.getrandbits(64), prev, rnd.randrange(1, 1 << 32))
                at = rnd.randrange(0, n - 20 + 1)
                pl[at:at + 20] = forged
            if bytes(pl) == b"\x00":
                pl = bytearray(b"\x01")
            batch.append((kh, bytes(pl)))
        t = O.write_entries(buf, t, batch, allow_null=True)
        ends.append(t)
    store = np.frombuffer(bytes(buf), np.uint8).copy()
    cut = rnd.random()
    if cut < 0.15 and store.size > 1:
        store = store[: rnd.randrange(1, store.size)]
    elif cut < 0.25 and len(ends) > 2:
        e = rnd.choice(ends[1:])
        store = store[: max(1, min(store.size, e + rnd.choice([-21, -20, -19, -1, 1, 7])))]
    elif cut < 0.35:
        tail = b"CORRUPT" if rnd.random() < 0.5 else rnd.randbytes(rnd.randrange(1, 300))
        store = np.concatenate([store, np.frombuffer(tail, np.uint8)])
    elif cut < 0.5 and store.size:
        pos = rnd.randrange(max(0, store.size - 20), store.size) if rnd.random() < 0.5 else rnd.randrange(store.size)
        store[pos] ^= 1 << rnd.randrange(8)
    elif cut < 0.55 and store.size >= 64:
        at = rnd.randrange(0, store.size - 63)
        store[at:at + 64] = 0
    return store


def test_fuzz_adversarial_stores(ctx):
    """120 random stores (_fuzz_store), each then torn, cut around an entry
    end, given a junk or b"CORRUPT" tail, bit-flipped (often inside the last
    metadata record) or given a zeroed line -- both passes against the
    oracle's recover_valid_chain / chain / KeyIndexer::build."""
    rnd = random.Random(int(os.environ.get("SRD_FUZZ_SEED", 2026)))  # (SRD_FUZZ_SEED / SRD_FUZZ_N: longer runs)
    modes = {S.SRD_MODE_OPTIMISTIC: 0, S.SRD_MODE_FULL: 0}
    for i in range(int(os.environ.get("SRD_FUZZ_N", 120))):
        store = _fuzz_store(rnd)
        for flags in (0, S.SRD_FLAG_FORCE_FULL):
            r = check_against_oracle(store, ctx, flags, "fuzz%d/%d" % (i, flags))
            if flags == 0:
                modes[r.mode] = modes.get(r.mode, 0) + 1
    # both passes ran on the default flags: most stores stay optimistic, the
    # damaged ones take the full pass
    assert modes[S.SRD_MODE_OPTIMISTIC] > 0 and modes[S.SRD_MODE_FULL] > 0, modes


@pytest.mark.parametrize("flags", [0, S.SRD_FLAG_FORCE_FULL])
def test_torn_tail_start_search(ctx, flags):
    """recover_valid_chain walks the cursor down from file_len and skips every
    t whose metadata fails entry_start < metadata_offset (data_store.rs:388-420).
    The optimistic pass starts at the largest such t within 256 bytes of
    file_len (find_top): b"CORRUPT" (persistence_tests.rs:126-173) and short
    junk stay in the optimistic mode; trailing zeros make the whole file one
    root entry (prev 0); a cut deep in the last entry, or junk longer than the
    window, goes to the full pass.  Every case against the oracle."""
    rnd = random.Random(17)
    base = O.synth_store(30, 100)
    lens = _zipf_lens(40, seed=3)
    mixed = O.synth_store(len(lens), lens=lens)
    tails = [b"CORRUPT", b"\x00", b"\x01" * 19, b"\x00" * 20, b"\x00" * 64, bytes(rnd.randrange(1, 256) for _ in range(100)),
             bytes(rnd.randrange(1, 256) for _ in range(255)), bytes(rnd.randrange(1, 256) for _ in range(300)),
             rnd.randbytes(64) + b"\x00" * 40]
    for store in (base, mixed):
        for i, tail in enumerate(tails):
            data = np.concatenate([store, np.frombuffer(tail, np.uint8)])
            check_against_oracle(data, ctx, flags, "tail%d" % i)
            r = S.validate_index(data, flags, ctx)
            want = O.recover_valid_chain(data)
            if flags == 0 and want == store.size and len(tail) <= 256:
                assert r.mode == S.SRD_MODE_OPTIMISTIC, ("tail%d" % i, r.mode)
        # cuts inside the last entry (its metadata or payload): junk below the window -> either mode, same answer
        for cut in (store.size - 1, store.size - 19, store.size - 21, store.size - 60, store.size - 300):
            check_against_oracle(store[:cut], ctx, flags, "cut%d" % cut)


def test_datastore_open_truncates_torn_tail(tmp_path, ctx):
    # persistence_tests.rs:126-173
    p = tmp_path / "store.bin"
    s = O.synth_store(20, 100)
    p.write_bytes(s.tobytes() + b"CORRUPT")
    with pytest.warns(UserWarning):
        ds = S.DataStore.open(str(p), ctx)
    assert os.path.getsize(p) == s.size and ds.tail_offset == s.size
    e = ds.read(b"bench-key-7")
    assert e is not None and e.is_valid_checksum()
    assert ds.len() == 20


def test_full_size_c2_properties(ctx):
    """C2 (1M x 4 KiB, 4.06 GiB) device-resident, checked by size-independent
    properties + a sampled oracle comparison."""
    import torch
    n = 1 << 20
    size = S.synth_store_len(n)
    t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
    S.synth_store_device(t.data_ptr(), n, 4096, ctx=ctx)
    torch.cuda.synchronize()
    r = S.validate_index_device(t.data_ptr(), size, 0, ctx)
    assert (r.final_len, r.n_chain, r.n_index, r.n_crc_bad, r.mode) == (size, n, n, 0, 0)
    host = t[:size].cpu().numpy()
    st = O.validate_index(host, 8)
    assert (st.final_len, st.n_chain, st.n_index, st.n_crc_bad) == (size, n, n, 0)
    # the full index against KeyIndexer::build (key_indexer.rs:98-124) of the
    # oracle: every (key_hash, packed) pair, not just the count
    keys, packed = O.key_indexer_arrays(host, size)
    ik = S.device_to_numpy(r.index_key_hash, n, np.uint64)
    iv = S.device_to_numpy(r.index_packed, n, np.uint64)
    o = np.argsort(ik, kind="stable")
    assert np.array_equal(ik[o], keys) and np.array_equal(iv[o], packed)
    # and every chain entry's computed CRC against the oracle's independent
    # PCLMUL CRC (entry_handle.rs:260-275)
    mo = S.device_to_numpy(r.meta_off, n, np.uint64)
    ln = S.device_to_numpy(r.payload_len, n, np.uint64)
    crc = S.device_to_numpy(r.crc_computed, n, np.uint32)
    assert np.array_equal(O.crc32_ranges(host, mo - ln, ln, threads=16), crc)
    del ik, iv, keys, packed, mo, ln, crc
    # flip one payload byte deep in the store -> exactly one bad CRC
    pos = 4160 * 777_777 + 1234
    t[pos] ^= 0x40
    r = S.validate_index_device(t.data_ptr(), size, 0, ctx)
    assert (r.final_len, r.n_chain, r.n_crc_bad) == (size, n, 1)
    # torn tail: drop the last 100 bytes -> oracle decides final_len
    cut = size - 100
    r = S.validate_index_device(t.data_ptr(), cut, 0, ctx)
    host[pos] ^= 0x40
    assert r.final_len == O.recover_valid_chain(host[:cut])


def _fake_record(key: int, prev: int, crc: int) -> bytes:
    return struct.pack("<QQI", key, prev, crc)


def _false_chain_store(root_variant):
    """Payload bytes that look like a chain of two metadata records (B links
    to A, A links nowhere -- or to a zero region, i.e. the root rule)."""
    buf = bytearray()
    t = 0
    t = O.write_entries(buf, t, [(0x1111, bytes(3000))])  # zero payload: a zero region for the root variant
    for i in range(5):
        t = O.write_entries(buf, t, [(0x2000 + i, random.Random(i).randbytes(700))])
    # fake A inside a payload (100 bytes into it): its "prev" is 25 (no record
    # there) or a zero region
    pl = bytearray(random.Random(99).randbytes(400))
    prev_a = 2000 if root_variant else 25
    pl[100:120] = _fake_record(0xAAAA, prev_a, 0x12345678)
    pad = (64 - len(buf) % 64) % 64
    a_pos = len(buf) + pad + 100
    t = O.write_entries(buf, t, [(0x3000, bytes(pl))])
    # fake B in a later payload, linking to A's tail
    pl2 = bytearray(random.Random(98).randbytes(500))
    pl2[200:220] = _fake_record(0xBBBB, a_pos + 20, 0x9ABCDEF0)
    t = O.write_entries(buf, t, [(0x3001, bytes(pl2))])
    for i in range(5):
        t = O.write_entries(buf, t, [(0x4000 + i, random.Random(50 + i).randbytes(300))])
    return bytes(buf)


@pytest.mark.parametrize("root_variant", [False, True])
def test_false_candidate_chain_is_pruned(ctx, root_variant):
    """A false chain in payload bytes (_false_chain_store): the reference never
    visits it (it only follows back-pointers from the tail); the optimistic
    pass must prune it and stay optimistic."""
    data = _false_chain_store(root_variant)
    r = check_against_oracle(data, ctx, 0, "fakechain")
    assert r.mode == S.SRD_MODE_OPTIMISTIC and r.final_len == len(data)


def test_c3_shape_200k_stays_optimistic(ctx):
    """C3-shaped store (Zipf 64 B..1 MiB), 200k entries, device-resident:
    the optimistic pass must prove it (structural false candidates are
    common: records shifted by +10 bytes whose 'prev' is the CRC's top half)."""
    import torch
    n = 200_000
    lens = S.zipf_lens(n)
    size = S.synth_store_len(n, 4096, lens)
    t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
    S.synth_store_device(t.data_ptr(), n, 4096, lens, seed=0x5EED0004, ctx=ctx)
    torch.cuda.synchronize()
    r = S.validate_index_device(t.data_ptr(), size, 0, ctx)
    assert (r.mode, r.final_len, r.n_chain, r.n_index, r.n_crc_bad) == (0, size, n, n, 0)
    host = t[:size].cpu().numpy()
    st = O.validate_index(host, 8)
    assert (st.final_len, st.n_chain, st.n_index, st.n_crc_bad) == (size, n, n, 0)
    # the full index against KeyIndexer::build (key_indexer.rs:98-124) of the
    # oracle: every (key_hash, packed) pair, not just the count
    keys, packed = O.key_indexer_arrays(host, size)
    ik = S.device_to_numpy(r.index_key_hash, n, np.uint64)
    iv = S.device_to_numpy(r.index_packed, n, np.uint64)
    o = np.argsort(ik, kind="stable")
    assert np.array_equal(ik[o], keys) and np.array_equal(iv[o], packed)
    # and every chain entry's computed CRC against the oracle's independent
    # PCLMUL CRC (entry_handle.rs:260-275)
    mo = S.device_to_numpy(r.meta_off, n, np.uint64)
    ln = S.device_to_numpy(r.payload_len, n, np.uint64)
    crc = S.device_to_numpy(r.crc_computed, n, np.uint32)
    assert np.array_equal(O.crc32_ranges(host, mo - ln, ln, threads=16), crc)
    del ik, iv, keys, packed, mo, ln, crc
    crc = S.device_to_numpy(r.crc_computed, n, np.uint32)
    mo = S.device_to_numpy(r.meta_off, n, np.uint64)
    ln = S.device_to_numpy(r.payload_len, n, np.uint64)
    assert np.array_equal(ln, lens)
    for i in np.random.default_rng(1).integers(0, n, 200):
        s0 = int(mo[i] - ln[i])
        assert int(crc[i]) == zlib.crc32(host[s0:int(mo[i])].tobytes())


@pytest.mark.parametrize("flags", [0, S.SRD_FLAG_FORCE_FULL])
def test_hot_key_overflows_its_bucket(ctx, flags):
    """One key overwritten 3000 times (more than a bucket's LDS table holds,
    IDX_TCAP = 2048) among 700 other keys, plus tombstones of the hot key:
    the index build's skewed-bucket fallback must still give latest-wins
    (key_indexer.rs:98-124) exactly as the oracle does."""
    rnd = random.Random(5)
    hot = xxhash.xxh3_64_intdigest(b"hot")
    buf, t = bytearray(), 0
    for i in range(3700):
        if i % 5 == 4 or rnd.random() < 0.6:
            kh = hot
        else:
            kh = xxhash.xxh3_64_intdigest(b"k%d" % rnd.randrange(700))
        if kh == hot and rnd.random() < 0.05:
            t = O.write_entries(buf, t, [(kh, b"\x00")], allow_null=True)
        else:
            pl = rnd.randbytes(rnd.choice([1, 8, 60, 64, 200]))
            t = O.write_entries(buf, t, [(kh, b"\x01" if pl == b"\x00" else pl)])
    r = check_against_oracle(bytes(buf), ctx, flags, "hot")
    assert r.n_index < 710


def test_index_build_device_hot_key(ctx):
    """srd_index_build_device (the sharded exchange's owner build) on pairs
    with one key repeated 5000 times: latest position wins."""
    import torch
    rnd = random.Random(9)
    keys = [0xABCDEF if rnd.random() < 0.7 else rnd.getrandbits(64) for _ in range(7000)]
    pairs = np.array([[k, 64 * i + 7] for i, k in enumerate(keys)], np.uint64).reshape(-1)
    d = torch.from_numpy(pairs.view(np.int64)).cuda()
    ok = torch.empty(7000, dtype=torch.int64, device="cuda")
    op = torch.empty(7000, dtype=torch.int64, device="cuda")
    n = S.index_build_device(d.data_ptr(), 7000, ok.data_ptr(), op.data_ptr(), ctx)
    want = {}
    for i, k in enumerate(keys):
        want[k] = ((k >> 48) << 48) | (64 * i + 7)
    got = dict(zip(ok[:n].cpu().numpy().view(np.uint64).tolist(), op[:n].cpu().numpy().view(np.uint64).tolist()))
    assert n == len(want) and got == want


def test_timing_levels_do_not_change_results():
    """srd_ctx_set_timing: events are opt-in (none by default); every level
    returns the same outputs, and srd_ctx_timings reports only what was timed."""
    import torch
    c = S.Context(0)
    try:
        n, L = 3000, 4096
        size = S.synth_store_len(n, L)
        t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
        S.synth_store_device(t.data_ptr(), n, L, seed=0x5EED0001, ctx=c)
        torch.cuda.synchronize()
        outs = []
        for level in (S.TIMING_NONE, S.TIMING_SCAN, S.TIMING_CALL, S.TIMING_NONE):
            c.set_timing(level)
            r = S.validate_index_device(t.data_ptr(), size, 0, c)
            outs.append((r.final_len, r.n_chain, r.n_crc_bad, r.n_index, r.mode))
            scan_ms, launches, total_ms = c.timings()
            if level == S.TIMING_NONE:
                assert (scan_ms, launches, total_ms) == (0.0, 0, 0.0)
            else:
                assert launches == 1 and scan_ms > 0
                assert (total_ms > 0) == (level == S.TIMING_CALL)
        assert all(o == (size, n, 0, n, S.SRD_MODE_OPTIMISTIC) for o in outs), outs
        # the scan's event pairs are read out by srd_ctx_timings: summed over
        # every call since the last read, also past the 64-pair ring
        c.set_timing(S.TIMING_SCAN)
        for calls in (3, 70):
            for _ in range(calls):
                S.validate_index_device(t.data_ptr(), size, 0, c)
            scan_ms, launches, _ = c.timings()
            assert launches == calls and scan_ms > 0
            assert c.timings()[:2] == (0.0, 0)
        with pytest.raises(S.SrdError):
            c.set_timing(3)
    finally:
        c.close()


@pytest.mark.parametrize("weights", ["1,1,1,1", "3,0.3,1,2", "per-slot-random", "1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,8",
                                     "not,numbers", "inf,1,1,1", "nan,1,1,1", "1e308,1e308,1e308,1e308"])
def test_scan_wave_shares(weights):
    """The scan's wave partition (ScanPart, SRD_SCAN_WEIGHTS: 4 or 16 shares, read at srd_ctx_create): any
    shares give the same outputs -- link2 finds each span's records through the inverse of the same
    partition.  A store large enough for the full 256-block grid, several spans per wave."""
    if weights == "per-slot-random":
        rng = random.Random(7)
        weights = ",".join(f"{rng.uniform(0.3, 3.0):.3f}" for _ in range(16))
    old = os.environ.get("SRD_SCAN_WEIGHTS")
    os.environ["SRD_SCAN_WEIGHTS"] = weights
    try:
        c = S.Context(0)
    finally:
        if old is None:
            os.environ.pop("SRD_SCAN_WEIGHTS", None)
        else:
            os.environ["SRD_SCAN_WEIGHTS"] = old
    try:
        check_against_oracle(_shares_store(), c, 0, f"shares {weights}")
    finally:
        c.close()


_SHARES_STORE = []


def _shares_store():
    # 50K x 4 KiB = 206 MB: 12.6K spans, the full 256-block grid, ~3 spans per scan wave
    if not _SHARES_STORE:
        _SHARES_STORE.append(O.synth_store(50000))
    return _SHARES_STORE[0]
