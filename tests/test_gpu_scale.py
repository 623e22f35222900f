"""GPU parity at BASELINE.json's full sizes and on the remaining boundary rows:

  - a8: the device Xxh3BuildHasher (xxh3_64(le8(key_hash)),
    xxh3_build_hasher.rs:11-13) against the fixtures' index_hash_le8 values;
  - 48-bit offsets: a span whose absolute offsets lie above 2^40 (the WIDE
    scan) equals the same entries at low offsets, shifted by 2^40;
  - the reference's own benchmark shape, benches/storage_benchmark.rs:20-26
    (1M entries of 8-byte little-endian counters, keys bench-key-{i}),
    bit-exact against the oracle in both modes;
  - the compiled C caller of include/srd_amd.h on the golden fixtures;
  - C3 at full size (10M Zipf-sized entries, 64 B .. 1 MiB) and C5 at full
    size (1M x 4 KiB written from pinned host memory), by size-independent
    properties: counts, sampled CRCs against zlib, one flipped byte = one bad
    CRC, the C5 bytes identical to the C2 store.
"""
import json
import os
import subprocess
import zlib

import numpy as np
import pytest
import xxhash

import oracle as O
import srd_amd as S

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ctx():
    c = S.Context(0)
    yield c
    c.close()


def test_index_hash_le8_goldens(golden_cases, ctx):
    import torch
    keys, want = [], []
    for name, (data, m) in golden_cases.items():
        for k, v in m.get("index_hash_le8", {}).items():
            keys.append(int(k, 16))
            want.append(int(v, 16))
    assert len(keys) > 50
    rnd = np.random.default_rng(3).integers(0, 2**63, 5000, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    keys += [0, 2**64 - 1] + [int(x) for x in rnd]
    want += [xxhash.xxh3_64_intdigest(k.to_bytes(8, "little")) for k in keys[len(want):]]
    d = torch.from_numpy(np.array(keys, np.uint64).view(np.int64)).cuda()
    out = torch.empty_like(d)
    S.index_hash_device(d.data_ptr(), d.numel(), out.data_ptr(), ctx)
    torch.cuda.synchronize()
    assert out.cpu().numpy().view(np.uint64).tolist() == want


def _span_result(ctx, lens, seed=0x5EED0007):
    """Entries 1.. of a synthetic store whose entry 0 ends at a 16 KiB boundary
    (lens[0] + 20 = lo): the span [lo, hi) validated in span mode."""
    import torch
    n = len(lens) - 1
    lo, hi = S.synth_span(None, 0, 1, n, 0, lens)
    assert lo % S.SPAN_ALIGN == 0
    t = torch.zeros(S.padded_size(hi - lo), dtype=torch.uint8, device="cuda")
    S.synth_span(t.data_ptr(), lo, 1, n, 0, lens, seed=seed, ctx=ctx)
    torch.cuda.synchronize()
    r = S.validate_span_device(t.data_ptr(), lo, lo, hi, 0, ctx)
    out = {"mode": r.mode, "final_len": r.final_len, "n_chain": r.n_chain, "n_crc_bad": r.n_crc_bad}
    for k, dt in (("meta_off", np.uint64), ("key_hash", np.uint64), ("prev_offset", np.uint64),
                  ("payload_start", np.uint64), ("payload_len", np.uint64), ("crc_stored", np.uint32),
                  ("crc_computed", np.uint32), ("crc_ok", np.uint8)):
        out[k] = S.device_to_numpy(getattr(r, k), r.n_chain, dt)
    out["index"] = dict(zip(S.device_to_numpy(r.index_key_hash, r.n_index).tolist(),
                            S.device_to_numpy(r.index_packed, r.n_index).tolist()))
    return lo, hi, out, t[: hi - lo].cpu().numpy()


def test_span_above_2_40_matches_low_offsets(ctx):
    """key_indexer.rs:12-15, 41-45: offsets are 48-bit.  The same entries at
    absolute offsets above 2^40 (WIDE scan: prev's bytes 5 may be nonzero)
    and at low offsets: every output equal up to the 2^40 shift."""
    body = np.minimum(S.zipf_lens(700, seed=21), 1 << 17)
    body[::7] = 8  # dense small entries too
    shift = 1 << 40
    lens_hi = np.concatenate([[shift + S.SPAN_ALIGN - 20], body]).astype(np.uint64)
    lens_lo = np.concatenate([[S.SPAN_ALIGN - 20], body]).astype(np.uint64)
    lo_h, hi_h, rh, bh = _span_result(ctx, lens_hi)
    lo_l, hi_l, rl, bl = _span_result(ctx, lens_lo)
    assert lo_h - lo_l == shift and hi_h - hi_l == shift
    assert rh["mode"] == rl["mode"] == S.SRD_MODE_OPTIMISTIC
    assert (rh["final_len"], rh["n_chain"], rh["n_crc_bad"]) == (hi_h, 700, 0)
    for k in ("meta_off", "prev_offset", "payload_start"):
        assert np.array_equal(rh[k] - np.uint64(shift), rl[k]), k
    for k in ("key_hash", "payload_len", "crc_stored", "crc_computed", "crc_ok"):
        assert np.array_equal(rh[k], rl[k]), k
    m48 = (1 << 48) - 1
    assert {k: v - shift for k, v in rh["index"].items()} == rl["index"]
    assert all((v & m48) >= shift for v in rh["index"].values())
    # the low-offset span against the oracle's whole store (entries 1..)
    store = O.synth_store(len(lens_lo), lens=lens_lo, seed=0x5EED0007)
    ch = O.chain_arrays(store, store.size)[1:]
    for k in ("meta_off", "key_hash", "prev_offset", "payload_start", "payload_len", "crc_stored", "crc_computed",
              "crc_ok"):
        assert np.array_equal(rl[k].astype(np.uint64), ch[k].astype(np.uint64)), k
    # the high span's bytes are the low span's bytes except the prev fields
    assert bh.size == bl.size


def _storage_benchmark_store(n=1_000_000):
    """benches/storage_benchmark.rs:20-26,55-68: key bench-key-{i}, payload =
    i as 8 little-endian bytes, written in batches of 1024 (the layout does
    not depend on the batching)."""
    kh = [xxhash.xxh3_64_intdigest(b"bench-key-%d" % i) for i in range(n)]
    buf = bytearray()
    t = 0
    for b0 in range(0, n, 1 << 16):
        t = O.write_entries(buf, t, [(kh[i], i.to_bytes(8, "little")) for i in range(b0, min(n, b0 + (1 << 16)))])
    return np.frombuffer(bytes(buf), np.uint8)


@pytest.mark.parametrize("flags", [0, S.SRD_FLAG_FORCE_FULL])
def test_storage_benchmark_shape_1m(ctx, flags):
    store = _storage_benchmark_store()
    assert store.size == 64 * 1_000_000 - 36  # entry i: payload at 64 i, 8 + 20 bytes
    r = S.validate_index(store, flags, ctx)
    ch = O.chain_arrays(store, store.size)
    assert (r.final_len, r.n_chain, r.n_crc_bad) == (store.size, 1_000_000, 0)
    for k in ("meta_off", "key_hash", "prev_offset", "payload_start", "payload_len", "crc_stored", "crc_computed",
              "crc_ok"):
        assert np.array_equal(getattr(r, k).astype(np.uint64), ch[k].astype(np.uint64)), k
    keys, packed = O.key_indexer_arrays(store, store.size)
    o = np.argsort(r.index_key_hash, kind="stable")
    assert np.array_equal(r.index_key_hash[o], keys) and np.array_equal(r.index_packed[o], packed)


def _abi_bin():
    return os.path.join(ROOT, "tests", "abi_c", "build", "srd_abi_check")


@pytest.mark.parametrize("n_ctx", [1, 3])
def test_c_caller_on_golden_fixtures(golden_cases, n_ctx):
    exe = _abi_bin()
    assert os.path.exists(exe), "build() compiles tests/abi_c"
    for name, (data, m) in golden_cases.items():
        path = os.path.join(ROOT, "tests", "golden", m["file"])
        p = subprocess.run([exe, path, str(m["final_len"]), str(len(m["chain"])), str(len(m["index"])), str(n_ctx)],
                           capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, (name, p.stdout, p.stderr)
        out = json.loads(p.stdout)
        assert out["bad"] == 0 and out["n_crc_bad"] == sum(1 - e["crc_ok"] for e in m["chain"]), name


def test_full_c3_properties(ctx):
    """C3 at its BASELINE size: 10M entries, Zipf over 2^k (k = 6..20, s = 2),
    unaligned tails -- ~67 GiB device-resident."""
    import torch
    n = 10_000_000
    lens = S.zipf_lens(n)
    size = S.synth_store_len(n, 4096, lens)
    assert size > 60 * 2**30
    t = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
    S.synth_store_device(t.data_ptr(), n, 4096, lens, seed=0x5EED0004, ctx=ctx)
    torch.cuda.synchronize()
    r = S.validate_index_device(t.data_ptr(), size, 0, ctx)
    assert (r.mode, r.final_len, r.n_chain, r.n_index, r.n_crc_bad) == (0, size, n, n, 0)
    mo = S.device_to_numpy(r.meta_off, n, np.uint64)
    ln = S.device_to_numpy(r.payload_len, n, np.uint64)
    crc = S.device_to_numpy(r.crc_computed, n, np.uint32)
    st = S.device_to_numpy(r.crc_stored, n, np.uint32)
    assert np.array_equal(ln, lens) and np.array_equal(crc, st)
    assert int(mo[-1]) + 20 == size and np.all(np.diff(mo.astype(np.int64)) > 0)
    # the whole index (key_indexer.rs:98-124) independently of the device: in
    # chain order (every key distinct), key i = python-xxhash's XXH3-64 of
    # b"bench-key-{i}", packed = (hash >> 48) << 48 | its metadata offset
    ik = S.device_to_numpy(r.index_key_hash, n, np.uint64)
    iv = S.device_to_numpy(r.index_packed, n, np.uint64)
    want = np.fromiter((xxhash.xxh3_64_intdigest(b"bench-key-%d" % i) for i in range(n)), np.uint64, n)
    assert np.array_equal(ik, want)
    assert np.array_equal(iv, ((want >> np.uint64(48)) << np.uint64(48)) | mo)
    del ik, iv, want
    for i in np.random.default_rng(5).integers(0, n, 300):
        s0 = int(mo[i] - ln[i])
        assert int(crc[i]) == zlib.crc32(t[s0:int(mo[i])].cpu().numpy().tobytes()), i
    # every entry's crc_computed against an independent CRC (entry_handle.rs:
    # 260-275 / compute_checksum.rs:15-20): the oracle's PCLMUL CRC on the host
    # over the store streamed D2H in ~2 GiB groups of whole entries (crc_stored
    # was written by the device's synth_kernel, which shares the scan's CRC
    # machinery, so crc == st alone could hide a bug common to both)
    ps = (mo - ln).astype(np.uint64)
    host = torch.empty(2 << 30 | 1 << 21, dtype=torch.uint8, pin_memory=True)
    hn = host.numpy()
    i0 = checked = 0
    while i0 < n:
        g0 = int(ps[i0])
        i1 = int(np.searchsorted(mo, np.uint64(g0 + (2 << 30)), side="right"))
        i1 = max(i1, i0 + 1)
        g1 = int(mo[i1 - 1])
        host[: g1 - g0].copy_(t[g0:g1])
        got = O.crc32_ranges(hn[: g1 - g0], ps[i0:i1] - np.uint64(g0), ln[i0:i1], threads=16)
        bad = np.nonzero(got != crc[i0:i1])[0]
        assert bad.size == 0, ("crc_computed differs from the host CRC", int(i0 + bad[0]), bad.size)
        checked += i1 - i0
        i0 = i1
    assert checked == n
    del host, hn
    # one flipped byte in a 1 MiB entry -> exactly that entry's CRC is bad
    big = int(np.nonzero(ln > (1 << 19))[0][len(np.nonzero(ln > (1 << 19))[0]) // 2])
    pos = int(mo[big]) - 12345
    t[pos] ^= 0x08
    r = S.validate_index_device(t.data_ptr(), size, 0, ctx)
    assert (r.final_len, r.n_chain, r.n_crc_bad) == (size, n, 1)
    ok = S.device_to_numpy(r.crc_ok, n, np.uint8)
    assert np.nonzero(ok == 0)[0].tolist() == [big]
    t[pos] ^= 0x08
    del t
    torch.cuda.empty_cache()


def test_full_c5_write_equals_c2(ctx):
    """C5 at its BASELINE size: batch_write of 1M x 4 KiB from pinned host
    memory (chunked H2D on a side stream overlapped with the writer kernel)
    is byte-identical to the C2 store, and its (key_hash, offset) pairs are
    the C2 index."""
    import torch
    n, L = 1 << 20, 4096
    size = S.synth_store_len(n, L)
    store = torch.empty(S.padded_size(size), dtype=torch.uint8, device="cuda")
    S.synth_store_device(store.data_ptr(), n, L, ctx=ctx)
    pays = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    pays.copy_(store[: 4160 * n].view(n, 4160)[:, :L].reshape(-1))
    keys = [b"bench-key-%d" % i for i in range(n)]
    kl = np.array([len(k) for k in keys], np.uint64)
    ko = np.zeros(n, np.uint64)
    ko[1:] = np.cumsum(kl)[:-1]
    kpin = torch.empty(int(kl.sum()), dtype=torch.uint8, pin_memory=True)
    kpin.copy_(torch.frombuffer(bytearray(b"".join(keys)), dtype=torch.uint8))
    out = torch.zeros(size + 64, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    nt, kh, mo = S.batch_write_raw(out.data_ptr(), size + 64, 0, kpin.data_ptr(), ko, kl, pays.data_ptr(),
                                   np.arange(n, dtype=np.uint64) * L, np.full(n, L, np.uint64), 0, ctx)
    torch.cuda.synchronize()
    assert nt == size and torch.equal(out[:size], store[:size])
    r = S.validate_index_device(store.data_ptr(), size, 0, ctx)
    assert np.array_equal(S.device_to_numpy(r.index_key_hash, n), kh)
    assert np.array_equal(S.device_to_numpy(r.index_packed, n) & np.uint64((1 << 48) - 1), mo)
    # independently of the device: every key hash is python-xxhash's XXH3-64 of
    # the key (compute_hash, digest/compute_hash.rs), every offset the closed
    # form of the C2 layout (entry i's metadata at 4160 i + 4096), every tag
    # the hash's top 16 bits (key_indexer.rs:64-93)
    want = np.array([xxhash.xxh3_64_intdigest(k) for k in keys], np.uint64)
    assert np.array_equal(kh, want)
    assert np.array_equal(mo, np.arange(n, dtype=np.uint64) * np.uint64(4160) + np.uint64(4096))
    assert np.array_equal(S.device_to_numpy(r.index_packed, n) >> np.uint64(48), want >> np.uint64(48))


def test_overflow_after_large_call_one_context():
    """Regression test for the fault fixed in 46785b6: after a large call, a
    store whose candidate records overflow their regions (and, later, the
    dense candidate capacity capK the large call sized) made the shape
    kernels read parents link2 never wrote.  All on ONE context: the full C2
    store, the reference's storage_benchmark shape (1M x 8 B: ~256 records
    per 16 KiB span against 8 slots, so the regions overflow and grow), a
    5M x 8 B store (more candidates than C2's capK), then C2 again; each
    compared with the oracle (C2 by its closed form)."""
    import torch
    c = S.Context(0)
    try:
        n2 = 1 << 20
        size2 = S.synth_store_len(n2)
        t = torch.empty(S.padded_size(size2), dtype=torch.uint8, device="cuda")
        S.synth_store_device(t.data_ptr(), n2, 4096, ctx=c)
        torch.cuda.synchronize()

        def c2():
            r = S.validate_index_device(t.data_ptr(), size2, 0, c)
            assert (r.mode, r.final_len, r.n_chain, r.n_index, r.n_crc_bad) == (0, size2, n2, n2, 0)
            ln = S.device_to_numpy(r.payload_len, n2, np.uint64)
            assert np.all(ln == 4096)

        c2()
        for store in (_storage_benchmark_store(), None):
            if store is None:  # 5M x 8 B, generated on the device: 320 MB, ~5M candidates > C2's capK (4.26M)
                n = 5_000_000
                size = S.synth_store_len(n, 8)
                d = torch.zeros(S.padded_size(size), dtype=torch.uint8, device="cuda")
                S.synth_store_device(d.data_ptr(), n, 8, ctx=c)
                torch.cuda.synchronize()
                store = d[:size].cpu().numpy()
                del d
            r = S.validate_index(store, 0, c)
            ch = O.chain_arrays(store, store.size)
            assert (r.final_len, r.n_chain, r.n_crc_bad) == (store.size, len(ch), 0)
            for k in ("meta_off", "key_hash", "prev_offset", "payload_start", "payload_len", "crc_stored",
                      "crc_computed", "crc_ok"):
                assert np.array_equal(getattr(r, k).astype(np.uint64), ch[k].astype(np.uint64)), k
            keys, packed = O.key_indexer_arrays(store, store.size)
            o = np.argsort(r.index_key_hash, kind="stable")
            assert np.array_equal(r.index_key_hash[o], keys) and np.array_equal(r.index_packed[o], packed)
        c2()
        del t
        torch.cuda.empty_cache()
    finally:
        c.close()


@pytest.mark.parametrize("flags", [0, S.SRD_FLAG_FORCE_FULL])
def test_link_record_parents_across_empty_waves(ctx, flags):
    """link_record's parent lookup (link2_kernel, after the scan) across empty
    waves and distant spans: entries of 24 and 40 MiB between runs of small
    ones put hundreds of record-less scan waves between a node and its parent
    (the previous wave's region empty, the parent's span in a wave blocks
    away: the span_first / part_span_wave lookup), and a key is overwritten
    across them; every output equals the oracle's in both passes."""
    rng = np.random.default_rng(0x5EED0009)
    big = {300: 24 << 20, 700: 40 << 20, 701: 5 << 20}
    entries = []
    for i in range(1200):
        ln = big.get(i, int(rng.integers(1, 3000)))
        key = b"k-%d" % (i if i != 1100 else 7)  # entry 1100 overwrites key k-7
        entries.append((xxhash.xxh3_64_intdigest(key), rng.integers(0, 256, ln, dtype=np.uint8).tobytes()))
    buf = bytearray()
    t = O.write_entries(buf, 0, entries)
    store = np.frombuffer(bytes(buf[:t]), np.uint8)
    r = S.validate_index(store, flags, ctx)
    ch = O.chain_arrays(store, store.size)
    assert (r.final_len, r.n_chain, r.n_crc_bad) == (store.size, len(ch), 0)
    for k in ("meta_off", "key_hash", "prev_offset", "payload_start", "payload_len", "crc_stored", "crc_computed",
              "crc_ok"):
        assert np.array_equal(getattr(r, k).astype(np.uint64), ch[k].astype(np.uint64)), k
    keys, packed = O.key_indexer_arrays(store, store.size)
    assert len(keys) == 1199
    o = np.argsort(r.index_key_hash, kind="stable")
    assert np.array_equal(r.index_key_hash[o], keys) and np.array_equal(r.index_packed[o], packed)
