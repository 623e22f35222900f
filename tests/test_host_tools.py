"""CPU checks of the host side of the boundary (no GPU calls):
  - the ASan/UBSan build of the host parsers of untrusted store bytes
    (srd_host.cpp: srd_shard_cuts, srd_batch_layout) and of the oracle, over
    the golden fixtures (garbage included), their mutations and random bytes;
  - the compiled C caller of include/srd_amd.h builds and its struct layout
    equals the ctypes mirror and the #[repr(C)] Rust struct of INTEGRATION.md;
  - the single-process multi-GPU open's composition + latest-wins index merge
    (srd_validate_index_multi), restated with the oracle per shard: the
    concatenated shard chains and the shard-ordered merge give the whole-file
    result for every cut srd_shard_cuts makes."""
import ctypes as C
import glob
import json
import os
import subprocess

import numpy as np
import pytest

import oracle as O
import srd_amd as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sanitizer_harness():
    d = os.path.join(ROOT, "tests", "sanitize")
    subprocess.check_call(["make", "-s", "-C", d])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    fx = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "*.bin")))
    assert any("garbage" in f for f in fx)
    p = subprocess.run([os.path.join(d, "build", "host_fuzz")] + fx, capture_output=True, text=True, env=env,
                       timeout=600)
    assert p.returncode == 0 and "host_fuzz ok" in p.stdout, p.stderr[-3000:]


def _abi_check_bin():
    d = os.path.join(ROOT, "tests", "abi_c")
    if not os.path.exists(S.LIB_PATH):
        S.build()
    subprocess.check_call(["make", "-s", "-C", d])
    return os.path.join(d, "build", "srd_abi_check")


def test_c_abi_layout_matches_bindings():
    out = json.loads(subprocess.check_output([_abi_check_bin(), "--layout"], text=True))
    for name, _ in S.DeviceResult._fields_:
        assert out[f"srd_result.{name}"] == getattr(S.DeviceResult, name).offset, name
    for name, _ in S.WriteEntry._fields_:
        assert out[f"srd_write_entry.{name}"] == getattr(S.WriteEntry, name).offset, name
    for name, _ in S.MultiSummary._fields_:
        assert out[f"srd_multi_summary.{name}"] == getattr(S.MultiSummary, name).offset, name
    assert out["sizeof(srd_multi_summary)"] == C.sizeof(S.MultiSummary) == 112
    assert "pub mode: u32, pub path: u32, pub n_shards: u32, pub merged: u32," in open(
        os.path.join(ROOT, "INTEGRATION.md")).read()
    assert out["sizeof(srd_result)"] == C.sizeof(S.DeviceResult) == 144
    assert out["sizeof(srd_write_entry)"] == C.sizeof(S.WriteEntry) == 40
    # the Rust #[repr(C)] SrdResult of INTEGRATION.md: 7 u64, 2 u32, 10 pointers
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "pub mode: u32, pub reserved: u32," in text
    assert out["srd_result.mode"] == 7 * 8 and out["srd_result.meta_off"] == 7 * 8 + 8


def _chain_seg(store, lo, hi):
    """Entries of the whole file's chain with lo < meta_off + 20 <= hi, file order."""
    return [e for e in O.chain(store, O.recover_valid_chain(store)) if lo < e["meta_off"] + 20 <= hi]


def _stores():
    import random
    import xxhash
    rnd = random.Random(17)
    buf, t = bytearray(), 0
    for _ in range(500):
        kh = xxhash.xxh3_64_intdigest(b"k%d" % rnd.randrange(80))
        if rnd.random() < 0.1:
            t = O.write_entries(buf, t, [(kh, b"\x00")], allow_null=True)
        else:
            pl = rnd.randbytes(rnd.choice([1, 9, 64, 500, 4096, 9000]))
            t = O.write_entries(buf, t, [(kh, b"\x01" if pl == b"\x00" else pl)])
    lens = np.minimum(S.zipf_lens(400, seed=4), 1 << 16)
    return {"overwrites": np.frombuffer(bytes(buf), np.uint8), "zipf": O.synth_store(400, lens=lens),
            "c1": O.synth_store(300)}


@pytest.mark.parametrize("world", [2, 3, 5, 8])
def test_multi_composition_and_merge_restated(world):
    for name, store in _stores().items():
        cuts = S.shard_cuts(store, world)
        assert cuts[0] == 0 and cuts[-1] == store.size
        whole = O.chain(store, store.size)
        segs = [_chain_seg(store, cuts[r], cuts[r + 1]) for r in range(world)]
        # composition: every shard's segment is its chain from hi down to prev == lo
        for r in range(world):
            if cuts[r] == cuts[r + 1]:
                assert not segs[r]
                continue
            assert segs[r][-1]["meta_off"] + 20 == cuts[r + 1], (name, r)
            assert segs[r][0]["prev_offset"] == cuts[r], (name, r)
        assert [e["meta_off"] for s in segs for e in s] == [e["meta_off"] for e in whole]
        # merge: shard-local latest-wins indexes, then latest-wins over the
        # concatenation in shard order (what ctxs[0] builds on the device)
        merged = {}
        for s in segs:
            local = {}
            for e in s:
                local[e["key_hash"]] = ((e["key_hash"] >> 48) << 48) | e["meta_off"]
            for k, v in local.items():
                merged[k] = v
        want = O.key_indexer_build(store, store.size)
        assert merged == want, name
        order = sorted(v & ((1 << 48) - 1) for v in merged.values())
        assert order == sorted(v & ((1 << 48) - 1) for v in want.values())


def test_bench_scan_sample_and_traffic_tag():
    """bench.py stamps one in ten timed steps (>= 10 stamped scan launches per
    run), and profiles/traffic.json carries the hash of
    the kernel sources it was measured on: the line reports `traffic` only
    for those sources (the committed file matches the committed sources)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    for steps in (10, 20, 50, 100, 1000):
        k = bench.scan_sample(steps)
        assert k >= 1 and len(range(0, steps, k)) >= 10
    assert bench.scan_sample(3) == 1
    t = json.load(open(os.path.join(root, "profiles", "traffic.json")))
    assert t["kernel_sources_sha256"] == bench.kernel_sources_hash()
    assert t["scan_kernel_hbm_bytes_per_launch"] > 4_000_000_000
