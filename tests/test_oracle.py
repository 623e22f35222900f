"""Pin the CPU oracle (oracle/srd_oracle.c) before trusting it:
the reference's own golden vectors, the IEEE check value, zlib/python-xxhash
over random inputs, and the fixtures written by tests/golden/make_golden.py."""
import random
import struct
import zlib

import numpy as np
import pytest
import xxhash

import oracle as O


def test_xxh3_reference_goldens(ref_goldens):
    # tests/hash_stability_tests.rs:16-57
    for hexkey, want in ref_goldens["xxh3_64"].items():
        assert O.xxh3_64(bytes.fromhex(hexkey)) == int(want, 16)


def test_namespace_hasher_goldens(ref_goldens):
    # tests/hash_stability_tests.rs:76-100 ; src/utils/namespace_hasher.rs:33-65
    for g in ref_goldens["namespace"]:
        out = struct.pack("<QQ", O.xxh3_64(g["prefix"].encode()), O.xxh3_64(g["key"].encode()))
        assert out.hex() == g["out"]


def test_crc_check_values(ref_goldens):
    for hexdata, want in ref_goldens["crc32"].items():
        assert O.crc32(bytes.fromhex(hexdata)) == int(want, 16)


@pytest.mark.parametrize("seed", [1, 2])
def test_xxh3_and_crc_random(seed):
    rnd = random.Random(seed)
    lens = list(range(0, 300)) + [rnd.randrange(300, 5000) for _ in range(40)] + [1024, 1025, 4096, 65536 + 3]
    for n in lens:
        d = rnd.randbytes(n)
        assert O.xxh3_64(d) == xxhash.xxh3_64_intdigest(d), n
        assert O.crc32(d) == zlib.crc32(d), n


def test_fixtures(golden_cases):
    for name, (data, m) in golden_cases.items():
        assert O.recover_valid_chain(data) == m["final_len"], name
        ch = O.chain(data, m["final_len"])
        assert len(ch) == len(m["chain"]), name
        for a, b in zip(ch, m["chain"]):
            for k, v in b.items():
                v = int(v, 16) if isinstance(v, str) else v
                assert a[k] == v, (name, k)
        idx = O.key_indexer_build(data, m["final_len"])
        assert idx == {int(k, 16): int(v, 16) for k, v in m["index"].items()}, name
        st = O.validate_index(data, 1)
        assert st.final_len == m["final_len"] and st.n_chain == len(m["chain"])
        assert st.n_index == len(m["index"])
        assert st.n_crc_bad == sum(1 - e["crc_ok"] for e in m["chain"])


def test_synth_store_shape():
    # C1 = 1000 x 4096 B -> 4,159,956 bytes
    s = O.synth_store(1000)
    assert s.size == 4_159_956
    assert O.recover_valid_chain(s) == s.size
    ch = O.chain(s, s.size)
    assert len(ch) == 1000 and all(e["crc_ok"] for e in ch)
    assert ch[1]["payload_start"] == 4160 and ch[1]["meta_off"] == 8256
    assert ch[5]["key_hash"] == xxhash.xxh3_64_intdigest(b"bench-key-5")
    for t in (1, 3):
        st = O.validate_index(s, t)
        assert (st.final_len, st.n_chain, st.n_index, st.n_crc_bad) == (s.size, 1000, 1000, 0)


def test_writer_matches_fixture(golden_cases):
    # the C writer reproduces the Python writer's bytes (basic case)
    data, _ = golden_cases["basic"]
    buf = bytearray()
    t = 0
    for k in [b"alice", b"bob", b"carol", b"key1", b"test_key", b"longer_key_name"]:
        t = O.write_entries(buf, t, [(xxhash.xxh3_64_intdigest(k), b"value-of-" + k)])
    assert bytes(buf) == data
    with pytest.raises(ValueError):
        O.write_entries(buf, t, [(1, b"\x00")])
    with pytest.raises(ValueError):
        O.write_entries(buf, t, [(1, b"")])
