#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/.

An independent pure-Python restatement of the reference's on-disk writer and
open-time path, with the arithmetic taken from zlib (IEEE CRC-32, the
algorithm crc32fast 1.5.0 implements) and python-xxhash 3.8.1 (libxxhash,
the algorithm xxhash-rust 0.8.15's xxh3_64 implements).  Small cases only.

  writer            data_store.rs:847-939 (batch_write_with_key_hashes)
  recover           data_store.rs:383-482 (recover_valid_chain)
  KeyIndexer::build key_indexer.rs:98-124
  is_valid_checksum entry_handle.rs:260-275

The scenarios mirror the reference's own tests (persistence_tests.rs torn
tail b"CORRUPT", integrity_tests.rs byte flip, alignment_tests.rs payload
sizes, storage_operation_tests.rs nested store, parallel_iterator_tests.rs
tombstones/overwrites, storage_benchmark.rs 8-byte LE payloads) plus edge
cases (empty file, <20-byte file, torn tails at every byte of an entry,
zero-rich payloads that create many chain candidates).

Run:  python tests/golden/make_golden.py   (rewrites cases.json + *.bin)
"""
from __future__ import annotations

import json
import os
import random
import struct
import zlib

import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
MS = 20
M64 = (1 << 64) - 1


def h(key: bytes) -> int:
    return xxhash.xxh3_64_intdigest(key)


def prepad(off: int) -> int:  # data_store.rs:670-673
    return (64 - off % 64) & 63


class Store:
    """Append-only single file, as DataStore's writer lays it out."""

    def __init__(self):
        self.buf = bytearray()

    @property
    def tail(self):
        return len(self.buf)

    def batch(self, entries, allow_null=False):
        for kh, payload in entries:
            if payload == b"\x00":
                assert allow_null
                crc = zlib.crc32(payload)
                self.buf += b"\x00" + struct.pack("<QQI", kh, self.tail, crc)
                continue
            assert len(payload) > 0
            link = self.tail
            self.buf += b"\x00" * prepad(link)
            self.buf += payload + struct.pack("<QQI", kh, link, zlib.crc32(payload))

    def write(self, key: bytes, payload: bytes):
        self.batch([(h(key), payload)])

    def delete(self, key: bytes):
        self.batch([(h(key), b"\x00")], allow_null=True)


def rd64(b, o):
    return struct.unpack_from("<Q", b, o)[0]


def recover(mm: bytes, file_len: int) -> int:
    """data_store.rs:383-482, literal, with wrapping u64 adds."""
    if file_len < MS:
        return 0
    cursor = file_len
    while cursor >= MS:
        mo = cursor - MS
        prev_tail = rd64(mm, mo + 8)
        derived = (prev_tail + prepad(prev_tail)) & M64
        if mo > prev_tail and mo - prev_tail == 1 and mm[prev_tail] == 0:
            start = prev_tail
        else:
            start = derived
        if start >= mo:
            cursor -= 1
            continue
        valid = True
        back = prev_tail
        total = (mo - start) + MS
        while back != 0:
            if back < MS:
                valid = False
                break
            pmo = back - MS
            if pmo + MS > len(mm):
                valid = False
                break
            ppt = rd64(mm, pmo + 8)
            if pmo > ppt and pmo - ppt == 1 and mm[ppt] == 0:
                pes = ppt
            else:
                pes = (ppt + prepad(ppt)) & M64
            if pes >= pmo:
                valid = False
                break
            total += max(pmo - pes, 0) + MS
            if ppt >= pmo:
                valid = False
                break
            back = ppt
        if valid and back == 0 and total <= file_len:
            return mo + MS
        cursor -= 1
    return 0


def chain(mm: bytes, tail: int):
    out = []
    cur = tail
    while cur >= MS:
        mo = cur - MS
        kh, p, crc = struct.unpack_from("<QQI", mm, mo)
        if mo > p and mo - p == 1 and mm[p] == 0:
            start, tomb = p, True
        else:
            start, tomb = p + prepad(p), False
        comp = zlib.crc32(bytes(mm[start:mo]))
        out.append(dict(meta_off=mo, key_hash=kh, prev_offset=p, payload_start=start,
                        payload_len=mo - start, crc_stored=crc, crc_computed=comp,
                        crc_ok=int(comp == crc), is_tombstone=int(tomb)))
        if p == 0:
            break
        cur = p
    return out[::-1]


def build_index(mm: bytes, tail: int):
    """key_indexer.rs:98-124 (tombstones included, latest wins)."""
    index, seen = {}, set()
    cur = tail
    while cur >= MS:
        mo = cur - MS
        kh, p = struct.unpack_from("<QQ", mm, mo)
        if kh in seen:
            cur = p
            continue
        seen.add(kh)
        index[kh] = ((kh >> 48) << 48) | mo
        if p == 0:
            break
        cur = p
    return index


# ---------------------------------------------------------------- cases
def cases():
    rnd = random.Random(0x5EED)
    out = {}

    out["empty"] = b""
    out["short_7"] = b"CORRUPT"
    out["short_19"] = bytes(19)

    s = Store()
    for k in [b"alice", b"bob", b"carol", b"key1", b"test_key", b"longer_key_name"]:
        s.write(k, b"value-of-" + k)
    out["basic"] = bytes(s.buf)

    # persistence_tests.rs:126-173 torn tail: append b"CORRUPT"
    out["torn_corrupt"] = bytes(s.buf) + b"CORRUPT"

    # integrity_tests.rs:40-78: flip the first payload byte of one entry
    s2 = Store()
    s2.write(b"checksum_test", b"Testing checksum validation")
    s2.write(b"other", b"Other payload bytes")
    b2 = bytearray(s2.buf)
    b2[0] ^= 0xFF
    out["integrity_flip"] = bytes(b2)

    # overwrites + deletes (parallel_iterator_tests.rs, compaction_tests.rs)
    s3 = Store()
    for i in range(12):
        s3.write(b"k%d" % (i % 5), b"v%d-" % i * (i + 1))
    s3.delete(b"k1")
    s3.delete(b"k3")
    s3.write(b"k3", b"resurrected")
    s3.delete(b"k4")
    out["overwrite_delete"] = bytes(s3.buf)

    # alignment_tests.rs:136-245 payload sizes with delete + overwrite
    s4 = Store()
    for i, n in enumerate([3, 5, 7, 9, 20, 72, 64, 128]):
        s4.write(b"a%d" % i, bytes(rnd.getrandbits(8) for _ in range(n)))
    s4.delete(b"a2")
    s4.write(b"a5", b"x" * 63)
    s4.write(b"a0", b"y")
    out["alignment"] = bytes(s4.buf)

    # tombstone-heavy: consecutive deletes (no prepad between them)
    s5 = Store()
    for i in range(6):
        s5.write(b"t%d" % i, b"payload-%d" % i)
    for i in range(6):
        s5.delete(b"t%d" % i)
    s5.write(b"t0", b"back")
    out["tombstones"] = bytes(s5.buf)

    # storage_operation_tests.rs:321-380 nested store as a payload
    out["nested"] = None  # filled below
    inner = bytes(s.buf)
    s6 = Store()
    s6.write(b"outer1", b"hello")
    s6.write(b"nested", inner)
    s6.write(b"outer2", b"world")
    out["nested"] = bytes(s6.buf)

    # storage_benchmark.rs:20-26 shape: 8-byte LE payloads (zero rich)
    s7 = Store()
    for i in range(300):
        s7.write(b"bench-key-%d" % i, struct.pack("<Q", i))
    out["bench_8b"] = bytes(s7.buf)

    # 1-byte payloads
    s8 = Store()
    for i in range(40):
        s8.write(b"one-%d" % i, bytes([1 + i % 250]))
    out["one_byte"] = bytes(s8.buf)

    # payloads that embed fake metadata records / small integers
    s9 = Store()
    for i in range(20):
        pl = bytearray(struct.pack("<QQI", h(b"fake%d" % i), rnd.randrange(0, 5000), 0))
        pl += struct.pack("<QQQ", i, 64 * i, 21) + bytes(rnd.randrange(0, 3) for _ in range(40))
        s9.write(b"fk%d" % i, bytes(pl))
    out["fake_meta"] = bytes(s9.buf)

    # 4 KiB synthetic entries with torn writes at several cut points
    s10 = Store()
    for i in range(6):
        s10.write(b"bench-key-%d" % i, bytes(rnd.getrandbits(8) for _ in range(4096)))
    full = bytes(s10.buf)
    out["c1_shape_6x4k"] = full
    last_start = len(full) - 4096 - 20
    for cut in [len(full) - 1, len(full) - 10, len(full) - 21, last_start + 2048,
                last_start + 1, last_start - 10, last_start - 30]:
        out["torn_cut_%d" % cut] = full[:cut]

    # random garbage
    out["garbage_1k"] = bytes(rnd.getrandbits(8) for _ in range(1024))
    out["zeros_300"] = bytes(300)
    return out


def main():
    meta = {}
    for name, data in cases().items():
        fname = name + ".bin"
        with open(os.path.join(HERE, fname), "wb") as f:
            f.write(data)
        fl = recover(data, len(data))
        ch = chain(data, fl)
        idx = build_index(data, fl)
        meta[name] = dict(
            file=fname, file_len=len(data), final_len=fl,
            chain=[{k: (hex(v) if k in ("key_hash",) else v) for k, v in e.items()} for e in ch],
            index={hex(k): hex(v) for k, v in sorted(idx.items())},
            index_hash_le8={hex(k): hex(xxhash.xxh3_64_intdigest(struct.pack("<Q", k))) for k in sorted(idx)},
        )
    with open(os.path.join(HERE, "cases.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", len(meta), "cases")


if __name__ == "__main__":
    main()
