"""ctypes binding of the CPU oracle (oracle/srd_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libsrd_oracle.so")

_u64p = C.POINTER(C.c_uint64)


class Entry(C.Structure):
    _fields_ = [
        ("meta_off", C.c_uint64),
        ("key_hash", C.c_uint64),
        ("prev_offset", C.c_uint64),
        ("payload_start", C.c_uint64),
        ("payload_len", C.c_uint64),
        ("crc_stored", C.c_uint32),
        ("crc_computed", C.c_uint32),
        ("crc_ok", C.c_uint32),
        ("is_tombstone", C.c_uint32),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("final_len", C.c_uint64),
        ("n_chain", C.c_uint64),
        ("n_index", C.c_uint64),
        ("n_crc_bad", C.c_uint64),
        ("crc_xor", C.c_uint64),
        ("index_xor", C.c_uint64),
        ("t_recover_s", C.c_double),
        ("t_index_s", C.c_double),
        ("t_crc_s", C.c_double),
    ]


def build() -> str:
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(
        os.path.join(HERE, "srd_oracle.c")
    ):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        L.orc_xxh3_64.restype = C.c_uint64
        L.orc_xxh3_64.argtypes = [C.c_void_p, C.c_size_t]
        L.orc_crc32.restype = C.c_uint32
        L.orc_crc32.argtypes = [C.c_void_p, C.c_size_t]
        L.orc_crc32_ranges.restype = None
        L.orc_crc32_ranges.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_int]
        L.orc_crc32_table.restype = C.c_uint32
        L.orc_crc32_table.argtypes = [C.c_void_p, C.c_size_t]
        L.orc_recover_valid_chain.restype = C.c_uint64
        L.orc_recover_valid_chain.argtypes = [C.c_void_p, C.c_uint64]
        L.orc_chain.restype = C.c_uint64
        L.orc_chain.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(Entry), C.c_uint64, C.c_int]
        L.orc_key_indexer_build.restype = C.c_uint64
        L.orc_key_indexer_build.argtypes = [C.c_void_p, C.c_uint64, _u64p, _u64p, C.c_uint64]
        L.orc_validate_index.restype = C.c_int
        L.orc_validate_index.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.POINTER(Stats)]
        L.orc_synth_store.restype = C.c_uint64
        L.orc_synth_store.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_uint64]
        L.orc_write_entries.restype = C.c_int64
        L.orc_write_entries.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int]
        L.orc_has_pclmul.restype = C.c_int
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if isinstance(a, np.ndarray) else C.c_char_p(bytes(a))


def xxh3_64(data: bytes) -> int:
    return lib().orc_xxh3_64(C.c_char_p(bytes(data)), len(data))


def crc32(data) -> int:
    buf = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return lib().orc_crc32(buf.ctypes.data_as(C.c_void_p), buf.size)


def crc32_ranges(buf: np.ndarray, starts, lens, threads: int = 16) -> np.ndarray:
    """compute_checksum of buf[starts[i] : starts[i] + lens[i]] for every i
    (PCLMUL crc32, threaded): uint32 array."""
    buf = np.ascontiguousarray(buf, np.uint8)
    starts = np.ascontiguousarray(starts, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint64)
    assert starts.size == lens.size and (starts.size == 0 or int((starts + lens).max()) <= buf.size)
    out = np.zeros(starts.size, np.uint32)
    if starts.size:
        lib().orc_crc32_ranges(buf.ctypes.data_as(C.c_void_p), starts.ctypes.data_as(C.c_void_p),
                               lens.ctypes.data_as(C.c_void_p), starts.size, out.ctypes.data_as(C.c_void_p), threads)
    return out


def as_u8(file) -> np.ndarray:
    if isinstance(file, np.ndarray):
        return np.ascontiguousarray(file, dtype=np.uint8)
    return np.frombuffer(bytes(file), dtype=np.uint8)


def recover_valid_chain(file) -> int:
    """data_store.rs:383-482"""
    a = as_u8(file)
    return lib().orc_recover_valid_chain(a.ctypes.data_as(C.c_void_p), a.size)


def chain(file, tail: int, compute_crc: bool = True) -> list[dict]:
    a = as_u8(file)
    n = lib().orc_chain(a.ctypes.data_as(C.c_void_p), tail, None, 0, 0)
    out = (Entry * max(n, 1))()
    lib().orc_chain(a.ctypes.data_as(C.c_void_p), tail, out, n, int(compute_crc))
    return [{f: getattr(out[i], f) for f, _ in Entry._fields_} for i in range(n)]


def chain_arrays(file, tail: int, compute_crc: bool = True) -> np.ndarray:
    """The chain as a numpy structured array (Entry fields), for large stores."""
    a = as_u8(file)
    n = lib().orc_chain(a.ctypes.data_as(C.c_void_p), tail, None, 0, 0)
    out = (Entry * max(n, 1))()
    lib().orc_chain(a.ctypes.data_as(C.c_void_p), tail, out, n, int(compute_crc))
    dt = np.dtype([(f, np.uint64 if t is C.c_uint64 else np.uint32) for f, t in Entry._fields_])
    return np.frombuffer(bytes(out), dt)[:n].copy()


def key_indexer_arrays(file, tail: int) -> tuple[np.ndarray, np.ndarray]:
    """KeyIndexer::build as (keys, packed) arrays, sorted by key_hash."""
    a = as_u8(file)
    cap = max(1, lib().orc_chain(a.ctypes.data_as(C.c_void_p), tail, None, 0, 0))
    k = np.zeros(cap, np.uint64)
    v = np.zeros(cap, np.uint64)
    n = lib().orc_key_indexer_build(a.ctypes.data_as(C.c_void_p), tail,
                                    k.ctypes.data_as(_u64p), v.ctypes.data_as(_u64p), cap)
    return k[:n], v[:n]


def key_indexer_build(file, tail: int) -> dict[int, int]:
    """key_indexer.rs:98-124 -> {key_hash: packed}"""
    a = as_u8(file)
    cap = max(1, len(chain(file, tail, False)))
    k = np.zeros(cap, np.uint64)
    v = np.zeros(cap, np.uint64)
    n = lib().orc_key_indexer_build(a.ctypes.data_as(C.c_void_p), tail,
                                    k.ctypes.data_as(_u64p), v.ctypes.data_as(_u64p), cap)
    return {int(k[i]): int(v[i]) for i in range(n)}


def validate_index(file, threads: int = 1) -> Stats:
    a = as_u8(file)
    st = Stats()
    lib().orc_validate_index(a.ctypes.data_as(C.c_void_p), a.size, threads, C.byref(st))
    return st


def synth_store(n_entries: int, payload_len: int = 4096, lens=None, seed: int = 0x5EED0001):
    L = lib()
    lp = None
    if lens is not None:
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        lp = lens.ctypes.data_as(C.c_void_p)
    size = L.orc_synth_store(None, n_entries, payload_len, lp, seed)
    out = np.zeros(size, np.uint8)
    L.orc_synth_store(out.ctypes.data_as(C.c_void_p), n_entries, payload_len, lp, seed)
    return out


def write_entries(buf: bytearray, tail: int, entries, allow_null: bool = False) -> int:
    """batch_write_with_key_hashes (data_store.rs:847-939) into a bytearray.
    entries: list of (key_hash, payload bytes).  Returns the new tail."""
    n = len(entries)
    pay = b"".join(p for _, p in entries)
    offs = np.zeros(n, np.uint64)
    lens = np.array([len(p) for _, p in entries], np.uint64)
    if n:
        offs[1:] = np.cumsum(lens)[:-1]
    kh = np.array([k for k, _ in entries], np.uint64)
    need = tail + sum(len(p) + 84 for _, p in entries)
    out = np.zeros(need, np.uint8)
    out[:tail] = np.frombuffer(bytes(buf[:tail]), np.uint8)
    pb = np.frombuffer(pay, np.uint8) if pay else np.zeros(1, np.uint8)
    r = lib().orc_write_entries(out.ctypes.data_as(C.c_void_p), need, tail, kh.ctypes.data_as(C.c_void_p),
                                pb.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p),
                                lens.ctypes.data_as(C.c_void_p), n, int(allow_null))
    if r < 0:
        raise ValueError("invalid payload (empty or NULL byte)" if r == -1 else "capacity")
    del buf[tail:]
    buf[tail:] = out[tail:r].tobytes()
    return int(r)
