"""Python binding of the MI355X-native validate+index path (include/srd_amd.h).

Mirrors the reference's interface for this path (jzombie/rust-simd-r-drive):

  recover_valid_chain(file)      data_store.rs:383-482  -> final_len
  KeyIndexer.build(file, tail)   key_indexer.rs:98-124   -> {key_hash: packed}
  KeyIndexer.tag_from_hash/pack/unpack                   key_indexer.rs:64-93
  compute_checksum(data)         compute_checksum.rs:15-20 -> 4 LE bytes
  compute_hash(key)              compute_hash.rs:25-27
  compute_hash_batch(keys)       compute_hash.rs:64-77
  DataStore.open(path)           data_store.rs:84-117 (mmap -> recover ->
                                 truncate + re-open -> index), with every chain
                                 payload's CRC verified on the GPU
  EntryHandle.is_valid_checksum  entry_handle.rs:260-275

All compute runs in libsrd_amd.so (HIP, gfx950).  There is no CPU fallback:
if the library or a GPU is missing, calls raise.
"""
from __future__ import annotations

import ctypes as C
import mmap as _mmap
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SRD_LIB_PATH") or os.path.join(HERE, "build", "libsrd_amd.so")  # override: timing tools only

SRD_FLAG_FORCE_FULL = 1
SRD_FLAG_NO_CRC = 2
SRD_FLAG_STAGE_PAGEABLE = 4  # host input: one pageable hipMemcpy (measurement baseline)
SRD_FLAG_STAGE_REGISTER = 8  # host input: hipHostRegister the range (default: pinned bounce buffers)
STAGE_MODES = {0: "pinned input", 1: "registered mapping", 2: "bounce buffers", 3: "pageable copy"}
TIMING_NONE, TIMING_SCAN, TIMING_CALL = 0, 1, 2  # srd_ctx_set_timing levels
SRD_MODE_OPTIMISTIC = 0
SRD_MODE_FULL = 1
SRD_MODE_SPAN_UNPROVEN = 3
# srd_device_result.full_reason (include/srd_amd.h)
SRD_FULL_NONE, SRD_FULL_FORCED, SRD_FULL_SLOT_SPACE, SRD_FULL_WAVES = 0, 1, 2, 3
SRD_FULL_NO_START, SRD_FULL_UNPROVEN, SRD_FULL_CAP, SRD_FULL_LOOKBACK = 4, 5, 6, 7
SRD_FLAG_MERGE_INDEX = 16  # multi-GPU open: the whole index on ctxs[0] (default: by owner)
SRD_MULTI_COMPOSED, SRD_MULTI_NEIGHBOUR, SRD_MULTI_WHOLE_FILE = 0, 1, 2  # srd_multi_summary.path
SPAN_ALIGN = 16384  # span_off granularity of srd_validate_span_device
METADATA_SIZE = 20
NULL_BYTE = b"\x00"
TAG_BITS = 16
OFFSET_MASK = (1 << 48) - 1

# symbols include/srd_amd.h declares
EXPORTS = [
    "srd_ctx_create", "srd_ctx_destroy", "srd_ctx_stream", "srd_ctx_device_bytes", "srd_ctx_scan_loads",
    "srd_ctx_scan_trial",
    "srd_last_error", "srd_build_info",
    "srd_ctx_timings",
    "srd_ctx_set_timing",
    "srd_validate_index_device", "srd_validate_index", "srd_result_free",
    "srd_recover_valid_chain", "srd_key_indexer_build", "srd_crc32_batch",
    "srd_crc32_batch_device", "srd_xxh3_64_batch", "srd_xxh3_64_batch_device",
    "srd_synth_store_device", "srd_selftest_host", "srd_padded_size",
    "srd_validate_span_device", "srd_index_partition_device", "srd_index_build_device",
    "srd_synth_span_device", "srd_batch_layout", "srd_batch_write", "srd_batch_write_device",
    "srd_index_table_bytes", "srd_index_table_build_device", "srd_index_get_packed_device",
    "srd_batch_read_hashed_device", "srd_batch_read",
    "srd_iter_entries_device", "srd_estimate_compaction_savings_device", "srd_compact_device",
    "srd_shard_cuts", "srd_validate_index_multi", "srd_ctx_stage_info", "srd_index_hash_device",
    "srd_validate_index_multi_device", "srd_ctx_multi_summary", "srd_ctx_scan_list", "srd_ctx_set_timing_every",
    "srd_stream_probe_device", "srd_ctx_multi_shard_ms",
]


class DeviceResult(C.Structure):
    _fields_ = [
        ("file_len", C.c_uint64), ("final_len", C.c_uint64), ("n_chain", C.c_uint64),
        ("n_index", C.c_uint64), ("n_crc_bad", C.c_uint64), ("n_candidates", C.c_uint64),
        ("full_reason", C.c_uint64), ("mode", C.c_uint32), ("reserved", C.c_uint32),
        ("meta_off", C.c_void_p), ("key_hash", C.c_void_p), ("prev_offset", C.c_void_p),
        ("payload_start", C.c_void_p), ("payload_len", C.c_void_p),
        ("crc_stored", C.c_void_p), ("crc_computed", C.c_void_p), ("crc_ok", C.c_void_p),
        ("index_key_hash", C.c_void_p), ("index_packed", C.c_void_p),
    ]


class MultiSummary(C.Structure):
    """srd_multi_summary (include/srd_amd.h)"""
    _fields_ = [
        ("file_len", C.c_uint64), ("final_len", C.c_uint64), ("n_chain", C.c_uint64),
        ("n_index", C.c_uint64), ("n_crc_bad", C.c_uint64), ("n_candidates", C.c_uint64),
        ("mode", C.c_uint32), ("path", C.c_uint32), ("n_shards", C.c_uint32), ("merged", C.c_uint32),
        ("shard_errors", C.c_uint32), ("peer_errors", C.c_uint32),
        ("validate_ms", C.c_double), ("exchange_ms", C.c_double), ("total_ms", C.c_double),
        ("index_key_hash", C.c_void_p), ("index_packed", C.c_void_p),
    ]


def build_info() -> str:
    """srd_build_info(): the sha256 of the sources the loaded library was
    compiled from (equal to src_hash.source_hash(), or lib() refused it)."""
    return lib().srd_build_info().decode()


def build() -> str:
    """Compile the HIP library in-tree (hipcc --offload-arch=gfx950)."""
    subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C {HERE}` (no CPU fallback exists)")
        # One HIP runtime per process: if PyTorch is present, load it first so
        # that libsrd_amd.so binds to the libamdhip64.so.7 torch already mapped
        # (torch NEEDs "libamdhip64.so", we NEED the soname "libamdhip64.so.7";
        # loading us first would map a second runtime from /opt/rocm).
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        L = C.CDLL(LIB_PATH)
        vp, u64, u32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
        L.srd_build_info.restype = C.c_char_p
        L.srd_ctx_device_bytes.argtypes = [vp]
        L.srd_ctx_device_bytes.restype = u64
        L.srd_ctx_scan_loads.argtypes = [vp]
        L.srd_ctx_scan_trial.argtypes = [vp, C.POINTER(C.c_double)]
        if not os.environ.get("SRD_LIB_PATH"):  # (timing tools load variant builds by path)
            import importlib.util
            spec = importlib.util.spec_from_file_location("srd_src_hash", os.path.join(HERE, "src_hash.py"))
            sh = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(sh)
            want, got = sh.source_hash(), L.srd_build_info().decode()
            if got != want:
                raise RuntimeError(f"{LIB_PATH} was built from other sources (sha256 {got}, the sources here "
                                   f"{want}): run `make -C {HERE}`")
        L.srd_ctx_create.argtypes = [i32, C.POINTER(vp)]
        L.srd_ctx_destroy.argtypes = [vp]
        L.srd_ctx_stream.argtypes = [vp]
        L.srd_ctx_stream.restype = vp
        L.srd_last_error.restype = C.c_char_p
        L.srd_ctx_timings.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_double)]
        L.srd_ctx_set_timing.argtypes = [vp, C.c_int]
        L.srd_ctx_scan_list.argtypes = [vp, C.POINTER(C.c_float), C.c_int]
        L.srd_ctx_set_timing_every.argtypes = [vp, C.c_int]
        L.srd_validate_index_device.argtypes = [vp, vp, u64, u32, C.POINTER(DeviceResult)]
        L.srd_validate_index.argtypes = [vp, vp, u64, u32, C.POINTER(DeviceResult)]
        L.srd_result_free.argtypes = [C.POINTER(DeviceResult)]
        L.srd_recover_valid_chain.argtypes = [vp, vp, u64, C.POINTER(u64)]
        L.srd_key_indexer_build.argtypes = [vp, vp, u64, vp, vp, u64, C.POINTER(u64)]
        L.srd_crc32_batch.argtypes = [vp, vp, u64, vp, vp, u64, vp]
        L.srd_crc32_batch_device.argtypes = [vp, vp, vp, vp, u64, vp, vp]
        L.srd_xxh3_64_batch.argtypes = [vp, vp, u64, vp, vp, u64, vp]
        L.srd_xxh3_64_batch_device.argtypes = [vp, vp, vp, vp, u64, vp, vp]
        L.srd_padded_size.argtypes = [u64]
        L.srd_padded_size.restype = u64
        L.srd_synth_store_device.argtypes = [vp, vp, u64, u64, vp, u64, C.POINTER(u64)]
        L.srd_validate_span_device.argtypes = [vp, vp, u64, u64, u64, u32, C.POINTER(DeviceResult)]
        L.srd_shard_cuts.argtypes = [vp, u64, u32, vp]
        L.srd_index_partition_device.argtypes = [vp, vp, vp, u64, u32, vp, vp]
        L.srd_index_build_device.argtypes = [vp, vp, u64, vp, vp, C.POINTER(u64)]
        L.srd_synth_span_device.argtypes = [vp, vp, u64, u64, u64, u64, vp, u64, C.POINTER(u64), C.POINTER(u64)]
        L.srd_batch_layout.argtypes = [u64, vp, vp, vp, vp, vp, u64, u32, vp, C.POINTER(u64)]
        L.srd_batch_write.argtypes = [vp, u64, vp, vp, vp, vp, vp, vp, u64, u32, vp, u64, C.POINTER(u64), vp, vp]
        L.srd_batch_write_device.argtypes = [vp, vp, vp, vp, u64, vp, u64, vp, vp, vp]
        L.srd_index_table_bytes.argtypes = [u64]
        L.srd_index_table_bytes.restype = u64
        L.srd_index_table_build_device.argtypes = [vp, vp, vp, u64, vp, u64]
        L.srd_index_get_packed_device.argtypes = [vp, vp, u64, vp, u64, vp, vp]
        L.srd_batch_read_hashed_device.argtypes = [vp, vp, u64, vp, u64, vp, vp, u64, vp, vp, vp]
        L.srd_batch_read.argtypes = [vp, vp, u64, vp, u64, vp, vp, vp, u64, vp, vp]
        L.srd_iter_entries_device.argtypes = [vp, vp, u64, vp, u64, vp, vp, vp, vp, C.POINTER(u64)]
        L.srd_estimate_compaction_savings_device.argtypes = [vp, vp, u64, vp, u64, C.POINTER(u64)]
        L.srd_compact_device.argtypes = [vp, vp, u64, vp, u64, vp, u64, C.POINTER(u64), vp, vp]
        L.srd_validate_index_multi.argtypes = [C.POINTER(vp), u32, vp, u64, u32, C.POINTER(DeviceResult)]
        L.srd_ctx_stage_info.argtypes = [vp, C.POINTER(i32), C.POINTER(C.c_double)]
        L.srd_index_hash_device.argtypes = [vp, vp, u64, vp, vp]
        L.srd_validate_index_multi_device.argtypes = [C.POINTER(vp), u32, C.POINTER(vp), vp, vp, u32,
                                                      C.POINTER(DeviceResult), C.POINTER(MultiSummary)]
        L.srd_ctx_multi_summary.argtypes = [vp, C.POINTER(MultiSummary)]
        L.srd_ctx_multi_shard_ms.argtypes = [vp, C.POINTER(C.c_double), i32]
        L.srd_stream_probe_device.argtypes = [vp, vp, u64, i32, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        for f in EXPORTS:
            if f not in ("srd_ctx_destroy", "srd_result_free", "srd_ctx_stream", "srd_ctx_device_bytes", "srd_last_error",
                         "srd_build_info",
                         "srd_padded_size", "srd_index_table_bytes"):
                getattr(L, f).restype = i32
        _lib = L
    return _lib


class WriteEntry(C.Structure):
    """srd_write_entry (include/srd_amd.h)"""
    _fields_ = [("src", C.c_uint64), ("len", C.c_uint64), ("key_src", C.c_uint64), ("tail", C.c_uint64),
                ("key_len", C.c_uint32), ("flags", C.c_uint32)]


WRITE_ALLOW_NULL = 1


class SrdError(RuntimeError):
    pass


def _check(rc):
    if rc != 0:
        raise SrdError(f"srd error {rc}: {lib().srd_last_error().decode()}")


class Context:
    """One GPU + stream + reusable HBM workspace (srd_ctx)."""

    def __init__(self, device: int = 0):
        self.device = device
        self.h = C.c_void_p()
        _check(lib().srd_ctx_create(device, C.byref(self.h)))

    def close(self):
        if self.h:
            lib().srd_ctx_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_timing(self, level: int):
        """HIP-event timing level: TIMING_NONE (default), TIMING_SCAN, TIMING_CALL."""
        _check(lib().srd_ctx_set_timing(self.h, level))

    def set_timing_every(self, n: int):
        """With TIMING_SCAN: stamp only every n-th scan launch (srd_ctx_set_timing_every)."""
        _check(lib().srd_ctx_set_timing_every(self.h, n))

    def device_bytes(self) -> int:
        """srd_ctx_device_bytes: the context's device workspace (+ staging copy)."""
        return int(lib().srd_ctx_device_bytes(self.h))

    def scan_loads(self) -> int:
        """srd_ctx_scan_loads: 0 coalesced, 1 line per lane, -1 none yet."""
        return int(lib().srd_ctx_scan_loads(self.h))

    def scan_trial(self):
        """srd_ctx_scan_trial: (choice, best coalesced ms, best line-per-lane ms); choice -1 = still measuring."""
        ms = (C.c_double * 2)()
        ch = int(lib().srd_ctx_scan_trial(self.h, ms))
        return ch, float(ms[0]), float(ms[1])

    def timings(self):
        """(scan_ms, scan_launches) summed over the validate calls since the last
        read, and total_ms of the last call (HIP events; srd_ctx_timings)."""
        a, n, b = C.c_double(), C.c_int(), C.c_double()
        _check(lib().srd_ctx_timings(self.h, C.byref(a), C.byref(n), C.byref(b)))
        return a.value, n.value, b.value

    def scan_list(self) -> list[float]:
        """The individual scan durations (ms) behind the last timings() read."""
        n = lib().srd_ctx_scan_list(self.h, None, 0)
        if n < 0:
            _check(n)
        buf = (C.c_float * max(n, 1))()
        lib().srd_ctx_scan_list(self.h, buf, n)
        return list(buf[:n])

    @property
    def stream(self) -> int:
        return lib().srd_ctx_stream(self.h)

    def stage_info(self) -> tuple[str, float]:
        """(how the last host-input call staged the store (STAGE_MODES), its host wall ms)."""
        m, ms = C.c_int(), C.c_double()
        _check(lib().srd_ctx_stage_info(self.h, C.byref(m), C.byref(ms)))
        return STAGE_MODES.get(m.value, "none"), ms.value

    def stage_mode(self) -> str:
        return self.stage_info()[0]

    def multi_summary(self) -> MultiSummary:
        """srd_multi_summary of the last multi-GPU open with this context as ctxs[0]."""
        m = MultiSummary()
        _check(lib().srd_ctx_multi_summary(self.h, C.byref(m)))
        return m


_default_ctx = None


def default_ctx() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(int(os.environ.get("SRD_DEVICE", "0")))
    return _default_ctx


def _u8(file) -> np.ndarray:
    if isinstance(file, np.ndarray):
        return np.ascontiguousarray(file, dtype=np.uint8).reshape(-1)
    return np.frombuffer(memoryview(file), dtype=np.uint8)


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data) if a.size else C.c_void_p(0)


class Result:
    """Host copy of srd_result: the recovered tail, the chain and the index."""

    def __init__(self, r: DeviceResult):
        self.file_len = r.file_len
        self.final_len = r.final_len
        self.n_chain = r.n_chain
        self.n_index = r.n_index
        self.n_crc_bad = r.n_crc_bad
        self.n_candidates = r.n_candidates
        self.full_reason = r.full_reason
        self.mode = r.mode

        def arr(p, n, dt):
            if n == 0 or not p:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(np.ctypeslib.as_ctypes_type(dt))), (n,)).copy()

        n, ni = r.n_chain, r.n_index
        self.meta_off = arr(r.meta_off, n, np.uint64)
        self.key_hash = arr(r.key_hash, n, np.uint64)
        self.prev_offset = arr(r.prev_offset, n, np.uint64)
        self.payload_start = arr(r.payload_start, n, np.uint64)
        self.payload_len = arr(r.payload_len, n, np.uint64)
        self.crc_stored = arr(r.crc_stored, n, np.uint32)
        self.crc_computed = arr(r.crc_computed, n, np.uint32)
        self.crc_ok = arr(r.crc_ok, n, np.uint8)
        self.index_key_hash = arr(r.index_key_hash, ni, np.uint64)
        self.index_packed = arr(r.index_packed, ni, np.uint64)

    def index(self) -> dict[int, int]:
        return {int(k): int(v) for k, v in zip(self.index_key_hash, self.index_packed)}

    def chain(self) -> list[dict]:
        keys = ["meta_off", "key_hash", "prev_offset", "payload_start", "payload_len",
                "crc_stored", "crc_computed", "crc_ok"]
        return [{k: int(getattr(self, k)[i]) for k in keys} for i in range(self.n_chain)]


def validate_index(file, flags: int = 0, ctx: Context | None = None) -> Result:
    """The fused open-time pass: recover_valid_chain + KeyIndexer::build +
    is_valid_checksum over every chain entry, on the GPU."""
    ctx = ctx or default_ctx()
    a = _u8(file)
    r = DeviceResult()
    _check(lib().srd_validate_index(ctx.h, _ptr(a), a.size, flags, C.byref(r)))
    try:
        return Result(r)
    finally:
        lib().srd_result_free(C.byref(r))


def validate_index_call(file, flags: int = 0, ctx: Context | None = None) -> DeviceResult:
    """srd_validate_index alone: the result's arrays stay in the context-owned
    pinned host buffers (valid until the next call on ctx; `Result(r)` copies
    them into numpy).  The end-to-end timing of the library call."""
    ctx = ctx or default_ctx()
    a = _u8(file)
    r = DeviceResult()
    _check(lib().srd_validate_index(ctx.h, _ptr(a), a.size, flags, C.byref(r)))
    return r


def validate_index_multi(file, ctxs, flags: int = 0) -> Result:
    """DataStore::open's pass over one host store on len(ctxs) GPUs in one
    process (srd_validate_index_multi): entry-range shards, host composition,
    index merged latest-wins on ctxs[0]'s device; no RCCL.  Same result as
    validate_index."""
    a = _u8(file)
    hs = (C.c_void_p * len(ctxs))(*[c.h.value for c in ctxs])
    r = DeviceResult()
    _check(lib().srd_validate_index_multi(hs, len(ctxs), _ptr(a), a.size, flags, C.byref(r)))
    try:
        return Result(r)
    finally:
        lib().srd_result_free(C.byref(r))


def validate_index_multi_device(ctxs, spans, span_offs, cuts, flags: int = 0):
    """DataStore::open of a store resident in the HBM of len(ctxs) GPUs, one
    entry-range shard per context (srd_validate_index_multi_device; no RCCL):
    spans[i] = device pointer of file byte span_offs[i] .. cuts[i+1] on
    ctxs[i]'s GPU (0 for an empty shard).  Returns (shard results -- chain
    segment i and, by default, the index part owned by i, device arrays on
    ctxs[i]'s GPU --, MultiSummary)."""
    n = len(ctxs)
    hs = (C.c_void_p * n)(*[c.h.value for c in ctxs])
    sp = (C.c_void_p * n)(*[int(x or 0) for x in spans])
    so = np.ascontiguousarray(span_offs, np.uint64)
    cu = np.ascontiguousarray(cuts, np.uint64)
    assert so.size == n and cu.size == n + 1
    res = (DeviceResult * n)()
    summ = MultiSummary()
    _check(lib().srd_validate_index_multi_device(hs, n, sp, _ptr(so), _ptr(cu), flags, res, C.byref(summ)))
    return list(res), summ


def index_hash_device(d_keys: int, n: int, d_out: int, ctx: Context | None = None) -> None:
    """xxh3_64(le8(k)) per key on the device (the KeyIndexer's Xxh3BuildHasher)."""
    ctx = ctx or default_ctx()
    _check(lib().srd_index_hash_device(ctx.h, C.c_void_p(d_keys), n, C.c_void_p(d_out), C.c_void_p(ctx.stream)))


def validate_index_device(d_ptr: int, file_len: int, flags: int = 0, ctx: Context | None = None) -> DeviceResult:
    """Device-resident variant: d_ptr is a device pointer (e.g. a torch
    uint8 CUDA tensor's data_ptr()).  Result arrays stay in HBM."""
    ctx = ctx or default_ctx()
    r = DeviceResult()
    _check(lib().srd_validate_index_device(ctx.h, C.c_void_p(d_ptr), file_len, flags, C.byref(r)))
    return r


class _DevView:
    def __init__(self, ptr: int, n: int, typestr: str):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False), "version": 3}


_TYPESTR = {np.uint64: "<i8", np.uint32: "<i4", np.uint8: "|u1"}


def device_view(ptr: int, n: int, dtype=np.uint64, device: int = 0):
    """Zero-copy torch view of n elements of a library-owned device array
    (result arrays of the *_device calls; int64/int32/uint8 bit patterns)."""
    import torch
    if n == 0 or not ptr:
        return torch.empty(0, dtype={np.uint64: torch.int64, np.uint32: torch.int32, np.uint8: torch.uint8}[dtype],
                           device=f"cuda:{device}")
    return torch.as_tensor(_DevView(ptr, n, _TYPESTR[dtype]), device=f"cuda:{device}")


def device_to_numpy(ptr: int, n: int, dtype=np.uint64) -> np.ndarray:
    return device_view(ptr, n, dtype).cpu().numpy().view(dtype).copy()


def validate_span_device(d_ptr: int, span_off: int, lo: int, hi: int, flags: int = 0,
                         ctx: Context | None = None) -> DeviceResult:
    """Entry-range shard [lo, hi) of a store, resident at d_ptr = file byte
    span_off (srd_validate_span_device).  mode == SRD_MODE_SPAN_UNPROVEN means
    the caller must use the whole-file path."""
    ctx = ctx or default_ctx()
    r = DeviceResult()
    _check(lib().srd_validate_span_device(ctx.h, C.c_void_p(d_ptr), span_off, lo, hi, flags, C.byref(r)))
    return r


def index_partition_device(d_keys: int, d_vals: int, n: int, world: int, d_out_pairs: int,
                           ctx: Context | None = None) -> list[int]:
    """Group n device (key_hash, value) pairs by owner rank into interleaved
    pairs at d_out_pairs; returns the per-owner counts."""
    ctx = ctx or default_ctx()
    counts = np.zeros(max(world, 1), np.uint64)
    _check(lib().srd_index_partition_device(ctx.h, C.c_void_p(d_keys), C.c_void_p(d_vals), n, world,
                                            C.c_void_p(d_out_pairs), _ptr(counts)))
    return [int(x) for x in counts[:world]]


def index_build_device(d_pairs: int, n: int, d_out_keys: int, d_out_packed: int,
                       ctx: Context | None = None) -> int:
    """KeyIndexer::build over n interleaved device (key_hash, offset) pairs in
    file order; returns the index size."""
    ctx = ctx or default_ctx()
    out = C.c_uint64()
    _check(lib().srd_index_build_device(ctx.h, C.c_void_p(d_pairs), n, C.c_void_p(d_out_keys),
                                        C.c_void_p(d_out_packed), C.byref(out)))
    return out.value


def synth_span(d_ptr: int | None, span_off: int, first: int, n: int, payload_len: int = 4096, lens=None,
               seed: int = 0x5EED0001, ctx: Context | None = None) -> tuple[int, int]:
    """Shard of the synthetic store holding entries [first, first+n): returns
    (lo, hi); writes file bytes [span_off, hi) at d_ptr when given."""
    lo, hi = C.c_uint64(), C.c_uint64()
    lp = None
    if lens is not None:
        lens = np.ascontiguousarray(lens, np.uint64)
        lp = _ptr(lens)
    h = (ctx or default_ctx()).h if d_ptr else C.c_void_p(0)
    _check(lib().srd_synth_span_device(h, C.c_void_p(d_ptr or 0), span_off, first, n, payload_len, lp, seed,
                                       C.byref(lo), C.byref(hi)))
    return lo.value, hi.value


def recover_valid_chain(file, ctx: Context | None = None) -> int:
    """data_store.rs:383-482: the largest valid tail <= file_len (0 if none)."""
    ctx = ctx or default_ctx()
    a = _u8(file)
    out = C.c_uint64()
    _check(lib().srd_recover_valid_chain(ctx.h, _ptr(a), a.size, C.byref(out)))
    return out.value


def compute_hash_batch(keys, ctx: Context | None = None) -> list[int]:
    """compute_hash.rs:64-77"""
    ctx = ctx or default_ctx()
    keys = [bytes(k) for k in keys]
    buf = np.frombuffer(b"".join(keys) or b"\x00", np.uint8)
    lens = np.array([len(k) for k in keys], np.uint64)
    offs = np.zeros(len(keys), np.uint64)
    if len(keys) > 1:
        offs[1:] = np.cumsum(lens)[:-1]
    out = np.zeros(max(len(keys), 1), np.uint64)
    _check(lib().srd_xxh3_64_batch(ctx.h, _ptr(buf), buf.size, _ptr(offs), _ptr(lens), len(keys), _ptr(out)))
    return [int(x) for x in out[: len(keys)]]


def compute_hash(key: bytes) -> int:
    """compute_hash.rs:25-27"""
    return compute_hash_batch([key])[0]


def crc32_batch(buf, offs, lens, ctx: Context | None = None) -> np.ndarray:
    ctx = ctx or default_ctx()
    a = _u8(buf)
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint64)
    out = np.zeros(max(len(offs), 1), np.uint32)
    _check(lib().srd_crc32_batch(ctx.h, _ptr(a), a.size, _ptr(offs), _ptr(lens), len(offs), _ptr(out)))
    return out[: len(offs)]


def compute_checksum(data: bytes) -> bytes:
    """compute_checksum.rs:15-20: CRC-32 as 4 little-endian bytes."""
    d = bytes(data)
    v = int(crc32_batch(np.frombuffer(d or b"\x00", np.uint8), [0], [len(d)])[0])
    return v.to_bytes(4, "little")


class KeyIndexer:
    """key_indexer.rs: key_hash -> (tag16 << 48 | offset48).  Array-backed
    (the validate pass's index arrays, sorted by key_hash for lookups), so
    that adopting a million-key index costs a sort, not a Python dict."""

    def __init__(self, index: dict[int, int] | None = None, keys=None, packed=None):
        if index is not None:
            keys = np.fromiter(index.keys(), np.uint64, len(index))
            packed = np.fromiter(index.values(), np.uint64, len(index))
        keys = np.zeros(0, np.uint64) if keys is None else np.asarray(keys, np.uint64)
        packed = np.zeros(0, np.uint64) if packed is None else np.asarray(packed, np.uint64)
        o = np.argsort(keys, kind="stable")
        self._keys, self._packed = keys[o], packed[o]

    @classmethod
    def from_arrays(cls, keys: np.ndarray, packed: np.ndarray) -> "KeyIndexer":
        return cls(keys=keys, packed=packed)

    @property
    def index(self) -> dict[int, int]:
        return {int(k): int(v) for k, v in zip(self._keys, self._packed)}

    @staticmethod
    def tag_from_hash(key_hash: int) -> int:
        return key_hash >> (64 - TAG_BITS)

    @staticmethod
    def pack(tag: int, offset: int) -> int:
        return (tag << (64 - TAG_BITS)) | offset

    @staticmethod
    def unpack(packed: int) -> tuple[int, int]:
        return packed >> (64 - TAG_BITS), packed & OFFSET_MASK

    @classmethod
    def build(cls, file, tail: int, ctx: Context | None = None) -> "KeyIndexer":
        ctx = ctx or default_ctx()
        a = _u8(file)
        cap = max(1, tail // METADATA_SIZE + 1)
        k = np.zeros(cap, np.uint64)
        v = np.zeros(cap, np.uint64)
        n = C.c_uint64()
        _check(lib().srd_key_indexer_build(ctx.h, _ptr(a), tail, _ptr(k), _ptr(v), cap, C.byref(n)))
        return cls(keys=k[: n.value], packed=v[: n.value])

    def get_packed(self, key_hash: int):
        i = int(np.searchsorted(self._keys, np.uint64(key_hash)))
        if i < self._keys.size and int(self._keys[i]) == key_hash:
            return int(self._packed[i])
        return None

    def get_offset(self, key_hash: int):
        p = self.get_packed(key_hash)
        return None if p is None else p & OFFSET_MASK

    def __len__(self):
        return int(self._keys.size)


class EntryHandle:
    def __init__(self, store: "DataStore", i: int):
        self.store, self.i = store, i
        r = store.result
        self.metadata_offset = int(r.meta_off[i])
        self.start_offset = int(r.payload_start[i])
        self.end_offset = self.metadata_offset
        self.key_hash = int(r.key_hash[i])

    def as_slice(self) -> bytes:
        return bytes(self.store.mm[self.start_offset:self.end_offset])

    def checksum(self) -> int:
        return int(self.store.result.crc_stored[self.i])

    def is_valid_checksum(self) -> bool:
        """entry_handle.rs:260-275, computed on the GPU during open."""
        return bool(self.store.result.crc_ok[self.i])


class DataStore:
    """The part of DataStore::open (data_store.rs:84-117) this path replaces."""

    def __init__(self, path, mm, result: Result):
        self.path, self.mm, self.result = path, mm, result
        self.tail_offset = result.final_len
        self.key_indexer = KeyIndexer.from_arrays(result.index_key_hash, result.index_packed)

    @classmethod
    def open(cls, path, ctx: Context | None = None, ctxs=None, flags: int = 0) -> "DataStore":
        """ctxs: contexts of several GPUs (one process, srd_validate_index_multi);
        otherwise ctx (default: the default context).  The mapping is handed to
        the library as is; it stages it (registered mapping or bounce buffers)."""
        with open(path, "a+b"):
            pass
        size = os.path.getsize(path)
        with open(path, "r+b") as f:
            mm = _mmap.mmap(f.fileno(), 0, access=_mmap.ACCESS_READ) if size else b""
            view = np.frombuffer(mm, np.uint8) if size else b""
            if ctxs and len(ctxs) > 1:
                res = validate_index_multi(view, ctxs, flags)
            else:
                res = validate_index(view, flags, ctx=(ctxs[0] if ctxs else ctx))
            del view
        if res.final_len < size:
            # data_store.rs:91-104: warn, truncate to the valid tail, re-open
            import warnings
            warnings.warn(f"Truncating corrupted data in {path} from offset {res.final_len} to {size}.")
            if size and hasattr(mm, "close"):
                mm.close()
            with open(path, "r+b") as f:
                f.truncate(res.final_len)
                os.fsync(f.fileno())
            return cls.open(path, ctx, ctxs, flags)
        return cls(path, mm, res)

    def read_entry(self, key_hash: int):
        packed = self.key_indexer.get_packed(key_hash)
        if packed is None:
            return None
        tag, off = KeyIndexer.unpack(packed)
        if tag != KeyIndexer.tag_from_hash(key_hash):
            return None
        i = int(np.searchsorted(self.result.meta_off, np.uint64(off)))  # the chain is in file order
        if int(self.result.payload_len[i]) == 1 and self.mm[int(self.result.payload_start[i])] == 0:
            return None  # tombstone
        return EntryHandle(self, i)

    def read(self, key: bytes):
        return self.read_entry(compute_hash(key))

    def len(self) -> int:
        return len(self.key_indexer)


def shard_cuts(file: np.ndarray, world: int) -> list[int]:
    """Entry-tail cuts [0, c_1, .., file_len] splitting a host store into
    `world` byte-balanced entry ranges (host pre-pass, srd_shard_cuts)."""
    f = np.ascontiguousarray(file, dtype=np.uint8)
    cuts = np.zeros(world + 1, np.uint64)
    _check(lib().srd_shard_cuts(f.ctypes.data, f.size, world, cuts.ctypes.data))
    return [int(x) for x in cuts]


def padded_size(file_len: int) -> int:
    """Bytes a device buffer for validate_index_device must be readable for."""
    return int(lib().srd_padded_size(file_len))


def zipf_lens(n: int, seed: int = 0x5EED0003, s: float = 2.0) -> np.ndarray:
    """C3 payload sizes: 2^k bytes, k = 6..20, Zipf over
    rank k - 5 with exponent s; L = 2^k - j, j uniform in [0, 63], for k >= 7."""
    rng = np.random.default_rng(seed)
    r = np.arange(1, 16)
    p = 1.0 / r ** s
    p /= p.sum()
    k = rng.choice(np.arange(6, 21), size=n, p=p)
    j = rng.integers(0, 64, size=n)
    return ((1 << k) - np.where(k >= 7, j, 0)).astype(np.uint64)


def synth_store_len(n_entries: int, payload_len: int = 4096, lens=None) -> int:
    out = C.c_uint64()
    lp = None
    if lens is not None:
        lens = np.ascontiguousarray(lens, np.uint64)
        lp = _ptr(lens)
    _check(lib().srd_synth_store_device(C.c_void_p(0), None, n_entries, payload_len, lp, 0, C.byref(out)))
    return out.value


def synth_store_device(d_ptr: int, n_entries: int, payload_len: int = 4096, lens=None,
                       seed: int = 0x5EED0001, ctx: Context | None = None) -> int:
    ctx = ctx or default_ctx()
    out = C.c_uint64()
    lp = None
    if lens is not None:
        lens = np.ascontiguousarray(lens, np.uint64)
        lp = _ptr(lens)
    _check(lib().srd_synth_store_device(ctx.h, C.c_void_p(d_ptr), n_entries, payload_len, lp, seed, C.byref(out)))
    return out.value


# ---------------------------------------------------------------------------
# DataStoreWriter::batch_write (data_store.rs:838-939) -- the checksum-on-append
# writer (BASELINE config C5)

def _blob(parts):
    parts = [bytes(p) for p in parts]
    lens = np.array([len(p) for p in parts], np.uint64)
    offs = np.zeros(len(parts), np.uint64)
    if len(parts) > 1:
        offs[1:] = np.cumsum(lens)[:-1]
    buf = np.frombuffer(b"".join(parts) or b"\x00", np.uint8)
    return buf, offs, lens


def stream_probe_device(ptr: int, nbytes: int, reps: int = 8, ctx: Context | None = None):
    """srd_stream_probe_device: (best_ms, median_ms) of the scan-geometry
    streaming read of the first nbytes // 4096 tiles at device pointer ptr."""
    ctx = ctx or default_ctx()
    b, m = C.c_double(), C.c_double()
    _check(lib().srd_stream_probe_device(ctx.h, C.c_void_p(ptr), nbytes, reps, C.byref(b), C.byref(m)))
    return b.value, m.value


def batch_layout(tail: int, keys, payloads, allow_null: bool = False):
    """srd_batch_layout: (entries as a structured array, new tail); raises SrdError
    with the reference's InvalidInput messages (empty / NULL-byte payloads)."""
    kb, ko, kl = _blob(keys)
    pb, po, pl = _blob(payloads)
    n = len(payloads)
    out = (WriteEntry * max(n, 1))()
    nt = C.c_uint64()
    _check(lib().srd_batch_layout(tail, _ptr(pb), _ptr(ko), _ptr(kl), _ptr(po), _ptr(pl), n,
                                  WRITE_ALLOW_NULL if allow_null else 0, C.cast(out, C.c_void_p), C.byref(nt)))
    return out, int(nt.value)


def batch_write_raw(d_out: int, out_cap: int, tail: int, keys_ptr: int, key_offs: np.ndarray, key_lens: np.ndarray,
                    pay_ptr: int, pay_offs: np.ndarray, pay_lens: np.ndarray, flags: int = 0,
                    ctx: Context | None = None, want_index: bool = True):
    """srd_batch_write on caller buffers (host key / payload bytes at keys_ptr /
    pay_ptr, pinned for full PCIe rate; output in device memory d_out, which
    holds file bytes from tail & ~63).  Returns (new_tail, key_hashes, meta_offs)."""
    ctx = ctx or default_ctx()
    n = len(pay_lens)
    key_offs = np.ascontiguousarray(key_offs, np.uint64)
    key_lens = np.ascontiguousarray(key_lens, np.uint64)
    pay_offs = np.ascontiguousarray(pay_offs, np.uint64)
    pay_lens = np.ascontiguousarray(pay_lens, np.uint64)
    kh = np.zeros(max(n, 1), np.uint64) if want_index else None
    mo = np.zeros(max(n, 1), np.uint64) if want_index else None
    nt = C.c_uint64()
    _check(lib().srd_batch_write(ctx.h, tail, C.c_void_p(keys_ptr), _ptr(key_offs), _ptr(key_lens), C.c_void_p(pay_ptr),
                                 _ptr(pay_offs), _ptr(pay_lens), n, flags, C.c_void_p(d_out), out_cap, C.byref(nt),
                                 _ptr(kh) if want_index else None, _ptr(mo) if want_index else None))
    return int(nt.value), (kh[:n] if want_index else None), (mo[:n] if want_index else None)


def batch_write(keys, payloads, tail: int = 0, allow_null: bool = False, ctx: Context | None = None):
    """DataStoreWriter::batch_write on the GPU: keys hashed (compute_hash_batch),
    payloads CRC'd and serialized exactly as the reference appends them.
    Returns (new_tail, appended bytes [tail, new_tail), key_hashes, meta_offsets)."""
    import torch
    ctx = ctx or default_ctx()
    kb, ko, kl = _blob(keys)
    pb, po, pl = _blob(payloads)
    flags = WRITE_ALLOW_NULL if allow_null else 0
    nt = C.c_uint64()
    _check(lib().srd_batch_write(ctx.h, tail, _ptr(kb), _ptr(ko), _ptr(kl), _ptr(pb), _ptr(po), _ptr(pl),
                                 len(payloads), flags, None, 0, C.byref(nt), None, None))
    base = tail & ~63
    cap = max(int(nt.value) - base, 1)
    dev = torch.zeros(cap + 64, dtype=torch.uint8, device=f"cuda:{_ctx_device(ctx)}")
    new_tail, kh, mo = batch_write_raw(dev.data_ptr(), cap, tail, kb.ctypes.data, ko, kl, pb.ctypes.data, po, pl,
                                       flags, ctx)
    torch.cuda.synchronize()
    out = dev[tail - base: new_tail - base].cpu().numpy().tobytes()
    return new_tail, out, [int(x) for x in kh], [int(x) for x in mo]


def _ctx_device(ctx: Context) -> int:
    return int(os.environ.get("SRD_DEVICE", "0")) if ctx is None else getattr(ctx, "device", 0)


# ---------------------------------------------------------------------------
# Device KeyIndexer + batched keyed reads:
# KeyIndexer::get_packed (key_indexer.rs:164-167), batch_read /
# batch_read_hashed_keys (data_store.rs:1111-1158) over read_entry_with_context
# (:502-565)

INDEX_NONE = (1 << 64) - 1


class DeviceIndex:
    """The KeyIndexer adopted on the GPU: an open-addressing table in HBM built
    from n unique (key_hash, packed) device pairs -- e.g. the index arrays of a
    validate pass (DeviceResult.index_key_hash / index_packed)."""

    def __init__(self, d_keys: int, d_packed: int, n: int, ctx: Context | None = None):
        import torch
        self.ctx = ctx or default_ctx()
        self.n = n
        self.nbytes = int(lib().srd_index_table_bytes(n))
        self.table = torch.empty(self.nbytes, dtype=torch.uint8, device=f"cuda:{self.ctx.device}")
        _check(lib().srd_index_table_build_device(self.ctx.h, C.c_void_p(d_keys), C.c_void_p(d_packed), n,
                                                  C.c_void_p(self.table.data_ptr()), self.nbytes))

    def _dev_u64(self, a):
        import torch
        return torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(self.table.device)

    def get_packed(self, hashes) -> np.ndarray:
        """KeyIndexer::get_packed for each hash (INDEX_NONE when absent)."""
        import torch
        q = self._dev_u64(hashes)
        out = torch.empty_like(q)
        n = q.numel()
        _check(lib().srd_index_get_packed_device(self.ctx.h, C.c_void_p(self.table.data_ptr()), self.nbytes,
                                                 C.c_void_p(q.data_ptr()), n, C.c_void_p(out.data_ptr()),
                                                 C.c_void_p(self.ctx.stream)))
        torch.cuda.synchronize()
        return out.cpu().numpy().view(np.uint64)

    def batch_read_hashed_keys(self, d_file: int, file_len: int, hashes, non_hashed_keys=None):
        """batch_read_hashed_keys: [(start, end) | None] in query order; with
        non_hashed_keys, each read is verified by tag_from_key (data_store.rs:513-521)."""
        import torch
        if non_hashed_keys is not None and len(non_hashed_keys) != len(hashes):
            raise ValueError("Mismatched lengths for hashed and non-hashed keys.")
        q = self._dev_u64(hashes)
        v = self._dev_u64(compute_hash_batch(non_hashed_keys, self.ctx)) if non_hashed_keys is not None else None
        n = q.numel()
        st, en = torch.empty_like(q), torch.empty_like(q)
        torch.cuda.synchronize()
        _check(lib().srd_batch_read_hashed_device(self.ctx.h, C.c_void_p(self.table.data_ptr()), self.nbytes,
                                                  C.c_void_p(d_file), file_len, C.c_void_p(q.data_ptr()),
                                                  C.c_void_p(v.data_ptr()) if v is not None else None, n,
                                                  C.c_void_p(st.data_ptr()), C.c_void_p(en.data_ptr()),
                                                  C.c_void_p(self.ctx.stream)))
        torch.cuda.synchronize()
        s, e = st.cpu().numpy().view(np.uint64), en.cpu().numpy().view(np.uint64)
        return [None if a == b else (int(a), int(b)) for a, b in zip(s, e)]

    def batch_read(self, d_file: int, file_len: int, keys):
        """batch_read (data_store.rs:1111-1115): host keys, hashed and verified on the device."""
        kb, ko, kl = _blob(keys)
        n = len(keys)
        st = np.zeros(max(n, 1), np.uint64)
        en = np.zeros(max(n, 1), np.uint64)
        _check(lib().srd_batch_read(self.ctx.h, C.c_void_p(self.table.data_ptr()), self.nbytes, C.c_void_p(d_file),
                                    file_len, _ptr(kb), _ptr(ko), _ptr(kl), n, _ptr(st), _ptr(en)))
        return [None if a == b else (int(a), int(b)) for a, b in zip(st[:n], en[:n])]


# ---------------------------------------------------------------------------
# EntryIterator / par_iter_entries, estimate_compaction_savings and compact
# over the device index (data_store.rs:297-361, 605-749; entry_iterator.rs:69-126)

def iter_entries_device(d_file: int, file_len: int, d_index_packed: int, n_index: int, ctx: Context | None = None):
    """The latest non-tombstone entry per key, newest first (EntryIterator
    order): numpy arrays (start, end, meta_off, key_hash)."""
    import torch
    ctx = ctx or default_ctx()
    dev = f"cuda:{ctx.device}"
    outs = [torch.empty(max(n_index, 1), dtype=torch.int64, device=dev) for _ in range(4)]
    n = C.c_uint64()
    _check(lib().srd_iter_entries_device(ctx.h, C.c_void_p(d_file), file_len, C.c_void_p(d_index_packed), n_index,
                                         *[C.c_void_p(t.data_ptr()) for t in outs], C.byref(n)))
    k = int(n.value)
    return tuple(t[:k].cpu().numpy().view(np.uint64) for t in outs)


def estimate_compaction_savings_device(d_file: int, file_len: int, d_index_packed: int, n_index: int,
                                       ctx: Context | None = None) -> int:
    ctx = ctx or default_ctx()
    s = C.c_uint64()
    _check(lib().srd_estimate_compaction_savings_device(ctx.h, C.c_void_p(d_file), file_len,
                                                        C.c_void_p(d_index_packed), n_index, C.byref(s)))
    return int(s.value)


def compact_device(d_file: int, file_len: int, d_index_packed: int, n_index: int, ctx: Context | None = None):
    """compact(): the compacted store's bytes as a device tensor."""
    import torch
    ctx = ctx or default_ctx()
    nl = C.c_uint64()
    _check(lib().srd_compact_device(ctx.h, C.c_void_p(d_file), file_len, C.c_void_p(d_index_packed), n_index, None,
                                    0, C.byref(nl), None, None))
    out = torch.zeros(max(int(nl.value), 1) + 64, dtype=torch.uint8, device=f"cuda:{ctx.device}")
    _check(lib().srd_compact_device(ctx.h, C.c_void_p(d_file), file_len, C.c_void_p(d_index_packed), n_index,
                                    C.c_void_p(out.data_ptr()), out.numel(), C.byref(nl), None, None))
    torch.cuda.synchronize()
    return out[: int(nl.value)]
