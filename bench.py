#!/usr/bin/env python3
"""Headline benchmark: device-resident validate+index of a synthetic 4 KiB-entry
store (BASELINE.json metric "GiB/s hashed (device-resident), full-file
validate+index scan"), N=1 workload = configs[1] (1M x 4 KiB, 4.06 GiB).

One step = one full srd_validate_index_device() pass over the store already
resident in HBM: chain recovery (recover_valid_chain), CRC-32 of every chain
payload + compare (is_valid_checksum), and the latest-wins index rebuild
(KeyIndexer::build).  value = algorithmic bytes sum(payload_len + 20) over all
ranks / max-over-ranks wall time of K steps.

N>1 (`--gpus N`; under torchrun WORLD_SIZE must equal N): ONE global store of
N x --entries-per-gpu entries (default 2^21: the C4 partition, so N=8 is
exactly C4 -- 16M x 4 KiB, 65 GiB -- and N=2/4 its prefixes), sharded by entry
range: GPU i holds entries [i*n, (i+1)*n) in its HBM.  The
reference's open is one call, so ONE process (rank 0 under torchrun; the other
ranks exit) drives all N GPUs: a step is one srd_validate_index_multi_device
call -- per-GPU host threads run their shard's validate+index, the host
composes the shards, and the index is exchanged by owner with xGMI peer
copies (no RCCL).  Weak scaling; the call returns when every shard is done,
so the step time is the max over shards by construction.

Also prints: roofline of the dominant kernel (scan_kernel, HIP events on the
library's stream) and a CPU baseline (oracle/, the C restatement of the
reference path, timed on this host on rank 0 at N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rust-simd-r-drive_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import srd_amd as S  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def scan_sample(steps: int) -> int:
    """Stamp every k-th timed step: 10 stamped launches per run (k = steps // 10,
    at least 1) -- enough for min / median, and a stamped launch's ~7 us of
    extra wall time lands on a tenth of the steps, not half."""
    return max(1, steps // 10) if steps >= 10 else 1
PROBE_REPS = 8  # runs of the in-run streaming ceiling (srd_stream_probe_device; roofline.peak_measured)


def kernel_sources_hash() -> str:
    """sha256 over the HIP sources of the library (the PMC traffic in
    profiles/traffic.json is reported only for the sources it was measured on)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(ROOT, "rust-simd-r-drive_amd", "csrc", "*"))):
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()


def algorithmic_bytes(n_entries: int, payload: int) -> int:
    return n_entries * (payload + 20)  # sum(L_i + 20)


def host_cpus():
    """CPU model, the machine's logical CPUs, and the CPUs this process may
    use (affinity mask, capped by a cgroup CPU quota when one is set)."""
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return {"model": model, "machine_logical_cpus": os.cpu_count(), "affinity_cpus": usable,
            "cgroup_cpu_quota": quota, "usable": min(usable, quota) if quota else usable}


def cpu_baseline(store_dev: torch.Tensor, size: int, bytes_alg: int, budget_s: float):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # the checker / CPU restatement (test infrastructure)

    cpus = host_cpus()
    host = store_dev[:size].cpu().numpy()
    O.validate_index(host[: min(size, 1 << 26)], 1)  # warm the page cache / tables
    res = {}
    for threads in sorted({1, cpus["usable"]}):
        reps, t0 = 0, time.perf_counter()
        while True:
            st = O.validate_index(host, threads)
            reps += 1
            if time.perf_counter() - t0 > budget_s / 2 or reps >= 5:
                break
        dt = (time.perf_counter() - t0) / reps
        res[threads] = (bytes_alg / dt / 2**30, st, dt)
    one = res[1]
    allc = max(k for k in res)
    # C1 (BASELINE configs[0], benches/storage_benchmark.rs shape at 1000 x
    # 4 KiB): the same CPU open+validate+index on the plumbing-size store
    c1 = O.synth_store(1000)
    O.validate_index(c1, 1)
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        O.validate_index(c1, 1)
        reps += 1
    c1_ms = (time.perf_counter() - t0) / reps * 1e3
    return {
        "value": round(one[0], 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"full C2 store ({size} B) in host RAM (page cache warm: the bytes are resident, no I/O), "
        f"oracle/srd_oracle.c faithful single-thread open() + is_valid_checksum per chain entry "
        f"(PCLMUL CRC), {one[2]*1e3:.1f} ms/pass",
        "host": cpus,
        "all_cores": {"value": round(res[allc][0], 3), "cores": allc, "ms_per_pass": round(res[allc][2] * 1e3, 2),
                      "note": "CRC pass split over the usable CPUs (par_iter_entries analogue)"},
        "c1_plumbing": {"entries": 1000, "store_bytes": int(c1.size), "ms_per_open": round(c1_ms, 3),
                        "cores": 1},
        "check": {"final_len": one[1].final_len, "n_chain": one[1].n_chain, "n_index": one[1].n_index},
    }


def e2e(store, size, bytes_alg, ctx, reps=3):
    """End to end from host memory (the path starts in the mmap'd file,
    data_store.rs:172-174): host bytes -> HBM -> validate+index -> host
    result arrays (srd_validate_index, the library call: its arrays left in
    the context's pinned buffers).  Variants: a pinned host buffer; the
    store as a FILE in the page cache, mapped afresh each time (mmap ->
    srd_validate_index -> munmap, page faults included) under each staging
    mode, and with MAP_POPULATE; the same after posix_fadvise(DONTNEED) (a
    cold page cache when the kernel honours it); and the whole Python
    DataStore.open mirror (its dict-building is host Python, not the path).
    `stage_ms` = the library's staging share of each call."""
    import mmap as M
    import tempfile
    res = {"store_bytes": size}

    def row(dt, r=None):
        mode, st = ctx.stage_info()
        out = {"ms": round(dt * 1e3, 2), "GiBps": round(bytes_alg / dt / 2**30, 3), "staging": mode,
               "stage_ms": round(st, 2), "after_stage_ms": round(dt * 1e3 - st, 2)}
        if r is not None:
            assert r.final_len == size and r.n_crc_bad == 0
        return out

    host = torch.empty(size, dtype=torch.uint8).pin_memory()
    host.copy_(store[:size])
    torch.cuda.synchronize()
    S.validate_index_call(host.numpy(), 0, ctx)
    t0 = time.perf_counter()
    for _ in range(reps):
        r = S.validate_index_call(host.numpy(), 0, ctx)
    res["pinned_buffer"] = row((time.perf_counter() - t0) / reps, r)
    # the Python mirror's Result copies the ~77 MB of host arrays into numpy:
    # its cost, apart from the library call
    t0 = time.perf_counter()
    S.Result(r)
    res["python_result_copy_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
    del host
    d = tempfile.mkdtemp(prefix="srd_e2e_")
    path = os.path.join(d, "c2.store")

    def mapped(flags, populate=False):
        fd = os.open(path, os.O_RDONLY)
        try:
            mm = M.mmap(fd, 0, flags=M.MAP_SHARED | (M.MAP_POPULATE if populate else 0), prot=M.PROT_READ)
            v = np.frombuffer(mm, np.uint8)
            r = S.validate_index_call(v, flags, ctx)
            del v
            mm.close()
            return r
        finally:
            os.close(fd)

    try:
        with open(path, "wb") as f:
            store[:size].cpu().numpy().tofile(f)
            f.flush()
            os.fsync(f.fileno())
        for name, flags, pop in (("mmap_default", 0, False), ("mmap_register", S.SRD_FLAG_STAGE_REGISTER, False),
                                 ("mmap_pageable", S.SRD_FLAG_STAGE_PAGEABLE, False),
                                 ("mmap_populate_register", S.SRD_FLAG_STAGE_REGISTER, True)):
            best = None
            for _ in range(reps):
                t0 = time.perf_counter()
                r = mapped(flags, pop)
                dt = time.perf_counter() - t0
                if best is None or dt < best[0]:
                    best = (dt, row(dt, r))
            res[name] = best[1]
        fd = os.open(path, os.O_RDONLY)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
        os.close(fd)
        t0 = time.perf_counter()
        r = mapped(0)
        res["mmap_after_fadvise_dontneed"] = row(time.perf_counter() - t0, r)
        t0 = time.perf_counter()
        ds = S.DataStore.open(path, ctx)
        res["datastore_open_python_mirror"] = row(time.perf_counter() - t0)
        assert ds.tail_offset == size
        del ds
    finally:
        try:
            os.remove(path)
            os.rmdir(d)
        except OSError:
            pass
    return {"e2e": res}


def bench_c5(args, ctx, local):
    """BASELINE config C5: DataStoreWriter::batch_write of 1M x 4 KiB entries
    (keys bench-key-{i}, splitmix64 payloads) from PINNED host memory into HBM:
    srd_batch_write copies 64 MiB chunks on a side stream while write_kernel
    serializes the previous chunk (XXH3 key hash, prepad, payload copy + CRC-32,
    metadata).  The output must equal the C2 store byte for byte.  Also times
    the writer kernel alone on HBM-resident inputs (srd_batch_write_device)."""
    import ctypes as C
    n = args.entries_per_gpu or (1 << 20)
    L = 4096
    size = S.synth_store_len(n, L)
    dev = f"cuda:{local}"
    store = torch.empty(S.padded_size(size), dtype=torch.uint8, device=dev)
    S.synth_store_device(store.data_ptr(), n, L, ctx=ctx)
    pays_dev = store[: 4160 * n].view(n, 4160)[:, :L].contiguous()
    pin = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    pin.copy_(pays_dev.reshape(-1))
    keys = [b"bench-key-%d" % i for i in range(n)]
    kl = np.array([len(k) for k in keys], np.uint64)
    ko = np.zeros(n, np.uint64)
    ko[1:] = np.cumsum(kl)[:-1]
    kpin = torch.empty(int(kl.sum()), dtype=torch.uint8, pin_memory=True)
    kpin.copy_(torch.frombuffer(bytearray(b"".join(keys)), dtype=torch.uint8))
    lens = np.full(n, L, np.uint64)
    offs = np.arange(n, dtype=np.uint64) * L
    out = torch.empty(size + 64, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def step():
        return S.batch_write_raw(out.data_ptr(), size + 64, 0, kpin.data_ptr(), ko, kl, pin.data_ptr(), offs, lens,
                                 0, ctx, want_index=False)[0]
    for _ in range(args.warmup):
        assert step() == size
    torch.cuda.synchronize()
    assert torch.equal(out[:size], store[:size]), "C5 output differs from the C2 store"
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # the writer kernel alone, inputs resident in HBM (layout from srd_batch_layout)
    ents = (S.WriteEntry * n)()
    nt = C.c_uint64()
    S._check(S.lib().srd_batch_layout(0, None, S._ptr(ko), S._ptr(kl), S._ptr(offs), S._ptr(lens), n, 0,
                                      C.cast(ents, C.c_void_p), C.byref(nt)))
    d_ent = torch.frombuffer(bytearray(bytes(ents)), dtype=torch.uint8).to(dev)
    d_keys = kpin.to(dev)
    d_kh = torch.empty(n, dtype=torch.int64, device=dev)
    d_mo = torch.empty(n, dtype=torch.int64, device=dev)
    # everything on the library's stream (an ExternalStream view of it for torch)
    lib_stream = torch.cuda.ExternalStream(ctx.stream, device=dev)

    def kstep():
        S._check(S.lib().srd_batch_write_device(ctx.h, C.c_void_p(d_keys.data_ptr()), C.c_void_p(pays_dev.data_ptr()),
                                                C.c_void_p(d_ent.data_ptr()), n, C.c_void_p(out.data_ptr()), 0,
                                                C.c_void_p(d_kh.data_ptr()), C.c_void_p(d_mo.data_ptr()),
                                                C.c_void_p(ctx.stream)))
    torch.cuda.synchronize()
    with torch.cuda.stream(lib_stream):
        out.zero_()
        kstep()
    torch.cuda.synchronize()
    assert torch.equal(out[:size], store[:size]), "C5 device-resident output differs from the C2 store"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(lib_stream):
        e0.record()
        for _ in range(args.steps):
            kstep()
        e1.record()
    torch.cuda.synchronize()
    kms = e0.elapsed_time(e1) / args.steps
    written = size  # file bytes appended per step
    res = {
        "metric": "GiB/s appended (checksum-on-append batch write, pinned host -> HBM)",
        "value": round(written * args.steps / dt / 2**30, 3),
        "unit": "GiB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (keys bench-key-{i}, splitmix64 4 KiB payloads in pinned host memory); "
                "output verified byte-identical to the C2 store",
        "config": {"workload": f"C5: batch_write of {n} x {L} B entries, {size} B appended, 64 MiB chunks, "
                               "H2D on a side stream overlapped with write_kernel", "entries": n,
                   "payload_bytes": L, "store_bytes": size},
        "device_resident": {"kernel": "write_kernel", "ms": round(kms, 4),
                            "GBps_read_plus_write": round((n * L + int(kl.sum()) + size) / (kms * 1e-3) / 1e9, 1),
                            "GiBps_appended": round(size / (kms * 1e-3) / 2**30, 3)},
    }
    print(json.dumps(res), flush=True)


def bench_ops(args, ctx, local):
    """SURVEY.md 8(f) rows 2-4 on the C2 store (1M x 4 KiB, one validate pass
    first): device KeyIndexer adoption, batched keyed reads (batch_read_hashed_keys
    of every key, tag-verified), the EntryIterator, estimate_compaction_savings
    and compact (a full rewrite here: every key is live).  Device-resident;
    times are HIP-event / wall times per call (not the headline metric)."""
    import ctypes as C
    n = args.entries_per_gpu or (1 << 20)
    size = S.synth_store_len(n)
    dev = f"cuda:{local}"
    store = torch.empty(S.padded_size(size), dtype=torch.uint8, device=dev)
    S.synth_store_device(store.data_ptr(), n, 4096, ctx=ctx)
    r = S.validate_index_device(store.data_ptr(), size, 0, ctx)
    assert r.final_len == size and r.n_index == n
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    packed = torch.empty(n, dtype=torch.int64, device=dev)
    keys.copy_(torch.from_numpy(S.device_to_numpy(r.index_key_hash, n).view(np.int64)).to(dev))
    packed.copy_(torch.from_numpy(S.device_to_numpy(r.index_packed, n).view(np.int64)).to(dev))
    torch.cuda.synchronize()

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3
    idx = S.DeviceIndex(keys.data_ptr(), packed.data_ptr(), n, ctx)
    t_build = timed(lambda: S.DeviceIndex(keys.data_ptr(), packed.data_ptr(), n, ctx))
    st, en = torch.empty_like(keys), torch.empty_like(keys)

    def reads():
        S._check(S.lib().srd_batch_read_hashed_device(ctx.h, C.c_void_p(idx.table.data_ptr()), idx.nbytes,
                                                      C.c_void_p(store.data_ptr()), size, C.c_void_p(keys.data_ptr()),
                                                      C.c_void_p(keys.data_ptr()), n, C.c_void_p(st.data_ptr()),
                                                      C.c_void_p(en.data_ptr()), C.c_void_p(ctx.stream)))
        torch.cuda.synchronize()
    t_read = timed(reads)
    assert int((en - st).min()) == 4096
    outs = [torch.empty(n, dtype=torch.int64, device=dev) for _ in range(4)]
    nn = C.c_uint64()

    def it():
        S._check(S.lib().srd_iter_entries_device(ctx.h, C.c_void_p(store.data_ptr()), size,
                                                 C.c_void_p(packed.data_ptr()), n,
                                                 *[C.c_void_p(t.data_ptr()) for t in outs], C.byref(nn)))
    t_iter = timed(it)
    assert nn.value == n
    t_sav = timed(lambda: S.estimate_compaction_savings_device(store.data_ptr(), size, packed.data_ptr(), n, ctx))
    cout = torch.empty(S.padded_size(size), dtype=torch.uint8, device=dev)
    nl = C.c_uint64()

    def compact():
        S._check(S.lib().srd_compact_device(ctx.h, C.c_void_p(store.data_ptr()), size, C.c_void_p(packed.data_ptr()),
                                            n, C.c_void_p(cout.data_ptr()), size + 64, C.byref(nl), None, None))
    t_comp = timed(compact, 3)
    # the compacted store reopens to the same live key set, every CRC valid
    r2 = S.validate_index_device(cout.data_ptr(), nl.value, 0, ctx)
    assert (r2.final_len, r2.n_chain, r2.n_crc_bad, r2.n_index) == (nl.value, n, 0, n)
    k2 = torch.from_numpy(S.device_to_numpy(r2.index_key_hash, n).view(np.int64)).to(dev)
    assert torch.equal(torch.sort(k2).values, torch.sort(keys).values)
    res = {
        "metric": "device index + iterator + compaction ops on the C2 store (8(f) rows 2-4)",
        "config": {"workload": f"C2: {n} x 4096 B entries, {size} B store, every key live", "entries": n},
        "index_table_build_ms": round(t_build, 3),
        "batch_read_hashed_keys_all_ms": round(t_read, 3),
        "batch_read_Mkeys_per_s": round(n / t_read / 1e3, 1),
        "iter_entries_ms": round(t_iter, 3),
        "estimate_compaction_savings_ms": round(t_sav, 3),
        "compact_ms": round(t_comp, 3),
        "compact_GBps_read_plus_write": round(2 * nl.value / (t_comp * 1e-3) / 1e9, 1),
        "compacted_bytes": int(nl.value),
    }
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)  # ~55 ms timed: host-side jitter of single calls averages out
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", choices=["c2", "c2torn", "c2full", "c3", "c5", "ops"], default="c2",
                    help="c2: 4 KiB entries (headline); c2torn: the C2 store + b'CORRUPT' (persistence_tests.rs:"
                         "126-173: the torn-tail open; its start tail lies 7 bytes below file_len); c2full: the C2 "
                         "store through the full pass (SRD_FLAG_FORCE_FULL: what a store the optimistic pass cannot "
                         "prove costs); c3: Zipf-sized entries 64 B..1 MiB "
                         "(variable length); c5: checksum-on-append batch write of 1M x 4 KiB from pinned host memory")
    ap.add_argument("--entries-per-gpu", type=int, default=None)
    ap.add_argument("--payload", type=int, default=4096)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--e2e", action="store_true", help="also time host->HBM->result end to end (stderr)")
    args = ap.parse_args()

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = args.gpus
    if world_env > 1 and world_env != world:
        sys.exit(f"bench.py: --gpus {world} but WORLD_SIZE={world_env}: launch one rank per GPU with --gpus N")
    if world_env > 1:
        # DataStore::open is ONE call (data_store.rs:84-117): rank 0 drives all
        # N GPUs of the node in one process (srd_validate_index_multi_device,
        # per-GPU host threads, index exchange over xGMI peer copies, no RCCL);
        # the other ranks of a torchrun launch have nothing to do
        if rank != 0:
            return
        local = 0
    same_dev = bool(os.environ.get("SRD_BENCH_SAME_DEVICE"))  # rehearsal of N>1 on a 1-GPU box: every shard on cuda:0
    if world > 1 and not same_dev and torch.cuda.device_count() < local + world:
        sys.exit(f"bench.py: --gpus {world} needs {world} visible GPUs (found {torch.cuda.device_count()})")
    devs = [local if same_dev else local + i for i in range(world)]
    torch.cuda.set_device(local)
    ctx = S.Context(local)
    # the roofline's kernel time: HIP events stamped by the scan dispatch on
    # the library's stream, inside the timed region, on every scan_sample()-th
    # launch (an event-stamped launch costs ~7 us more wall time than a plain
    # one: a systematic sample keeps that off the other steps; the product
    # default is no events)
    ctx.set_timing(S.TIMING_SCAN)
    ctx.set_timing_every(scan_sample(args.steps))

    if args.config == "c5":
        return bench_c5(args, ctx, local)
    if args.config == "ops":
        return bench_ops(args, ctx, local)
    n, L = args.entries_per_gpu, args.payload
    torn = args.config == "c2torn"
    full = args.config == "c2full"
    if (torn or full) and world != 1:
        sys.exit(f"bench.py: --config {args.config} runs on one GPU")
    if n is None:  # N=1: C2 (1M x 4 KiB); N>1: the C4 partition (2^21 per GPU; N=8 is C4)
        n = (1 << 20 if world == 1 else 1 << 21) if args.config in ("c2", "c2torn", "c2full") else 10_000_000
    lens, seed = None, 0x5EED0001
    if args.config == "c3":
        lens, seed = S.zipf_lens(n * world), 0x5EED0004
    multi = None
    if world == 1:
        size = S.synth_store_len(n, L, lens)
        flen = size + (7 if torn else 0)  # c2torn: the tail b"CORRUPT" (persistence_tests.rs:126-173)
        store = torch.empty(S.padded_size(flen), dtype=torch.uint8, device=f"cuda:{local}")
        S.synth_store_device(store.data_ptr(), n, L, lens, seed=seed, ctx=ctx)
        if torn:
            store[size:flen].copy_(torch.frombuffer(bytearray(b"CORRUPT"), dtype=torch.uint8))
        span = (0, 0, size)

        vflags = S.SRD_FLAG_FORCE_FULL if full else 0

        def step():
            r = S.validate_index_device(store.data_ptr(), flen, vflags, ctx)
            return r.final_len, r.n_chain, r.n_crc_bad, r.n_index, r.mode
        expect = (size, n, 0, n, S.SRD_MODE_FULL if full else S.SRD_MODE_OPTIMISTIC)
    else:
        import ctypes as C
        import srd_shard as SH
        ctxs = [ctx] + [S.Context(d) for d in devs[1:]]
        for c in ctxs:
            c.set_timing(S.TIMING_SCAN)
            c.set_timing_every(scan_sample(args.steps))
        spans, soffs, cuts, keep = [], [], [0], []
        for i, (first, cnt) in enumerate(SH.plan_entry_shards(n * world, world)):
            lo, hi = S.synth_span(None, 0, first, cnt, L, lens)
            so = lo - lo % S.SPAN_ALIGN
            t = torch.empty(S.padded_size(hi - so), dtype=torch.uint8, device=f"cuda:{devs[i]}")
            S.synth_span(t.data_ptr(), so, first, cnt, L, lens, seed=seed, ctx=ctxs[i])
            keep.append(t)
            spans.append(t.data_ptr())
            soffs.append(so)
            cuts.append(hi)
        for d in set(devs):
            torch.cuda.synchronize(d)
        file_len = cuts[-1]
        store = keep[0]
        size = cuts[1] - cuts[0]
        span = (0, 0, size)
        hs = (C.c_void_p * world)(*[c.h.value for c in ctxs])
        sp = (C.c_void_p * world)(*spans)
        so_a = np.array(soffs, np.uint64)
        cu_a = np.array(cuts, np.uint64)
        res = (S.DeviceResult * world)()
        summ = S.MultiSummary()
        multi = {"validate_ms": 0.0, "exchange_ms": 0.0, "total_ms": 0.0, "scan_ms": [0.0] * world, "n": 0}

        def step():
            S._check(S.lib().srd_validate_index_multi_device(hs, world, sp, S._ptr(so_a), S._ptr(cu_a), 0, res,
                                                             C.byref(summ)))
            return summ.final_len, summ.n_chain, summ.n_crc_bad, summ.n_index, summ.path
        expect = (file_len, n * world, 0, n * world, S.SRD_MULTI_COMPOSED)
    # algorithmic bytes, SURVEY.md 8(d): sum(L_i + 20) over every chain entry
    # of the whole store (all N shards); bytes_alg = the first shard's share
    if lens is None:
        bytes_total = algorithmic_bytes(n * world, L)
        bytes_alg = algorithmic_bytes(n, L)
    else:
        bytes_total = int(lens[: n * world].sum()) + 20 * n * world
        bytes_alg = int(lens[:n].sum()) + 20 * n

    for _ in range(args.warmup):
        got = step()
    assert got == expect, (got, expect)

    for d in set(devs):
        torch.cuda.synchronize(d)
    # the warmup's scan events are read out (and dropped) here; the timed
    # steps' are read after the timed region (srd_ctx_timings sums every scan
    # launch since its previous call)
    for c in (ctxs if multi is not None else [ctx]):
        c.timings()
        c.set_timing_every(scan_sample(args.steps))  # restarts the sample: timed steps 0, k, 2k, ...
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if multi is not None:
            for k in ("validate_ms", "exchange_ms", "total_ms"):
                multi[k] += getattr(summ, k)
            multi["n"] += 1
    for d in set(devs):
        torch.cuda.synchronize(d)
    dt = time.perf_counter() - t0
    scan_ms_sum, scan_n, _ = ctx.timings()
    shard_ms = None
    if multi is not None:
        buf = (C.c_double * world)()
        k = S.lib().srd_ctx_multi_shard_ms(ctx.h, buf, world)
        shard_ms = [round(buf[i], 4) for i in range(min(k, world))]
    # the streaming-read ceiling of the scan's geometry on these very bytes,
    # after the timed region (the measured stream-read peak)
    probe_bytes = (flen if multi is None else cuts[1] - soffs[0]) // 4096 * 4096
    probe_best, probe_med = S.stream_probe_device(store.data_ptr(), probe_bytes, PROBE_REPS, ctx)
    scan_each = sorted(ctx.scan_list())  # the sampled timed steps' scan durations (ms), one per launch
    if multi is not None:
        multi["scan_ms"] = [(scan_ms_sum, scan_n)] + [c.timings()[:2] for c in ctxs[1:]]

    ms_per_step = dt / args.steps * 1e3
    value = bytes_total / dt * args.steps / 2**30
    scan_ms = scan_ms_sum / max(scan_n, 1)  # (the full pass too: one scan per call)
    if multi is not None:  # the slowest shard's scan bounds the step
        shard_scan = [x / max(k, 1) for x, k in multi["scan_ms"]]
        scan_ms = max(shard_scan)
    achieved = bytes_alg / (scan_ms * 1e-3) / 1e9
    traffic, traffic_note = None, None
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    if world == 1 and n == 1 << 20 and L == 4096 and args.config == "c2":  # measured on the C2 workload only
        try:
            t = json.load(open(tf))
            if t.get("kernel_sources_sha256") == kernel_sources_hash():
                traffic = t.get("scan_kernel_hbm_bytes_per_launch")
                traffic_note = f"PMC FETCH_SIZE x2 (gfx950) + WRITE_SIZE of these kernel sources ({t.get('measured')})"
            else:
                traffic_note = "profiles/traffic.json was measured on other kernel sources: not reported"
        except (OSError, ValueError):
            traffic_note = "no profiles/traffic.json"

    out = {
        "metric": "GiB/s hashed (device-resident), full-file validate+index scan",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (counter-mode splitmix64 payloads, keys bench-key-{i}), generated in HBM",
        # the sha256 baked into the loaded libsrd_amd.so (srd_build_info), equal to
        # the sources beside it (srd_amd.lib() refuses anything else)
        "build": {"libsrd_amd_src_sha256": S.build_info()},
        "config": {
            "workload": (("C4 partition at N=1 (the weak-scaling base: 2^21 x 4 KiB per GPU, as at N = 2/4/8)"
                          if args.config == "c2" and n == 1 << 21 and L == 4096 else args.config.upper()) +
                         f": {n} x " + (f"{L} B" if lens is None else "Zipf 64 B..1 MiB") +
                         f" entries, {size} B store" + (" + the 7-byte torn tail b'CORRUPT' (recovered: final_len = "
                                                        f"{size}, the optimistic pass from the start tail 7 bytes "
                                                        "below file_len)" if torn else "") +
                         (" through the full pass (SRD_FLAG_FORCE_FULL)" if full else "") +
                         ", validate+index (recover_valid_chain + CRC-32 every payload + "
                         f"KeyIndexer::build)") if world == 1 else
                        ((f"C4 partition ({'= C4' if world == 8 else f'prefix of C4, {world} of its 8 shards'})"
                          if args.config == "c2" and n == 1 << 21 and L == 4096 else args.config.upper()) +
                         f": {n * world} x {L} B entries, one store sharded by entry range over {world} "
                         f"GPUs ({n} entries per GPU), validate+index + index exchange"),
            "entries_per_gpu": n,
            "payload_bytes": L,
            "store_bytes_per_gpu": span[2] - span[1],
            "algorithmic_bytes_per_gpu": bytes_alg,
            "parallelism": "1 GPU" if world == 1 else
                           f"{world} entry-range shards, one per GPU, one process (srd_validate_index_multi_device): "
                           f"per-GPU host threads, host composition, index by owner via xGMI peer copies; no RCCL"
                           + (" [rehearsal: every shard on cuda:0]" if same_dev else ""),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "scan_kernel<true> (the full pass)" if full else "scan_kernel<false>",
            "kernel_ms": round(scan_ms, 4),
            # the distribution behind the mean (rocprof's kernel_stats for the same command: profiles/)
            "kernel_ms_min": round(scan_each[0], 4) if scan_each else None,
            "kernel_ms_median": round(scan_each[len(scan_each) // 2], 4) if scan_each else None,
            "kernel_launches": len(scan_each),
            "kernel_timing": "HIP events stamped with the scan dispatch's own start / stop (hipExtLaunchKernel) "
                             f"on the library stream, every {scan_sample(args.steps)}th timed step (a systematic sample: a "
                             "stamped launch costs ~7 us more wall time; read out after the timed region)",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            # the measured ceiling: srd_stream_probe_device streams the same
            # store with the scan's geometry (one 16-wave block per CU, 64 B
            # per lane, 3-deep ring) and does nothing with the bytes, best of
            # PROBE_REPS runs in this process.  peak_measured = file bytes /
            # probe ms; frac_measured = probe ms / scan ms (the scan against
            # streaming alone, in algorithmic bytes: both read the same file)
            "peak_measured": round(probe_bytes / (probe_best * 1e-3) / 1e9, 1),
            "probe_ms_best": round(probe_best, 4),
            "probe_ms_median": round(probe_med, 4),
            "frac_measured": round(probe_best / scan_ms, 4),
            "traffic": traffic,
            "traffic_note": traffic_note,
            # the whole step (scan + glue + one host sync) against the same peak
            "step_achieved": round(bytes_total / (ms_per_step * 1e-3) / 1e9 / world, 1),
            "step_frac": round(bytes_total / world / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        },
    }
    if multi is not None:
        k = max(multi["n"], 1)
        path_name = {S.SRD_MULTI_COMPOSED: "composed", S.SRD_MULTI_NEIGHBOUR: "neighbour",
                     S.SRD_MULTI_WHOLE_FILE: "whole_file"}.get(summ.path, str(summ.path))
        out["multi"] = {"devices": devs, "shard_scan_ms": [round(x, 4) for x in shard_scan],
                        "validate_ms": round(multi["validate_ms"] / k, 4),
                        "shard_validate_ms_last_call": shard_ms,
                        "exchange_ms": round(multi["exchange_ms"] / k, 4),
                        "call_ms": round(multi["total_ms"] / k, 4),
                        "path": path_name, "mode": int(summ.mode),
                        "peer_errors": int(summ.peer_errors), "shard_errors": int(summ.shard_errors),
                        "note": "validate_ms = the slowest shard's validate (host wall, its own thread); "
                                "exchange_ms = index by owner over xGMI peer reads + owner builds; path = how "
                                "the store composed (composed: every shard proven alone); peer_errors = cross-GPU "
                                "copies staged by the runtime because peer access was refused (0: every exchange "
                                "read the peers' HBM directly); step = max over shards by construction"}
    if world == 1:  # the library context's device workspace after the run (srd_ctx_device_bytes)
        out["workspace_bytes"] = ctx.device_bytes()
        # the tile-load pattern the pass measured fastest for this store (srd_ctx_scan_loads)
        out["roofline"]["scan_loads"] = {0: "coalesced + transpose", 1: "line per lane"}.get(ctx.scan_loads(), "none")
        _, t_co, t_li = ctx.scan_trial()  # the trial's fastest device-timed scan per pattern (srd_ctx_scan_trial)
        out["roofline"]["scan_loads_trial_ms"] = {"coalesced": round(t_co, 4), "lines": round(t_li, 4)}
    if world == 1 and not args.no_cpu and args.config == "c2":
        out["cpu_baseline"] = cpu_baseline(store, size, bytes_alg, args.cpu_budget)
    if args.e2e and world == 1:
        out_e2e = e2e(store, size, bytes_alg, ctx)
        print(json.dumps(out_e2e), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
