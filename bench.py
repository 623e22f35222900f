#!/usr/bin/env python3
"""Headline benchmark: device-resident validate+index of a synthetic 4 KiB-entry
store (BASELINE.json metric "GiB/s hashed (device-resident), full-file
validate+index scan"), N=1 workload = configs[1] (1M x 4 KiB, 4.06 GiB).

One step = one full srd_validate_index_device() pass over the store already
resident in HBM: chain recovery (recover_valid_chain), CRC-32 of every chain
payload + compare (is_valid_checksum), and the latest-wins index rebuild
(KeyIndexer::build).  value = algorithmic bytes sum(payload_len + 20) over all
ranks / max-over-ranks wall time of K steps.

N>1 (torchrun, one process per GPU): ONE global store of N x --entries-per-gpu
entries, sharded by entry range (SURVEY.md 8(e), config C4 at N=8 with 2^21
entries per GPU): rank r holds entries [r*n, (r+1)*n) in its HBM and a step
is srd_shard.sharded_validate_index -- its shard's validate+index
(srd_validate_span_device), the boundary composition check (all_gather) and
the owner-partitioned index exchange (all_to_all over RCCL, 16 B per key) +
owner-side KeyIndexer build.  Weak scaling; the step time is the MAX over
ranks.

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


def algorithmic_bytes(n_entries: int, payload: int) -> int:
    return n_entries * (payload + 20)  # sum(L_i + 20)


def cpu_baseline(store_dev: torch.Tensor, size: int, bytes_alg: int, budget_s: float):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # the checker / CPU restatement (test infrastructure)

    host = store_dev[:size].cpu().numpy()
    O.validate_index(host[: min(size, 1 << 26)], 1)  # warm the page cache / tables
    res = {}
    for threads in (1, os.cpu_count() or 1):
        threads = min(threads, 16)
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
    return {
        "value": round(one[0], 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"full C2 store ({size} B), oracle/srd_oracle.c faithful single-thread open()+"
        f"is_valid_checksum per chain entry (PCLMUL CRC), {one[2]*1e3:.1f} ms/pass",
        "all_cores": {"value": round(res[allc][0], 3), "cores": allc, "ms_per_pass": round(res[allc][2] * 1e3, 2)},
        "check": {"final_len": one[1].final_len, "n_chain": one[1].n_chain, "n_index": one[1].n_index},
    }


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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["c2", "c3", "c5", "ops"], default="c2",
                    help="c2: 4 KiB entries (headline); c3: Zipf-sized entries 64 B..1 MiB (variable length); "
                         "c5: checksum-on-append batch write of 1M x 4 KiB from pinned host memory")
    ap.add_argument("--entries-per-gpu", type=int, default=None)
    ap.add_argument("--payload", type=int, default=4096)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--e2e", action="store_true", help="also time host->HBM->result end to end (stderr)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if os.environ.get("SRD_BENCH_SAME_DEVICE"):  # rehearsal of N>1 on a 1-GPU box (gloo, all ranks on cuda:0)
        local = 0
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(os.environ.get("SRD_DIST_BACKEND", "nccl"), init_method="env://")
    torch.cuda.set_device(local)
    ctx = S.Context(local)

    if args.config == "c5":
        return bench_c5(args, ctx, local)
    if args.config == "ops":
        return bench_ops(args, ctx, local)
    n, L = args.entries_per_gpu, args.payload
    if n is None:
        n = 1 << 20 if args.config == "c2" else 10_000_000
    lens, seed = None, 0x5EED0001
    if args.config == "c3":
        lens, seed = S.zipf_lens(n * world), 0x5EED0004
    if world == 1:
        size = S.synth_store_len(n, L, lens)
        store = torch.empty(S.padded_size(size), dtype=torch.uint8, device=f"cuda:{local}")
        S.synth_store_device(store.data_ptr(), n, L, lens, seed=seed, ctx=ctx)
        span = (0, 0, size)

        def step():
            r = S.validate_index_device(store.data_ptr(), size, 0, ctx)
            return r.final_len, r.n_chain, r.n_crc_bad, r.n_index
        expect = (size, n, 0, n)
    else:
        import srd_shard as SH
        first, cnt = SH.plan_entry_shards(n * world, world)[rank]
        lo, hi = S.synth_span(None, 0, first, cnt, L, lens)
        file_len = S.synth_store_len(n * world, L, lens)
        span_off = lo - lo % S.SPAN_ALIGN
        size = hi - span_off
        store = torch.empty(S.padded_size(size), dtype=torch.uint8, device=f"cuda:{local}")
        S.synth_span(store.data_ptr(), span_off, first, cnt, L, lens, seed=seed, ctx=ctx)
        span = (span_off, lo, hi)
        backend = SH.HipBackend(ctx, local)

        def step():
            r = SH.sharded_validate_index(backend, store, span_off, lo, hi, file_len)
            return r.final_len, r.n_chain, r.n_crc_bad, r.n_index
        expect = (file_len, n * world, 0, n * world)
    torch.cuda.synchronize()
    if lens is None:
        bytes_alg = algorithmic_bytes(n, L)
    else:  # this rank's entries: sum(L_i + 20)
        f0 = rank * n if world > 1 else 0
        bytes_alg = int(lens[f0:f0 + n].sum()) + 20 * n

    for _ in range(args.warmup):
        got = step()
    assert got == expect, (got, expect)

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    scan_ms_sum, scan_n = 0.0, 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        sm, sn, _ = ctx.timings()
        scan_ms_sum += sm
        scan_n += sn
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], device="cpu" if dist.get_backend() == "gloo" else f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    ms_per_step = dt / args.steps * 1e3
    value = bytes_alg * world / dt * args.steps / 2**30
    scan_ms = scan_ms_sum / max(scan_n, 1)
    achieved = bytes_alg / (scan_ms * 1e-3) / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tf) and world == 1 and n == 1 << 20 and L == 4096 and args.config == "c2":  # measured on the C2 workload only
        try:
            traffic = json.load(open(tf)).get("scan_kernel_hbm_bytes_per_launch")
        except Exception:
            traffic = None

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
        "config": {
            "workload": (f"{args.config.upper()}: {n} x " + (f"{L} B" if lens is None else "Zipf 64 B..1 MiB") +
                         f" entries, {size} B store, validate+index (recover_valid_chain + CRC-32 every payload + "
                         f"KeyIndexer::build)") if world == 1 else
                        (f"{args.config.upper()}: {n * world} entries, one store sharded by entry range over {world} "
                         f"GPUs ({n} entries per GPU), validate+index + index exchange"),
            "entries_per_gpu": n,
            "payload_bytes": L,
            "store_bytes_per_gpu": span[2] - span[1],
            "algorithmic_bytes_per_gpu": bytes_alg,
            "parallelism": "1 GPU" if world == 1 else
                           f"{world} entry-range shards, one per GPU; all_gather (boundaries) + "
                           f"all_to_all (index owners) over RCCL",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "scan_kernel<false>",
            "kernel_ms": round(scan_ms, 4),
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu and args.config == "c2":
        out["cpu_baseline"] = cpu_baseline(store, size, bytes_alg, args.cpu_budget)
    if args.e2e and rank == 0:
        host = torch.empty(size, dtype=torch.uint8).pin_memory()
        host.copy_(store[:size])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            res = S.validate_index(host.numpy(), 0, ctx)
        e2e = (time.perf_counter() - t0) / 3
        print(json.dumps({"e2e_host_to_index_ms": round(e2e * 1e3, 2),
                          "e2e_GiBps": round(bytes_alg / e2e / 2**30, 3),
                          "final_len": res.final_len}), file=sys.stderr)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
