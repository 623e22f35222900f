"""CPU-side checks of the drop-in boundary: the HIP library builds/loads and
exports every symbol include/srd_amd.h declares; host-side CRC algebra
self-test (no GPU calls)."""
import os
import re
import subprocess

import srd_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "srd_amd.h")).read()
    return sorted(set(re.findall(r"\b(srd_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_binding_list():
    assert declared_symbols() == sorted(srd_amd.EXPORTS)


def test_library_exports_every_declared_symbol():
    if not os.path.exists(srd_amd.LIB_PATH):
        srd_amd.build()
    out = subprocess.check_output(["nm", "-D", "--defined-only", srd_amd.LIB_PATH], text=True)
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing


def test_library_loads_and_host_selftest():
    L = srd_amd.lib()
    assert L.srd_selftest_host() == 0


def test_synth_len_matches_oracle():
    import oracle as O
    import numpy as np
    assert srd_amd.synth_store_len(1000) == 4_159_956
    assert srd_amd.synth_store_len(1 << 20) == 4_362_076_116
    lens = np.array([64, 1, 4096, 1000, 3, 1 << 20], np.uint64)
    assert srd_amd.synth_store_len(len(lens), lens=lens) == O.synth_store(len(lens), lens=lens).size


def test_kernel_pack_semantics():
    K = srd_amd.KeyIndexer
    kh = 0xABCD_1234_5678_9ABC
    assert K.tag_from_hash(kh) == 0xABCD
    assert K.unpack(K.pack(K.tag_from_hash(kh), 12345)) == (0xABCD, 12345)
