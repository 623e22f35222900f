"""sha256 over the sources libsrd_amd.so is compiled from: every file under
csrc/ (.hip, .h, .cpp) and include/srd_amd.h, in sorted order, each as its
repo-relative name + NUL + its bytes.  The Makefile bakes it into the
library (srd_build_info); srd_amd.lib() recomputes it over the sources beside
the library and refuses a library built from other sources, so a GPU record
that prints the hash names the exact sources that ran."""
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def source_files() -> list[str]:
    csrc = os.path.join(HERE, "csrc")
    files = [os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".h", ".cpp"))]
    files.append(os.path.join(ROOT, "include", "srd_amd.h"))
    return sorted(files, key=lambda p: os.path.relpath(p, ROOT))


def source_hash() -> str:
    h = hashlib.sha256()
    for p in source_files():
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


if __name__ == "__main__":
    sys.stdout.write(source_hash())
