"""Build libcimq.so in-tree for gfx950 (MI355X) with hipcc.

    python -m cim_quantization_amd.build [--force]

hipcc cross-compiles without a GPU.  ``-ffp-contract=off`` keeps every fp32 operation
a separate IEEE operation (the bit-exact emulation of the reference's op sequence relies
on it); fp32 division stays correctly rounded (hipcc's default).
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libcimq.so")
ARCH = os.environ.get("CIMQ_OFFLOAD_ARCH", "gfx950")
# the kernels are written for 64-lane waves (wave-id = threadIdx >> 6, 32..1 shuffle
# butterflies); gfx9 targets (CDNA) have no wave32 mode, so anything else is refused
if not ARCH.startswith("gfx9"):
    raise SystemExit(f"libcimq targets wave64 CDNA GPUs (gfx9xx); CIMQ_OFFLOAD_ARCH={ARCH!r} refused")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) +
                  [os.path.join(REPO, "include", "cimq.h")])


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(s) <= t for s in sources())


def build(force: bool = False, verbose: bool = True, out: str = OUT, defines=()) -> str:
    """Compile libcimq.so (``defines``/``out``: experiment variants for tools/, never shipped)."""
    if not force and out == OUT and up_to_date():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-munsafe-fp-atomics", "-Wno-pass-failed"]
    cmd += [f"-D{d}" for d in defines]
    cmd += ["-o", out + ".tmp", os.path.join(CSRC, "cimq_api.hip")]
    if verbose:
        print("[cimq] " + " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
