"""Build libcimq.so in-tree for gfx950 (MI355X) with hipcc.

    python -m cim_quantization_amd.build [--force]

hipcc cross-compiles without a GPU.  ``-ffp-contract=off`` keeps every fp32 operation
a separate IEEE operation (the bit-exact emulation of the reference's op sequence relies
on it); fp32 division stays correctly rounded (hipcc's default).
"""
from __future__ import annotations

import concurrent.futures
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


def units():
    """Translation units of libcimq.so: the C-ABI entry points and the kernel-family launchers
    (cimq_part_*.hip), compiled in parallel and linked into one shared library."""
    return [os.path.join(CSRC, "cimq_api.hip")] + sorted(glob.glob(os.path.join(CSRC, "cimq_part_*.hip")))


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
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wno-pass-failed"]
    # MFMA results straight into arch VGPRs: the epilogues read every partial sum / product,
    # and the default AGPR form costs one v_accvgpr_read per element (about 9 % of the forward's
    # VALU issue per slice pair)
    flags += ["-mllvm", "-amdgpu-mfma-vgpr-form"]
    flags += [f"-D{d}" for d in defines]
    objdir = out + ".objs"
    os.makedirs(objdir, exist_ok=True)
    jobs = []
    for u in units():
        obj = os.path.join(objdir, os.path.basename(u) + ".o")
        jobs.append((obj, [hipcc] + flags + ["-c", "-o", obj, u]))

    def run(job):
        obj, cmd = job
        if verbose:
            print("[cimq] " + " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        return obj

    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with concurrent.futures.ThreadPoolExecutor(workers) as ex:
        objs = list(ex.map(run, jobs))
    link = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wl,--no-undefined", "-o", out + ".tmp"] + objs
    if verbose:
        print("[cimq] " + " ".join(link), flush=True)
    subprocess.run(link, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
