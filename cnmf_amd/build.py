"""Build libcnmf_hip.so in-tree with hipcc for gfx950 (no JIT cache, no torch extension machinery).

    python -m cnmf_amd.build [--verbose]
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "cnmf_hip.hip")
OUT = os.path.join(HERE, "libcnmf_hip.so")
ARCH = os.environ.get("CNMF_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set HIPCC or install ROCm)")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    out_m = os.path.getmtime(OUT)
    deps = [SRC, os.path.join(ROOT, "include", "cnmf_hip.h")]
    return any(os.path.getmtime(d) > out_m for d in deps if os.path.exists(d))


def build(verbose: bool = False, force: bool = False, stamps: bool = False, diag: bool = False) -> str:
    """Compile libcnmf_hip.so.  Diagnostic builds, never loaded by the product (select one with
    CNMF_HIP_LIB=<path> in tools/ runs): stamps=True -> libcnmf_hip_stamps.so (in-kernel s_memtime /
    s_memrealtime stamps: per-phase sums, persistent-launch timelines; implies diag); diag=True ->
    libcnmf_hip_diag.so (the A/B environment switches CNMF_* and cnmf_hbm_probe)."""
    out = OUT.replace(".so", "_stamps.so") if stamps else (OUT.replace(".so", "_diag.so") if diag else OUT)
    if not force and not stamps and not diag and not needs_build():
        return OUT
    cmd = [hipcc(), "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-shared",
           "-I", os.path.join(ROOT, "include"), "-o", out + ".tmp", SRC]
    if stamps or diag:
        cmd.insert(1, "-DCNMF_DIAG")
    if stamps:
        cmd.insert(1, "-DCNMF_STAMPS")
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    if not stamps and not diag:
        # the shipped wave-tile kernels' prefetch registers must never be spilled (tools/kcheck.py)
        chk = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kcheck.py"), out + ".tmp"],
                             capture_output=True, text=True)
        if chk.returncode != 0:
            os.remove(out + ".tmp")
            raise RuntimeError("kernel check failed (prefetch registers touched outside their loads):\n"
                               + chk.stdout[-3000:])
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(verbose="--verbose" in sys.argv, force="--force" in sys.argv,
                stamps="--stamps" in sys.argv, diag="--diag" in sys.argv))
