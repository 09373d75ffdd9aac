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


def _variant_out(stamps: bool, diag: bool) -> str:
    return OUT.replace(".so", "_stamps.so") if stamps else (OUT.replace(".so", "_diag.so") if diag else OUT)


def _compile_cmd(out: str, stamps: bool, diag: bool) -> list[str]:
    cmd = [hipcc(), "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-shared",
           "-I", os.path.join(ROOT, "include"), "-o", out + ".tmp", SRC]
    if stamps or diag:
        cmd.insert(1, "-DCNMF_DIAG")
    if stamps:
        cmd.insert(1, "-DCNMF_STAMPS")
    return cmd


def _finish(out: str, product: bool) -> str:
    if product:
        # the shipped wave-tile kernels' prefetch registers must never be spilled (tools/kcheck.py)
        env = dict(os.environ, HIPCC=hipcc(), CNMF_OFFLOAD_ARCH=ARCH)
        chk = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kcheck.py"), out + ".tmp",
                              "--arch", ARCH], capture_output=True, text=True, env=env)
        if chk.returncode == 2:  # the check could not run (tools / arch): not a finding
            os.remove(out + ".tmp")
            raise RuntimeError("kernel check could not run on the built library:\n" + chk.stderr[-3000:])
        if chk.returncode != 0:
            os.remove(out + ".tmp")
            raise RuntimeError("kernel check failed (prefetch registers touched outside their loads):\n"
                               + chk.stdout[-3000:] + chk.stderr[-2000:])
    os.replace(out + ".tmp", out)
    return out


def build(verbose: bool = False, force: bool = False, stamps: bool = False, diag: bool = False) -> str:
    """Compile libcnmf_hip.so.  Diagnostic builds, never loaded by the product (select one with
    CNMF_HIP_LIB=<path> in tools/ runs): stamps=True -> libcnmf_hip_stamps.so (in-kernel s_memtime /
    s_memrealtime stamps: per-phase sums, persistent-launch timelines; implies diag); diag=True ->
    libcnmf_hip_diag.so (the A/B environment switches CNMF_*, cnmf_hbm_probe and the layouts kept out
    of the product: 1-3 and the k = 8 matrix-core tiles, tests/test_gpu_mf8.py)."""
    out = _variant_out(stamps, diag)
    if not force and not stamps and not diag and not needs_build():
        return OUT
    cmd = _compile_cmd(out, stamps, diag)
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return _finish(out, not stamps and not diag)


def build_many(variants, verbose: bool = False) -> list[str]:
    """Compile several variants ((stamps, diag) pairs) as concurrent hipcc processes (one ~2.5 min
    compile each); the product variant is kcheck'ed as in build()."""
    procs = []
    for stamps, diag in variants:
        out = _variant_out(stamps, diag)
        cmd = _compile_cmd(out, stamps, diag)
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd), out, not stamps and not diag))
    bad = [(p.wait(), out) for p, out, _ in procs]
    bad = [out for rc, out in bad if rc != 0]
    if bad:
        raise RuntimeError(f"hipcc failed for {bad}")
    return [_finish(out, product) for _, out, product in procs]


if __name__ == "__main__":
    if "--all" in sys.argv:  # product + diagnostic + stamps, concurrently
        print(build_many([(False, False), (False, True), (True, True)], verbose="--verbose" in sys.argv))
    else:
        print(build(verbose="--verbose" in sys.argv, force="--force" in sys.argv,
                    stamps="--stamps" in sys.argv, diag="--diag" in sys.argv))
