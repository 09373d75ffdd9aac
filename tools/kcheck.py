"""Check of the BUILT library's persistent kernels (build and test infrastructure, not the product):
the prefetch registers of every wave-tile kernel must be touched only by their counted loads, the
LDS staging stores and the counted waits.

Why: the X / W prefetch of the wave-tile kernels lands in AGPRs through
inline-asm `global_load_dwordx4 a[..]` whose completion the kernel tracks with exact
`s_waitcnt vmcnt(N)`.  If the register allocator cannot keep all PD prefetch sets in AGPRs it
spills them — `scratch_store_dwordx4 a[..]` right after the load, before the data has landed — and
the staged tile is stale: the round-4 experiment at PD = 6 for the k = 8 streamed-W kernel did
exactly that (400 B of scratch, every load followed by a scratch store) and produced an all-NaN W
at 2.5x the time (profiles/r04/k8pd/).  The compiler does not report it, so the shipped code object
is checked here, from the library file itself:

    python tools/kcheck.py [cnmf_amd/libcnmf_hip.so]

Extracts the gfx950 code object (llvm-objcopy .hip_fatbin, clang-offload-bundler), disassembles it
(llvm-objdump) and, per kernel whose name matches the wave-tile families, collects the AGPRs that
are destinations of `global_load_dwordx4 a[..]` and lists every other instruction that reads or
writes one of them (besides the `ds_write_b128` / `ds_write_b64` staging stores from them and
`s_waitcnt`), plus any `vmcnt` immediate
above the 6-bit field.  Exit status 1 on a finding.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
FAMILIES = re.compile(r"(mu_iter_wt_kernel|mu_iter_mf8_kernel|wmu_iter_wt_kernel|als_iter_wt_kernel|"
                      r"mu_pass_bfw_kernel|mu_iter_bfw_kernel)")
OK_OPS = ("global_load_dwordx4", "ds_write_b128", "ds_write_b64", "s_waitcnt")


def disassemble(lib: str) -> str:
    """The gfx950 code object of `lib`, disassembled."""
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "dev.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.devnull],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                       check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                              capture_output=True, text=True).stdout


def kernels(dis: str):
    """(name, [instruction lines]) per function of the disassembly."""
    out, name, body = [], None, []
    for ln in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:$", ln)
        if m:
            if name:
                out.append((name, body))
            name, body = m.group(1), []
        elif name and ln.startswith("\t"):
            body.append(ln.split("//")[0].strip())
    if name:
        out.append((name, body))
    return out


def regs(text: str) -> set[int]:
    rs = set()
    for m in re.finditer(r"\ba(\d+)\b|\ba\[(\d+):(\d+)\]", text):
        rs.update([int(m.group(1))] if m.group(1) else range(int(m.group(2)), int(m.group(3)) + 1))
    return rs


def check_kernel(body):
    """(prefetch AGPR count, [offending instructions], [vmcnt immediates > 63])."""
    dst = set()
    for ins in body:
        if ins.startswith("global_load_dwordx4 a"):
            dst |= regs(ins.split(",")[0])
    bad = []
    for ins in body:
        if not ins or ins.startswith(OK_OPS):
            continue
        if regs(ins) & dst:
            bad.append(ins)
    big = [int(v) for v in re.findall(r"vmcnt\((\d+)\)", "\n".join(body)) if int(v) > 63]
    return len(dst), bad, big


def main(lib: str) -> int:
    dis = disassemble(lib)
    n_bad, n_k = 0, 0
    for name, body in kernels(dis):
        if not FAMILIES.search(name):
            continue
        n_k += 1
        nreg, bad, big = check_kernel(body)
        if bad or big:
            n_bad += 1
            print(f"FAIL {name}: prefetch AGPRs {nreg}, {len(bad)} other touches, vmcnt > 63: {big}")
            for ins in bad[:4]:
                print("     ", ins)
    print(f"kcheck: {n_k} wave-tile kernels checked, {n_bad} with prefetch registers touched outside "
          f"their loads / staging / waits")
    return 1 if n_bad or n_k == 0 else 0


if __name__ == "__main__":
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(root, "cnmf_amd", "libcnmf_hip.so")))
