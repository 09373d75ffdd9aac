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

    python tools/kcheck.py [cnmf_amd/libcnmf_hip.so] [--arch gfx950] [--llvm DIR]

Extracts the gfx950 code object (llvm-objcopy .hip_fatbin, clang-offload-bundler), disassembles it
(llvm-objdump) and, per kernel whose name matches the wave-tile families, collects the AGPRs that
are destinations of `global_load_dwordx4 a[..]` and lists every other instruction that reads or
writes one of them (besides the `ds_write_b128` / `ds_write_b64` staging stores from them and
`s_waitcnt`), plus any `vmcnt` immediate
above the 6-bit field.  Exit status 1 on a finding; 2 when the check itself could not run (LLVM
tools missing, no code object for the arch) — reported apart from findings.  The arch
defaults to CNMF_OFFLOAD_ARCH (the build's) or gfx950; the LLVM tools are taken from --llvm, else
next to the hipcc the build used (HIPCC / <rocm>/lib/llvm/bin), else /opt/rocm/lib/llvm/bin.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

import shutil

LLVM = "/opt/rocm/lib/llvm/bin"


def llvm_dir() -> str:
    """The LLVM tools next to the hipcc the build uses (HIPCC, else the one on PATH), else LLVM."""
    for hip in (os.environ.get("HIPCC"), shutil.which("hipcc")):
        if hip and os.path.exists(hip):
            root = os.path.dirname(os.path.dirname(os.path.realpath(hip)))
            for d in (os.path.join(root, "lib", "llvm", "bin"), os.path.join(root, "llvm", "bin")):
                if os.path.exists(os.path.join(d, "llvm-objdump")):
                    return d
    return LLVM


class ToolError(RuntimeError):
    """The check could not run (not a finding)."""
FAMILIES = re.compile(r"(mu_iter_wt_kernel|mu_iter_mf8_kernel|wmu_iter_wt_kernel|als_iter_wt_kernel|"
                      r"mu_pass_bfw_kernel|mu_iter_bfw_kernel)")
OK_OPS = ("global_load_dwordx4", "ds_write_b128", "ds_write_b64", "s_waitcnt")


def disassemble(lib: str, arch: str = "gfx950", llvm: str = LLVM) -> str:
    """The `arch` code object of `lib`, disassembled; ToolError when a tool is missing or fails."""
    def run(cmd, **kw):
        if not os.path.exists(cmd[0]):
            raise ToolError(f"{cmd[0]} not found (pass --llvm DIR)")
        r = subprocess.run(cmd, capture_output=True, **kw)
        if r.returncode != 0:
            err = r.stderr if isinstance(r.stderr, str) else r.stderr.decode(errors="replace")
            raise ToolError(f"{os.path.basename(cmd[0])} failed ({r.returncode}): {err.strip()[-500:]}")
        return r
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "dev.co")
        run([f"{llvm}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.devnull])
        run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
             f"--targets=hipv4-amdgcn-amd-amdhsa--{arch}", f"--output={co}"])
        if not os.path.exists(co) or os.path.getsize(co) == 0:
            raise ToolError(f"{lib} holds no {arch} code object")
        dis = run([f"{llvm}/llvm-objdump", "-d", "--no-show-raw-insn", co], text=True).stdout
        readelf = f"{llvm}/llvm-readelf"
        notes = run([readelf, "--notes", co], text=True).stdout if os.path.exists(readelf) else ""
        return dis + "\n" + NOTES_MARK + "\n" + notes


NOTES_MARK = "=== kcheck: code object notes ==="
# VGPRs spilled to scratch per kernel family (round 6, from the code object's metadata): the wave-tile
# kernels run one or two waves per SIMD at their register ceiling, where a spill is a scratch round
# trip inside the streaming loop.  Budgets: 0, but the constrained ALS's TOL form, whose two spilled
# registers sit outside the loop.
SPILL_BUDGET = {"als_iter_wt_kernel": 2}


def spills(text: str) -> dict:
    """{kernel symbol: VGPR spill count} from the notes part of disassemble()'s output."""
    notes = text.split(NOTES_MARK, 1)[1] if NOTES_MARK in text else ""
    out = {}
    for blk in re.split(r"\n\s*- \.agpr_count", notes)[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk)
        sp = re.search(r"\.vgpr_spill_count:\s+(\d+)", blk)
        if name and sp:
            out[name.group(1)] = int(sp.group(1))
    return out


def kernels(dis: str):
    """(name, [instruction lines]) per function of the disassembly."""
    out, name, body = [], None, []
    for ln in dis.split(NOTES_MARK, 1)[0].splitlines():
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


def main(lib: str, arch: str | None = None, llvm: str | None = None) -> int:
    arch = arch or os.environ.get("CNMF_OFFLOAD_ARCH", "gfx950")
    try:
        dis = disassemble(lib, arch, llvm or llvm_dir())
    except ToolError as e:
        print(f"kcheck: could not check {lib} ({arch}): {e}", file=sys.stderr)
        return 2
    n_bad, n_k, n_sp = 0, 0, 0
    sp = spills(dis)
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
        fam = FAMILIES.search(name).group(1)
        if sp.get(name, 0) > SPILL_BUDGET.get(fam, 0):
            n_sp += 1
            print(f"FAIL {name}: {sp[name]} VGPRs spilled to scratch (budget {SPILL_BUDGET.get(fam, 0)})")
    print(f"kcheck: {n_k} wave-tile kernels checked, {n_bad} with prefetch registers touched outside "
          f"their loads / staging / waits, {n_sp} over their VGPR spill budget"
          + ("" if sp else " (no code object notes: spills not checked)"))
    return 1 if n_bad or n_sp or n_k == 0 else 0


if __name__ == "__main__":
    import argparse
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(root, "cnmf_amd", "libcnmf_hip.so"))
    ap.add_argument("--arch", default=None)
    ap.add_argument("--llvm", default=None)
    a = ap.parse_args()
    sys.exit(main(a.lib, a.arch, a.llvm))
