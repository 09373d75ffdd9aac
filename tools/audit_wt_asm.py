"""Audit of the wave-tile kernels' assembly (hipcc -S --cuda-device-only): the X / W prefetch
AGPRs (inline-asm global_load_dwordx4 destinations) may be touched only by those loads, the
ds_write_b128 that stage them and the waits — any other access (a copy, a spill) would read data
that has not landed.  Also reports the vmcnt of the staging waits.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -S -I include --cuda-device-only \\
        cnmf_amd/csrc/cnmf_hip.hip -o /tmp/all.s && python tools/audit_wt_asm.py /tmp/all.s
"""
import re
import sys


def main(path):
    s = open(path).read()
    names = re.findall(r"^(_ZN4cnmf17mu_iter_wt_kernel\w+|_ZN4cnmf18mu_iter_mf8_kernel\w+|_Z18wmu_iter_wt_kernel\w+|_Z18als_iter_wt_kernel\w+):", s, re.M)
    bad_total = 0
    for name in names:
        i = s.index(name + ":")
        j = s.index(".Lfunc_end", i)
        lines = s[i:j].splitlines()
        dst = set()
        for ln in lines:
            m = re.search(r"global_load_dwordx4 a\[(\d+):(\d+)\]", ln)
            if m:
                dst.update(range(int(m.group(1)), int(m.group(2)) + 1))
        bad = []
        for n, ln in enumerate(lines):
            t = ln.strip()
            if not t or t.startswith(";") or "global_load_dwordx4" in t or "ds_write_b128" in t:
                continue
            for m in re.finditer(r"\ba(\d+)\b|a\[(\d+):(\d+)\]", t):
                rs = [int(m.group(1))] if m.group(1) else range(int(m.group(2)), int(m.group(3)) + 1)
                if any(r in dst for r in rs):
                    bad.append((n, t))
        waits = sorted({int(m) for m in re.findall(r"s_waitcnt vmcnt\((\d+)\)", s[i:j])})
        print(f"{name}: prefetch AGPRs {len(dst)}, other touches {len(bad)}, vmcnt values {waits}")
        for b in bad[:5]:
            print("   ", b)
        bad_total += len(bad)
    return 1 if bad_total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "/tmp/all.s"))
