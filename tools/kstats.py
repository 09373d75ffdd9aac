"""Per-kernel resource summary of a device assembly file (hipcc -S --cuda-device-only): VGPRs,
AGPRs, SGPRs, spills, scratch bytes and LDS, from the kernels' amdhsa metadata — the check that a
kernel change did not push a product kernel into scratch.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 -S -I include --cuda-device-only \\
        cnmf_amd/csrc/cnmf_hip.hip -o /tmp/all.s && python tools/kstats.py /tmp/all.s [name-regex]
"""
import re
import subprocess
import sys

KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
        ".private_segment_fixed_size", ".group_segment_fixed_size")


def demangle(names):
    try:
        out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt"], input="\n".join(names), text=True,
                             capture_output=True, check=True).stdout.splitlines()
        return out
    except Exception:
        return names


def main(path, pat=None):
    s = open(path).read()
    meta = s[s.index("amdhsa.kernels:"):]
    blocks = re.split(r"\n  - \.", meta)[1:]
    rows = []
    for b in blocks:
        name = re.search(r"\.name:\s+(\S+)", b)
        if not name:
            continue
        vals = {}
        for k in KEYS:
            m = re.search(re.escape(k) + r":\s+(\d+)", b)
            vals[k] = int(m.group(1)) if m else -1
        rows.append((name.group(1), vals))
    pretty = demangle([r[0] for r in rows])
    for (name, v), p in zip(rows, pretty):
        if pat and not re.search(pat, p):
            continue
        print(f"vgpr {v['.vgpr_count']:4d} agpr {v['.agpr_count']:4d} sgpr {v['.sgpr_count']:3d} "
              f"vspill {v['.vgpr_spill_count']:3d} sspill {v['.sgpr_spill_count']:3d} "
              f"scratch {v['.private_segment_fixed_size']:5d} lds {v['.group_segment_fixed_size']:6d}  {p[:150]}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/tmp/all.s", sys.argv[2] if len(sys.argv) > 2 else None)
