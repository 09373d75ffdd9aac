"""Compare two .npz files array by array, bit for bit (tools/wmu_bits_probe.py output).  With one file
and two key prefixes, compare those arrays inside it:  python tools/npz_bits_cmp.py a.npz b.npz
|  python tools/npz_bits_cmp.py a.npz --within single_ multi15_"""
import sys

import numpy as np


def cmp(x, y, name):
    d = np.abs(x.astype(np.float64) - y.astype(np.float64)).max() if x.size else 0.0
    print(name, "equal" if np.array_equal(x, y) else f"DIFF max {d:.3e} n={np.count_nonzero(x != y)}")


if __name__ == "__main__":
    a = np.load(sys.argv[1])
    if sys.argv[2] == "--within":
        p, q = sys.argv[3], sys.argv[4]
        for k in a.files:
            if k.startswith(p) and q + k[len(p):] in a.files:
                cmp(a[k], a[q + k[len(p):]], f"{k} vs {q + k[len(p):]}")
    else:
        b = np.load(sys.argv[2])
        for k in a.files:
            if k in b.files:
                cmp(a[k], b[k], k)
