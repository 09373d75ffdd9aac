"""Diagnostic: the streaming-read ceiling of the box for the persistent kernel's access shape
(tools/csrc/stream_probe.hip, built into tools/libstream_probe.so).  Prints GB/s per kernel and
workgroups per CU over a ~330 MB buffer read `passes` times per launch."""
from __future__ import annotations

import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    import torch
    lib = ctypes.CDLL(os.path.join(HERE, "libstream_probe.so"))
    lib.probe_name.restype = ctypes.c_char_p
    lib.probe_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_void_p]
    total = int(os.environ.get("PROBE_MB", "330")) << 20
    buf = torch.ones(total // 4, dtype=torch.float32, device="cuda")
    out = torch.zeros(8192, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    passes = int(os.environ.get("PROBE_PASSES", "20"))
    res = {}
    warm = torch.empty(1 << 28, dtype=torch.float32, device="cuda")
    for _ in range(50):
        warm.mul_(1.0001)  # clocks up
    only = os.environ.get("PROBE_ONLY")
    for i in range(lib.probe_count()):
        name = lib.probe_name(i).decode()
        if only and name not in only.split(","):
            continue
        U = lib.probe_U(i)
        tile = 256 * U * 16
        for wpc in (1, 2, 4):
            G = 256 * wpc
            nbt = total // (tile * G)
            nbt -= nbt % 4
            if nbt < 4:
                continue
            rc = lib.probe_launch(i, buf.data_ptr(), G, nbt, 1, out.data_ptr(), st.cuda_stream)
            if rc != 0:
                res[f"{name}_wpc{wpc}"] = f"launch failed {rc}"
                continue
            best = 0.0
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                lib.probe_launch(i, buf.data_ptr(), G, nbt, passes, out.data_ptr(), st.cuda_stream)
                e1.record(st)
                torch.cuda.synchronize()
                gbs = G * nbt * tile * passes / (e0.elapsed_time(e1) / 1e3) / 1e9
                best = max(best, gbs)
            res[f"{name}_wpc{wpc}"] = round(best, 1)
            print(f"{name:16s} {wpc} WG/CU  tile {tile // 1024} KB  {G * nbt * tile / 1e6:.0f} MB: {best:.0f} GB/s", flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
