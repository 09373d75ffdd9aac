"""The C ABI's host code under AddressSanitizer: the library
source compiled with -Xarch_host -fsanitize=address (device code unsanitized: GPU ASan is not
available on this pool) and linked into tests/asan/abi_asan_main.cpp, which drives every entry
point's argument checks without a GPU (null pointers, bad shapes / dtypes / layouts / worlds, the
bounded error message).  The binary is cached under build/asan and rebuilt when a source is newer
(the host-sanitized build takes ~2.5 min)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "asan")
BIN = os.path.join(OUT, "abi_asan")
SRCS = [os.path.join(ROOT, "cnmf_amd", "csrc", "cnmf_hip.hip"), os.path.join(ROOT, "include", "cnmf_hip.h"),
        os.path.join(ROOT, "tests", "asan", "abi_asan_main.cpp"), os.path.join(ROOT, "tests", "asan", "build.sh")]


def _stale():
    return not os.path.exists(BIN) or any(os.path.getmtime(s) > os.path.getmtime(BIN) for s in SRCS)


@pytest.mark.timeout(900)
def test_c_abi_argument_checks_under_asan():
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not in this image")
    if _stale():
        subprocess.run(["bash", os.path.join(ROOT, "tests", "asan", "build.sh"), OUT], check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=850)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120, env=env)
    assert "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "0 failure(s)" in r.stdout
