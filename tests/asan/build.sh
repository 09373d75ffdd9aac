#!/bin/bash
# AddressSanitizer build of the C ABI's HOST code (-Xarch_host: the device code is compiled normally
# and never sanitized — GPU ASan is not available on this pool; every check runs without a GPU):
#   tests/asan/build.sh <out-dir>   ->  <out-dir>/abi_asan
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$(cd "$HERE/../.." && pwd)"
OUT="${1:-$ROOT/build/asan}"
mkdir -p "$OUT"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
"$HIPCC" -std=c++17 -O1 -g --offload-arch=gfx950 -Xarch_host -fsanitize=address \
  -Xarch_host -fno-omit-frame-pointer -I "$ROOT/include" -c "$ROOT/cnmf_amd/csrc/cnmf_hip.hip" -o "$OUT/cnmf_hip_host.o"
CXX=/opt/rocm/lib/llvm/bin/clang++
"$CXX" -std=c++17 -O1 -g -fsanitize=address -fno-omit-frame-pointer -I "$ROOT/include" \
  -c "$HERE/abi_asan_main.cpp" -o "$OUT/abi_asan_main.o"
"$CXX" -fsanitize=address "$OUT/abi_asan_main.o" "$OUT/cnmf_hip_host.o" -L/opt/rocm/lib -lamdhip64 \
  -Wl,-rpath,/opt/rocm/lib -o "$OUT/abi_asan"
echo "$OUT/abi_asan"
