#!/bin/bash
# Host ASan + UBSan build of the C-ABI library (device code unsanitised; GPU sanitizers are not
# available on this pool), with the setup calls backed by host memory (-DSIT_HOST_MEMORY_TEST), then
# tests/test_abi_host.py against it on this GPU-less host.  Output: build_san/sanitize.log.
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build_san
mkdir -p "$OUT"
CLANG_LIB=$(ls -d /opt/rocm/lib/llvm/lib/clang/*/lib/linux | head -1)
cd /tmp
/opt/rocm/bin/hipcc -O1 -g -std=c++17 --offload-arch=gfx950 -fPIC -shared -DSIT_HOST_MEMORY_TEST \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all \
  -Xarch_host -fno-omit-frame-pointer \
  -I "$ROOT/include" -I "$ROOT/sac_maritime_ast_amd/csrc" \
  "$ROOT/sac_maritime_ast_amd/csrc/sit_kernels.hip" -o "$OUT/libsit_san.so" 2> "$OUT/build.log" || { tail -20 "$OUT/build.log"; exit 1; }
cd "$ROOT"
export LD_PRELOAD="$CLANG_LIB/libclang_rt.asan-x86_64.so${LD_PRELOAD:+:$LD_PRELOAD}"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export SIT_LIBRARY="$OUT/libsit_san.so"
python -m pytest tests/test_abi_host.py -v -p no:cacheprovider 2>&1 | tee "$OUT/sanitize.log" | tail -15
