#!/bin/bash
# Build libsit.so from a git revision into build_diag/libsit_<name>.so (A/B timing on one box).
#   usage: tools/build_rev.sh <rev> <name> [extra hipcc flags]
set -eu
cd "$(dirname "$0")/.."
rev=$1; name=$2; shift 2
d=$(mktemp -d)
mkdir -p "$d/include" "$d/csrc" build_diag
git show "$rev:include/sit.h" > "$d/include/sit.h"
git show "$rev:sac_maritime_ast_amd/csrc/sit_device.h" > "$d/csrc/sit_device.h"
git show "$rev:sac_maritime_ast_amd/csrc/sit_kernels.hip" > "$d/csrc/sit_kernels.hip"
# single-TU build (no -DSIT_F32_TU): pass "-Xarch_device -ffast-math" to match the float32 TU
for f in $(git ls-tree --name-only "$rev" sac_maritime_ast_amd/csrc/ | xargs -n1 basename | grep '\.h$'); do
  if git cat-file -e "$rev:sac_maritime_ast_amd/csrc/$f" 2>/dev/null; then
    git show "$rev:sac_maritime_ast_amd/csrc/$f" > "$d/csrc/$f"
  fi
done
(cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared \
   -fno-hip-fp32-correctly-rounded-divide-sqrt -I "$d/include" -I "$d/csrc" "$@" \
   "$d/csrc/sit_kernels.hip" -o "$OLDPWD/build_diag/libsit_$name.so")
rm -rf "$d"
