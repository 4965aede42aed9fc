#!/bin/bash
# Build the working tree's libsit as one TU into build_diag/libsit_<name>.so (A/B timing against
# tools/build_rev.sh builds of a commit).   usage: tools/build_tree.sh <name> [extra hipcc flags]
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build_diag
(cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared \
   -fno-hip-fp32-correctly-rounded-divide-sqrt -I "$OLDPWD/include" -I "$OLDPWD/sac_maritime_ast_amd/csrc" "$@" \
   "$OLDPWD/sac_maritime_ast_amd/csrc/sit_kernels.hip" -o "$OLDPWD/build_diag/libsit_$name.so")
