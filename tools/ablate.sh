#!/bin/bash
# Build diagnostic variants of libsit.so (never shipped) for phase timing:
#   libsit_nopred.so  polygon predicates removed (-DSIT_ABLATE_PREDICATES)
#   libsit_nohull.so  hull and IW polygon tests removed, boundary distance kept (-DSIT_ABLATE_HULL)
set -eu
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -shared -fno-hip-fp32-correctly-rounded-divide-sqrt -I include -I sac_maritime_ast_amd/csrc"
(cd /tmp && /opt/rocm/bin/hipcc $F -I "$OLDPWD/include" -I "$OLDPWD/sac_maritime_ast_amd/csrc" -DSIT_ABLATE_PREDICATES \
   "$OLDPWD/sac_maritime_ast_amd/csrc/sit_kernels.hip" -o "$OLDPWD/build_diag/libsit_nopred.so")
(cd /tmp && /opt/rocm/bin/hipcc $F -I "$OLDPWD/include" -I "$OLDPWD/sac_maritime_ast_amd/csrc" -DSIT_ABLATE_HULL \
   "$OLDPWD/sac_maritime_ast_amd/csrc/sit_kernels.hip" -o "$OLDPWD/build_diag/libsit_nohull.so")
