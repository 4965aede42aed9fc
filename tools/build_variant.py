#!/usr/bin/env python3
"""Build a variant of libsit.so from the working tree into build_diag/libsit_<name>.so (A/B timing
with SIT_LIBRARY=...; tools/ab_libs.sh).  usage: tools/build_variant.py <name> [hipcc flags ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

name, extra = sys.argv[1], sys.argv[2:]
os.makedirs(os.path.join(ROOT, "build_diag"), exist_ok=True)
g.compile_library(os.path.join(ROOT, "build_diag", f"libsit_{name}.so"), extra)
print("built", name)
