#!/usr/bin/env python3
"""Build a variant of libsit.so into build_diag/libsit_<name>.so for A/B timing on one box
(SIT_LIBRARY=build_diag/libsit_<name>.so; tools/ab_libs.sh), with the product's two-TU recipe
(__graft_entry__.compile_library).

  tools/build_variant.py <name> [--rev <git revision>] [--f32 "<flags for the float32 TU only>"] [--default-sched]
                         [hipcc flags ...]

--rev builds the sources of that revision (include/ and sac_maritime_ast_amd/csrc/ from git) instead
of the working tree."""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

args = sys.argv[1:]
name, rest = args[0], args[1:]
rev = None
if rest[:1] == ["--rev"]:
    rev, rest = rest[1], rest[2:]
f32 = []
if rest[:1] == ["--f32"]:
    f32, rest = rest[1].split(), rest[2:]
sched = None
if rest[:1] == ["--default-sched"]:   # the float32 TU without the max-ILP machine scheduler
    sched, rest = [], rest[1:]
os.makedirs(os.path.join(ROOT, "build_diag"), exist_ok=True)
out = os.path.join(ROOT, "build_diag", f"libsit_{name}.so")
if rev is None:
    g.compile_library(out, rest, f32, f32_sched=sched)
else:
    with tempfile.TemporaryDirectory() as d:
        for sub in ("include", "sac_maritime_ast_amd/csrc"):
            os.makedirs(os.path.join(d, sub), exist_ok=True)
            names = subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", f"{rev}:{sub}"], check=True,
                                   capture_output=True, text=True).stdout.split()
            for n in names:
                with open(os.path.join(d, sub, n), "wb") as f:
                    f.write(subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{sub}/{n}"], check=True,
                                           capture_output=True).stdout)
        g.ROOT, g.PKG = d, os.path.join(d, "sac_maritime_ast_amd")
        g.SOURCES = [os.path.join(g.PKG, "csrc", "sit_kernels.hip"), os.path.join(g.PKG, "csrc", "sit_steps_f32.hip")]
        g.compile_library(out, rest, f32, f32_sched=sched)
print("built", out)
