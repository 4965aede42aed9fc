"""Register / LDS / spill report of the gfx950 kernels in a built library, from the code objects'
metadata notes (no GPU needed): every offload bundle in the library's .hip_fatbin section is unbundled
(offload-bundle header parsed directly) and its AMDGPU metadata read with llvm-readelf --notes.

    python tools/kernel_resources.py [lib.so] [name-filter]
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib: str) -> list[bytes]:
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(d, "x")],
                       check=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        out = []
        for s in starts:   # bundle: magic, u64 entries, then (u64 offset, u64 size, u64 triple length, triple)
            p = s + len(MAGIC)
            n = struct.unpack_from("<Q", data, p)[0]
            p += 8
            for _ in range(n):
                off, size, tl = struct.unpack_from("<QQQ", data, p)
                p += 24
                triple = data[p:p + tl].decode()
                p += tl
                if "amdgcn" in triple and size:
                    out.append(data[s + off:s + off + size])
        return out


def kernels(lib: str) -> list[dict]:
    res = []
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".o") as f:
            f.write(co)
            f.flush()
            txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f.name], capture_output=True, text=True).stdout
        cur = None
        for line in txt.splitlines():
            m = re.match(r"\s*-?\s*\.(\w+):\s+(.*)$", line)
            if not m:
                continue
            k, v = m.group(1), m.group(2).strip()
            if k == "args":
                continue
            if k == "agpr_count":     # first key of a kernel record in the notes
                cur = {}
                res.append(cur)
            if cur is not None and k in ("agpr_count", "name", "vgpr_count", "sgpr_count", "vgpr_spill_count",
                                         "sgpr_spill_count", "group_segment_fixed_size",
                                         "private_segment_fixed_size", "max_flat_workgroup_size"):
                cur[k] = v
    return [k for k in res if "name" in k]


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "sac_maritime_ast_amd", "libsit.so")
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    for k in kernels(lib):
        name = subprocess.run(["c++filt"], input=k["name"], capture_output=True, text=True).stdout.strip()
        if flt and flt not in name:
            continue
        print(f"{k.get('vgpr_count'):>4} vgpr {k.get('agpr_count'):>3} agpr {k.get('sgpr_count'):>4} sgpr "
              f"spill v{k.get('vgpr_spill_count')} s{k.get('sgpr_spill_count')} "
              f"lds {k.get('group_segment_fixed_size'):>6} scratch {k.get('private_segment_fixed_size'):>4}  {name[:150]}")


if __name__ == "__main__":
    main()
