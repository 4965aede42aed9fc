#!/usr/bin/env python3
"""Per-kernel register / occupancy report of libsit's two translation units (CPU only, no GPU).

    python3 tools/resource_report.py [out.json]

Compiles each TU for gfx950 device-only with the release flags of __graft_entry__.compile_library plus
-Rpass-analysis=kernel-resource-usage and collects, per step kernel instantiation, the compiler's VGPRs,
SGPRs, scratch, occupancy (waves per SIMD) and LDS bytes.  The register budget of the step kernel is a
design constraint (two waves per SIMD: <= 256 VGPRs less the granule)."""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

FIELDS = {"TotalSGPRs": "sgprs", "VGPRs": "vgprs", "AGPRs": "agprs", "ScratchSize [bytes/lane]": "scratch_bytes_per_lane",
          "Occupancy [waves/SIMD]": "waves_per_simd", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill",
          "LDS Size [bytes/block]": "lds_bytes"}


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


def report(src, flags):
    cmd = [g._hipcc(), "-O3", "-std=c++17", f"--offload-arch={g.ARCH}", "-fPIC", "-fno-hip-fp32-correctly-rounded-divide-sqrt",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(g.PKG, "csrc"), *flags,
           "-Rpass-analysis=kernel-resource-usage", "--offload-device-only", "-c", src, "-o", "/tmp/_sit_ru.o"]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp")
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-2000:])
    kernels, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        txt = m.group(1).strip()
        if txt.startswith("Function Name:"):
            cur = txt.split(":", 1)[1].strip()
            kernels[cur] = {}
        elif cur and ":" in txt:
            k, v = txt.rsplit(":", 1)
            if k.strip() in FIELDS:
                v = v.strip()
                kernels[cur][FIELDS[k.strip()]] = int(v) if v.lstrip("-").isdigit() else v
    names = list(kernels)
    return {d: kernels[n] for n, d in zip(names, demangle(names)) if "k_env_steps" in d or "k_policy" in d}


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r06_step_kernel_resources.json")
    f32_flags = ["-Xarch_device", "-ffast-math", "-Xarch_device", "-ffp-contract=fast-honor-pragmas", "-Wno-overriding-option",
                 *g.F32_SCHED]
    res = {"what": __doc__.split("\n\n")[0], "arch": g.ARCH,
           os.path.basename(g.SOURCES[1]): report(g.SOURCES[1], f32_flags),
           os.path.basename(g.SOURCES[0]): report(g.SOURCES[0], ["-DSIT_F32_TU"])}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for tu in list(res)[2:]:
        for k, v in res[tu].items():
            print(f"{tu:20s} {k[:90]:90s} vgpr {v.get('vgprs')} waves/SIMD {v.get('waves_per_simd')} scratch {v.get('scratch_bytes_per_lane')}")


if __name__ == "__main__":
    main()
