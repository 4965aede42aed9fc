#!/usr/bin/env python3
"""Run the debug-variant workload of tests/test_gpu_debug.py against each given library (bounds-checked
builds of other revisions: tools/build_variant.py <name> --rev <rev> -DSIT_DEBUG) and print its flags."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from test_gpu_debug import WORKLOAD  # noqa: E402

for lib in sys.argv[1:]:
    p = subprocess.run([sys.executable, "-c", WORKLOAD, ROOT], env=dict(os.environ, SIT_LIBRARY=lib),
                       capture_output=True, text=True, timeout=240)
    print(lib, p.returncode, p.stdout.strip().splitlines()[-1] if p.stdout.strip() else p.stderr[-500:], flush=True)
