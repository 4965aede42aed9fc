#!/usr/bin/env python3
"""Commit the jittered starts of the benchmark scenario for N = 4096 envs.

The jitter (start position +-100 m, heading +-0.05 rad, per ship) is this repo's own synthetic
input, not a reference output: it is drawn per global env id with splitmix64 (a pure function of
(seed, env id), so GPU shards reproduce one large run) instead of SURVEY's
numpy.random.default_rng(25450) stream, which depends on the population size.  The fixture pins
the values the benches and parity tests use.

    python tests/golden/make_scenario_fixture.py       # writes tests/golden/scenario_jitter_4096.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from sac_maritime_ast_amd.scenario import make_scenario  # noqa: E402

sc = make_scenario(4096, seed=25450)
np.savez_compressed(os.path.join(HERE, "scenario_jitter_4096.npz"), seed=np.int64(25450),
                    start_north=sc.init[:, :, 0], start_east=sc.init[:, :, 1], start_yaw=sc.init[:, :, 2])
