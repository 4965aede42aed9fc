#!/usr/bin/env python3
"""Which SIMD each role of the two-wave kernel lands on (a -DSIT_DIAG_PLACE build, diagnostic only):

    tools/build_variant.py place -DSIT_DIAG_PLACE
    SIT_LIBRARY=build_diag/libsit_place.so python tools/diag_place.py

One C3-size launch (32 768 envs = 512 blocks of 4 waves); per SIMD, the roles of the waves resident on
it (HW_ID), counted by pair type: a D (dynamics) wave beside a P (predicates) wave is the intended
placement, two D or two P waves compete for the same issue slots."""
import collections
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sac_maritime_ast_amd import VecMultiShipRLEnv, _lib, make_scenario  # noqa: E402

n_env = 32768
lib = ctypes.CDLL(_lib.LIB_PATH)
env = VecMultiShipRLEnv(scenario=make_scenario(n_env, cap=48), precision=32, device="cuda:0")
env.reset()
env.init_step()
env.rollout(20, seed=25450)
torch.cuda.synchronize()
nw = 4 * ((n_env + 63) // 64)
buf = (ctypes.c_ulonglong * (4 * nw))()
assert lib.sit_diag_read_waves_f32(buf, nw) == 0
w = np.array(buf[:], dtype=np.uint64).reshape(nw, 4)
role, block, hw, xcc = w[:, 0].astype(int), w[:, 1].astype(int), (w[:, 3] & 0xffffffff).astype(np.int64), (w[:, 3] >> 32).astype(int)
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
per_simd = collections.defaultdict(list)
per_cu_blocks = collections.defaultdict(set)
block_simds = collections.defaultdict(set)
for i in range(nw):
    per_simd[(cu_key[i], simd[i])].append(int(role[i]))
    per_cu_blocks[cu_key[i]].add(int(block[i]))
    block_simds[int(block[i])].add(int(simd[i]))
kinds = collections.Counter()
for roles in per_simd.values():
    kinds["".join(sorted("D" if r < 2 else "P" for r in roles))] += 1
pairs = collections.Counter(tuple(sorted(b % 2 for b in bl)) for bl in per_cu_blocks.values())
gaps = collections.Counter(tuple(sorted(bl))[1] - tuple(sorted(bl))[0] if len(bl) == 2 else -1 for bl in per_cu_blocks.values())
print(json.dumps({"waves": nw, "cus": len(per_cu_blocks), "simds": len(per_simd),
                  "roles_per_simd": dict(kinds),
                  "blocks_per_cu": dict(collections.Counter(len(b) for b in per_cu_blocks.values())),
                  "block_parities_per_cu": {str(k): v for k, v in pairs.items()},
                  "block_index_gap_per_cu (top 5)": {str(k): v for k, v in gaps.most_common(5)},
                  "distinct_simds_per_block": dict(collections.Counter(len(s) for s in block_simds.values()))}, indent=1))
