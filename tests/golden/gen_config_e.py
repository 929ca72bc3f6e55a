#!/usr/bin/env python3
"""Generates tests/golden/config_e_full_seed1.npz — the oracle's exact sequential
outputs for BASELINE config E at its full size: 50k nodes x 200k pods,
NU + NRF + NN + LA, queue order with assume-on-select.

The single-thread oracle needs ~2-3 minutes for this, too long for a GPU test,
so the GPU test compares against this committed fixture (and against the
after-bind node table the fixture implies). Inputs are re-generated from
minisched_amd.synth (seed 1), so only outputs are stored, plus a digest of the
oracle's after-table columns that the test recomputes from the placements.

  python tests/golden/gen_config_e.py      # rewrites the fixture (~3 min)
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))
sys.path.insert(0, os.path.dirname(HERE))

N_NODES, N_PODS, SEED = 50_000, 200_000, 1


def table_digest(pod_count, req_cpu, req_mem, nz_cpu, nz_mem):
    h = hashlib.sha256()
    for a in (pod_count, req_cpu, req_mem, nz_cpu, nz_mem):
        h.update(np.ascontiguousarray(a, dtype=np.int64).tobytes())
    return h.hexdigest()


def main():
    import _oracle
    from minisched_amd import synth

    nr = synth.nodes(N_NODES, seed=SEED, resources=True)
    pr = synth.pods(N_PODS, seed=SEED, resources=True)
    t0 = time.time()
    o = _oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=SEED)
    dt = time.time() - t0
    c = o["cols"]
    np.savez_compressed(
        os.path.join(HERE, "config_e_full_seed1.npz"),
        node=o["node"].astype(np.int32),
        code=o["code"].astype(np.int8),
        score=o["score"].astype(np.int16),
        mask=o["mask"].astype(np.uint8),
        table_sha256=np.array(table_digest(c.pod_count, c.req_cpu, c.req_mem, c.nz_cpu, c.nz_mem)),
    )
    print(f"wrote config_e_full_seed1.npz ({dt:.0f} s oracle): {(o['code'] == 0).sum()} placed, "
          f"{(o['code'] == 2).sum()} FitError, {(o['code'] == 1).sum()} Error")


if __name__ == "__main__":
    main()
