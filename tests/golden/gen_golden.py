#!/usr/bin/env python3
"""Generates tests/golden/*.npz — frozen oracle outputs on small synthetic clusters.

The Go reference cannot run here, so these fixtures are the
oracle's own outputs: they pin the oracle and the GPU path against drift, not
against the reference. Inputs come from minisched_amd.synth with deliberate
edge cases (non-digit names, tolerating pods, tombstones, pre-loaded nodes).

  python tests/golden/gen_golden.py      # rewrites the fixtures
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mini-kube-scheduler_amd"))
sys.path.insert(0, os.path.dirname(HERE))

N_NODES, N_PODS = 64, 256


def make_inputs(plugin_set, seed):
    from minisched_amd import synth

    res = plugin_set == 1
    nr = synth.nodes(N_NODES, seed=seed, resources=res)
    pr = synth.pods(N_PODS, seed=seed, resources=res)
    nr["name_digit"][5::17] = 0xFF  # nodes whose names end in a letter
    nr["allowed_pods"][3::23] = -1  # tombstones (absent from the LIST)
    pr["name_digit"][7::31] = -1  # pods whose names end in a letter -> Error when F > 0
    pr["tolerates_unschedulable"][::9] = 1
    if res:
        nr["req_milli_cpu"] = nr["alloc_milli_cpu"] // 3
        nr["nonzero_milli_cpu"] = nr["req_milli_cpu"]
        nr["pod_count"][::11] = 109
        pr["req_milli_cpu"][::37] = 10**6  # fits nowhere -> FitError{NodeResourcesFit (+NU)}
    if seed == 3:
        nr["unschedulable"] = 1  # only tolerating pods fit -> FitError{NodeUnschedulable}
    return nr, pr


def cases():
    for plugin_set in (0, 1):
        for mode in (0, 1):
            for seed in (1, 2, 3):
                yield plugin_set, mode, seed


def name(plugin_set, mode, seed):
    return f"{'nunn' if plugin_set == 0 else 'full'}_{'batched' if mode == 0 else 'seq'}_{N_NODES}x{N_PODS}_seed{seed}.npz"


def main():
    import _oracle

    for plugin_set, mode, seed in cases():
        nr, pr = make_inputs(plugin_set, seed)
        if mode == 0:
            o = _oracle.schedule_batched_commit(nr, pr, plugin_set, seed=seed)
        else:
            o = _oracle.schedule(nr, pr, plugin_set=plugin_set, mode=1, seed=seed)
        c = o["cols"]
        np.savez(
            os.path.join(HERE, name(plugin_set, mode, seed)),
            nodes=nr,
            pods=pr,
            node=o["node"],
            score=o["score"],
            code=o["code"],
            mask=o["mask"],
            key=o["key"],
            after_pod_count=c.pod_count,
            after_req_cpu=c.req_cpu,
            after_req_mem=c.req_mem,
            after_nz_cpu=c.nz_cpu,
            after_nz_mem=c.nz_mem,
        )
        print("wrote", name(plugin_set, mode, seed))


if __name__ == "__main__":
    main()
