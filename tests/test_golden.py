"""Golden fixtures (tests/golden/*.npz, written by tests/golden/gen_golden.py).

CPU: the generator still reproduces the stored inputs and the oracle still
reproduces the stored outputs. GPU: the HIP path reproduces them through the
C ABI, including the node table after the binds.
"""
import glob
import json
import os

import numpy as np
import pytest

from minisched_amd import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(p for p in glob.glob(os.path.join(HERE, "golden", "*.npz")) if "x256_seed" in p)


def _meta(path):
    base = os.path.basename(path)
    plugin_set = 0 if base.startswith("nunn") else 1
    mode = 0 if "_batched_" in base else 1
    seed = int(base.split("seed")[1].split(".")[0])
    return plugin_set, mode, seed


def _load(path):
    return np.load(path, allow_pickle=False)


def test_fixture_set_is_complete():
    assert len(FIXTURES) == 12
    codes = np.concatenate([_load(p)["code"] for p in FIXTURES])
    # the fixtures exercise every outcome class
    assert {0, 1, 2} <= set(codes.tolist())
    masks = np.concatenate([_load(p)["mask"] for p in FIXTURES])
    assert {1, 2} <= set(masks.tolist())


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_generator_reproduces_inputs(path):
    import golden.gen_golden as gg

    f = _load(path)
    plugin_set, mode, seed = _meta(path)
    nr, pr = gg.make_inputs(plugin_set, seed)
    assert nr.tobytes() == f["nodes"].tobytes()
    assert pr.tobytes() == f["pods"].tobytes()


@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_oracle_reproduces_golden(oracle, path):
    f = _load(path)
    plugin_set, mode, seed = _meta(path)
    if mode == 0:
        o = oracle.schedule_batched_commit(f["nodes"], f["pods"], plugin_set, seed=seed)
    else:
        o = oracle.schedule(f["nodes"], f["pods"], plugin_set=plugin_set, mode=1, seed=seed)
    for k in ("node", "score", "code", "mask", "key"):
        assert np.array_equal(o[k], f[k]), k
    assert np.array_equal(o["cols"].pod_count, f["after_pod_count"])
    assert np.array_equal(o["cols"].req_cpu, f["after_req_cpu"])


def test_readme_scenario_fixture(oracle):
    kat = json.load(open(os.path.join(HERE, "golden", "readme_scenario.json")))
    from minisched_amd import synth

    first, node10, pod1 = synth.readme_scenario()
    o = oracle.schedule(first, pod1)
    got = dict(code=int(o["code"][0]), node=int(o["node"][0]), mask=int(o["mask"][0]))
    assert got == kat["before_node10"]
    o = oracle.schedule(np.concatenate([first, node10]), pod1)
    got = dict(code=int(o["code"][0]), node=int(o["node"][0]), mask=int(o["mask"][0]), score=int(o["score"][0]))
    assert got == kat["after_node10"]


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=os.path.basename)
def test_gpu_reproduces_golden(path):
    f = _load(path)
    plugin_set, mode, seed = _meta(path)
    nr = f["nodes"]
    present = np.nonzero(nr["allowed_pods"] >= 0)[0]
    with _lib.Engine(max_nodes=len(nr), plugin_set=plugin_set, seed=seed) as e:
        e.upsert(present, nr[present])
        r = e.schedule(f["pods"], mode)
        for a, b in (("node", "node"), ("code", "code"), ("score", "score"), ("plugin_mask", "mask")):
            assert np.array_equal(r[a], f[b]), a
        t = e.read(0, len(nr))
        assert np.array_equal(t["pod_count"][present], f["after_pod_count"][present])
        assert np.array_equal(t["req_milli_cpu"][present], f["after_req_cpu"][present])
        assert np.array_equal(t["nonzero_memory"][present], f["after_nz_mem"][present])


def test_config_e_fixture_consistent():
    # tests/golden/gen_config_e.py: the full-size config E outputs the GPU test compares
    # against; CPU-side sanity of the stored placements (the oracle needs minutes to redo them)
    from minisched_amd import synth

    fx = np.load(os.path.join(HERE, "golden", "config_e_full_seed1.npz"), allow_pickle=False)
    node, code, score, mask = fx["node"], fx["code"], fx["score"], fx["mask"]
    assert len(node) == 200_000
    placed = code == 0
    assert placed.sum() == 184_595 and (code == 2).sum() == 15_405
    assert np.all((node[placed] >= 0) & (node[placed] < 50_000)) and np.all(node[~placed] == -1)
    assert np.all(mask[placed] == 0) and np.all(mask[code == 2] != 0)
    # NodeNumber's 10 plus LeastAllocated in [0, 100]
    assert score.min() >= 0 and score.max() <= 110
    pr = synth.pods(200_000, seed=1, resources=True)
    nr = synth.nodes(50_000, seed=1, resources=True)
    # no node ever exceeds its allocatable with the placements applied in order
    cpu = np.bincount(node[placed], weights=pr["req_milli_cpu"][placed], minlength=50_000)
    mem = np.bincount(node[placed], weights=pr["req_memory"][placed].astype(np.float64), minlength=50_000)
    assert np.all(cpu <= nr["alloc_milli_cpu"]) and np.all(mem <= nr["alloc_memory"])
    assert np.all(np.bincount(node[placed], minlength=50_000) <= 110)
