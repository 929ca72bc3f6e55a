"""Randomised parity: clusters and pod queues far from the synthetic configs.

Each case draws a cluster from its own seeded generator: digit layouts that
cycle, follow the ordinal (K1's fixed-slot form), are i.i.d. or use two digits
only (the K1 bit-scan path), nodes
without a name digit, unschedulable fractions up to 60 %, tiny pod caps,
capacities from 0 to 2^48 (the int64 LeastAllocated form above 2^41),
pre-existing Requested up to 1.5x Allocatable, tombstoned nodes; pods with
zero, default and oversized requests, non-digit names (the Score error) and
tolerations. The HIP path (through the C ABI) must equal the oracle pod by pod,
and after sequential binds the node table must equal the oracle's columns.
A failure names its case; the case index is the generator seed.
"""
import os

import numpy as np
import pytest

from minisched_amd import _lib
from minisched_amd._lib import MODE_BATCHED, MODE_SEQUENTIAL, NODE_REC, POD_REC, PLUGINS_NU_NN, PLUGINS_NU_NRF_NN_LA
from test_gpu_parity import assert_same, engine_with

pytestmark = pytest.mark.gpu

MiB, GiB = 1 << 20, 1 << 30


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    _lib.load()
    if _lib.device_count() == 0:
        pytest.fail("gpu test collected on a host without a visible device")


def rand_nodes(rng, n, resources, base=0):
    rec = np.zeros(n, dtype=NODE_REC)
    layout = rng.integers(0, 4)
    if layout == 0:
        d = np.arange(n) % 10
    elif layout == 1:
        d = rng.integers(0, 10, n)
    elif layout == 2:
        d = rng.choice(rng.integers(0, 10, 2), n)
    else:  # digit = ordinal mod 10 (the allocator's layout: K1's fixed-slot form)
        d = (base + np.arange(n)) % 10
    d = np.where(rng.random(n) < 0.05, 0xFF, d)
    rec["name_digit"] = d.astype(np.uint8)
    rec["unschedulable"] = (rng.random(n) < rng.random() * 0.6).astype(np.uint8)
    rec["allowed_pods"] = rng.choice([0, 1, 2, 3, 110, 110, 110, 110], n)
    if resources:
        cpu = np.array([0, 1, 250, 1000, 4000, 8000, 96_000, (1 << 41) - 1, 1 << 41, 1 << 45], dtype=np.int64)
        mem = np.array([0, 1, GiB, 8 * GiB, 16 * GiB, 1 << 41, 1 << 48], dtype=np.int64)
        # most clusters stay in the binary64 form's range; some draw every capacity
        wide = rng.random() < 0.4
        ci = rng.integers(0, len(cpu) if wide else 7, n)
        mi = rng.integers(0, len(mem) if wide else 5, n)
        rec["alloc_milli_cpu"] = cpu[ci]
        rec["alloc_memory"] = mem[mi]
        busy = rng.random(n) < 0.5
        frac = rng.random(n) * 1.5
        rec["req_milli_cpu"] = np.where(busy, (rec["alloc_milli_cpu"] * frac).astype(np.int64), 0)
        rec["req_memory"] = np.where(busy, (rec["alloc_memory"] * frac).astype(np.int64), 0)
        rec["nonzero_milli_cpu"] = rec["req_milli_cpu"] + np.where(busy & (rng.random(n) < 0.3), 100, 0)
        rec["nonzero_memory"] = rec["req_memory"] + np.where(busy & (rng.random(n) < 0.3), 200 * MiB, 0)
        rec["pod_count"] = np.minimum(rng.integers(0, 5, n), rec["allowed_pods"])
    return rec


def rand_pods(rng, n, resources, start=0):
    rec = np.zeros(n, dtype=POD_REC)
    rec["ordinal"] = np.arange(start, start + n, dtype=np.uint32)
    rec["name_digit"] = np.where(rng.random(n) < 0.05, -1, rng.integers(0, 10, n)).astype(np.int8)
    rec["tolerates_unschedulable"] = (rng.random(n) < rng.random() * 0.3).astype(np.uint8)
    if resources:
        kind = rng.integers(0, 10, n)
        cpu = np.where(kind == 0, 0, np.where(kind == 9, 1 << 42, 100 * rng.integers(1, 41, n)))
        mem = np.where(kind == 0, 0, np.where(kind == 9, 1 << 44, 128 * MiB * rng.integers(1, 33, n)))
        rec["req_milli_cpu"] = cpu
        rec["req_memory"] = mem
        rec["nonzero_milli_cpu"] = np.where(cpu == 0, 100, cpu)
        rec["nonzero_memory"] = np.where(mem == 0, 200 * MiB, mem)
    return rec


def tombstone(rng, e, cols, n):
    dead = np.nonzero(rng.random(n) < rng.random() * 0.3)[0]
    if len(dead):
        e.delete(dead)
        cols.flags[dead] |= 0x80
    return dead


@pytest.mark.parametrize("case", range(64))
def test_fuzz_resource_sequential(oracle, case):
    rng = np.random.default_rng(1000 + case)
    n, p = int(rng.integers(1, 4000)), int(rng.integers(1, 2500))
    nr, pr = rand_nodes(rng, n, True), rand_pods(rng, p, True)
    seed = int(rng.integers(0, 1 << 40))
    cols = oracle.NodeCols(nr)
    with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=seed) as e:
        tombstone(rng, e, cols, n)
        o = oracle.schedule(nr, pr, plugin_set=1, mode=1, seed=seed, cols=cols)
        assert_same(e.schedule(pr, MODE_SEQUENTIAL), o)
        t = e.read(0, n)
        live = (cols.flags & 0x80) == 0
        for k_dev, k_or in (("pod_count", "pod_count"), ("req_milli_cpu", "req_cpu"), ("req_memory", "req_mem"),
                            ("nonzero_milli_cpu", "nz_cpu"), ("nonzero_memory", "nz_mem")):
            assert np.array_equal(t[k_dev][live], getattr(cols, k_or)[live]), (case, k_dev)
        assert e.info()._pad == 0


@pytest.mark.parametrize("case", range(24))
def test_fuzz_resource_batched(oracle, case):
    rng = np.random.default_rng(2000 + case)
    n, p = int(rng.integers(1, 4000)), int(rng.integers(1, 2500))
    nr, pr = rand_nodes(rng, n, True), rand_pods(rng, p, True)
    seed = int(rng.integers(0, 1 << 40))
    cols = oracle.NodeCols(nr)
    with engine_with(nr, plugin_set=PLUGINS_NU_NRF_NN_LA, seed=seed) as e:
        tombstone(rng, e, cols, n)
        o = oracle.schedule(nr, pr, plugin_set=1, mode=0, seed=seed, cols=cols)
        assert_same(e.schedule(pr, MODE_BATCHED), o)


@pytest.mark.parametrize("case", range(int(os.environ.get("MINISCHED_FUZZ_NUNN", "48"))))  # (extended runs: more)
def test_fuzz_nunn(oracle, case):
    rng = np.random.default_rng(3000 + case)
    n, p = int(rng.integers(1, 40_000)), int(rng.integers(1, 3000))
    base = int(rng.integers(0, 1 << 19))
    nr, pr = rand_nodes(rng, n, False, base), rand_pods(rng, p, False)
    seed = int(rng.integers(0, 1 << 40))
    cols = oracle.NodeCols(nr)
    with engine_with(nr, seed=seed, node_base=base) as e:
        dead = np.nonzero(rng.random(n) < rng.random() * 0.3)[0]
        if len(dead):
            e.delete(base + dead)
            cols.flags[dead] |= 0x80
        o = oracle.schedule(nr, pr, plugin_set=0, mode=0, seed=seed, node_base=base, cols=cols)
        assert_same(e.schedule(pr, MODE_BATCHED), o)
        out = np.zeros(p, dtype=_lib.RESULT)
        out[:] = e.schedule(pr, MODE_BATCHED)  # idempotent outcomes on a stateless set
        assert_same(out, o)


@pytest.mark.parametrize("case", range(24))
def test_fuzz_na(oracle, case):
    rng = np.random.default_rng(4000 + case)
    n, p = int(rng.integers(1, 20_000)), int(rng.integers(1, 1500))
    nr, pr = rand_nodes(rng, n, False), rand_pods(rng, p, False)
    nr["zone"] = np.where(rng.random(n) < 0.1, 0, rng.integers(1, 9, n))
    pz = rng.random(p) < 0.7
    pr["pref_zone"] = np.where(pz, rng.integers(1, 9, p), 0)
    pr["pref_weight"] = np.where(pz, rng.integers(1, 101, p), 0)
    seed = int(rng.integers(0, 1 << 40))
    with engine_with(nr, plugin_set=_lib.PLUGINS_NU_NN_NA, seed=seed) as e:
        o = oracle.schedule_na(nr, pr, seed=seed, literal=False)
        assert_same(e.schedule(pr, MODE_BATCHED), o)
