"""C++ host mirror (mini-kube-scheduler_amd/csrc/host) and sanitizer drivers.

The host mirror restates minisched's queue, plugin registry, event handlers
and ErrorFunc in C++ (the reference is Go; no Go toolchain here) and calls
the GPU through the C ABI. CPU mode covers queue/event/encoder semantics;
GPU mode replays the README scenario (sched.go:70-140) end to end.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mini-kube-scheduler_amd")
HOST_TEST = os.path.join(PKG, "bin", "ms_host_test")


def _ensure(target, path):
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", PKG, target], check=True)
    return path


def _run(args, env=None):
    out = subprocess.run(args, capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    return out.stdout


def test_host_mirror_cpu():
    out = _run([_ensure("host", HOST_TEST), "cpu"])
    assert "0 failed" in out


def test_host_mirror_cpu_asan():
    exe = _ensure("host-asan", os.path.join(PKG, "bin", "ms_host_test_asan"))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="halt_on_error=1")
    assert "0 failed" in _run([exe, "cpu"], env=env)


def test_oracle_asan():
    exe = os.path.join(ROOT, "oracle", "test_oracle_asan")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan-test"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1")
    assert _run([exe], env=env).strip().endswith("ok")


@pytest.mark.gpu
def test_host_mirror_gpu():
    out = _run([_ensure("host", HOST_TEST), "gpu"])
    assert "0 failed" in out, out


@pytest.mark.gpu
@pytest.mark.parametrize("plugin_set,n_nodes,n_pods,shuffle", [(1, 300, 1500, False), (0, 2000, 800, False),
                                                               (1, 300, 1500, True), (0, 2000, 800, True)])
def test_host_mirror_replay_matches_oracle(oracle, tmp_path, plugin_set, n_nodes, n_pods, shuffle):
    # the host mirror checked against the oracle, not against itself.
    # v1 objects go through the informer handlers, the queue (FIFO), the encoders, ScheduleOne,
    # the binder and ErrorFunc; every cycle's outcome must equal the sequential oracle's
    # for the same cluster, with pod ordinals in queue order and node ordinals from the
    # digit-aligned allocator (encode.DigitOrdinals, the host mirror's OrdinalAllocator):
    # in Add order node{i} gets ordinal i; shuffled, the Add order and the names differ and
    # some names end in a letter
    import numpy as np

    from minisched_amd import encode, synth

    seed = 17 + plugin_set
    nr = synth.nodes(n_nodes, seed=seed, resources=True)
    pr = synth.pods(n_pods, seed=seed, resources=True)
    pr["tolerates_unschedulable"][::9] = 1
    names = [f"pod{j}" if j % 37 else f"pod{j}x" for j in range(n_pods)]  # some names end in a letter
    pr["name_digit"] = [int(n[-1]) if n[-1].isdigit() else -1 for n in names]
    order = np.random.default_rng(seed).permutation(n_nodes) if shuffle else np.arange(n_nodes)
    node_names = [f"node{i}" if not shuffle or i % 23 else f"node{i}z" for i in range(n_nodes)]
    alloc = encode.DigitOrdinals(n_nodes)
    ords = np.zeros(n_nodes, dtype=np.int64)
    for i in order:
        ords[i] = alloc.allocate(encode.name_digit(node_names[i]))
    lines = []
    for i in order:
        lines.append(f"N {node_names[i]} {int(nr['unschedulable'][i])} {int(nr['alloc_milli_cpu'][i])} "
                     f"{int(nr['alloc_memory'][i])} {int(nr['allowed_pods'][i])}")
    # some pods also request a resource the records cannot carry (a GPU-only
    # pod among them); under NodeResourcesFit their cycle is a plain Error and they bind nothing
    extra = {j: ("amd.com/gpu=1" if j % 2 else "ephemeral-storage=1073741824") for j in range(5, n_pods, 41)}
    for j in extra:
        if j % 4 == 1:
            pr["req_milli_cpu"][j] = pr["req_memory"][j] = 0  # only the extended resource
    for j in range(n_pods):
        none = pr["req_milli_cpu"][j] == 0 and pr["req_memory"][j] == 0
        cpu = -1 if none else int(pr["req_milli_cpu"][j])
        mem = -1 if none else int(pr["req_memory"][j])
        lines.append(f"P {names[j]} {cpu} {mem} {int(pr['tolerates_unschedulable'][j])} {extra.get(j, '-')}")
    cluster = tmp_path / "cluster.txt"
    cluster.write_text("\n".join(lines) + "\n")
    out = tmp_path / "out.txt"
    _run([_ensure("host", HOST_TEST), "replay", str(cluster), str(out), str(seed), str(plugin_set)])
    rows = [l.split() for l in out.read_text().splitlines()]
    assert [r[0] for r in rows] == names  # one cycle per pod, in queue order
    code = np.array([{1: 0, 2: 2, 3: 1}[int(r[1])] for r in rows])
    by_name = {n: i for i, n in enumerate(node_names)}
    node = np.array([-1 if r[2] == "-" else int(ords[by_name[r[2]]]) for r in rows])
    score = np.array([int(r[3]) for r in rows])
    mask = np.array([int(r[4]) for r in rows])
    if plugin_set == 0:  # NU+NN reads no resources: the oracle's records need none
        nr["alloc_milli_cpu"] = nr["alloc_memory"] = 0
    nr["name_digit"] = [max(encode.name_digit(n), -1) & 0xFF for n in node_names]
    table = np.zeros(n_nodes, dtype=nr.dtype)  # the oracle's records at the allocated ordinals
    table[ords] = nr
    # NU+NN reads no resources: every pod is scheduled; NodeResourcesFit refuses the extra ones
    # (Error, no node, no mask) and the others equal the oracle's queue without them (same ordinals)
    keep = np.ones(n_pods, dtype=bool)
    if plugin_set == 1:
        keep[list(extra)] = False
        assert (code[~keep] == 1).all() and (node[~keep] == -1).all() and (mask[~keep] == 0).all()
    o = oracle.schedule(table, pr[keep], plugin_set=plugin_set, mode=1, seed=seed)
    code, node, score, mask = code[keep], node[keep], score[keep], mask[keep]
    assert np.array_equal(code, o["code"])
    assert np.array_equal(node, o["node"])
    assert np.array_equal(score, o["score"])
    assert np.array_equal(mask, o["mask"])
    if plugin_set == 1:
        assert (o["code"] == 2).sum() > 0 and (o["code"] == 1).sum() > 0


def test_copy_pool_tsan(tmp_path):
    # the host-copy helper threads of ms_schedule_batch(_compact) (csrc/ms_copy_pool.h)
    exe = str(tmp_path / "test_copy_pool")
    src = os.path.join(ROOT, "tests", "cpp", "test_copy_pool.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread",
                    "-I", os.path.join(PKG, "csrc"), src, "-o", exe], check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    assert "0 failed" in _run([exe], env=env)
