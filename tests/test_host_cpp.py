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
