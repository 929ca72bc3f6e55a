"""The C-ABI library loads and exports exactly what include/minisched_gpu.h declares.

CPU-only: no compute call is made without a GPU.
"""
import ctypes
import os
import re
import subprocess

import pytest

from minisched_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "minisched_gpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(ms_\w+)\s*\(", src, flags=re.M)))


def test_header_and_binding_agree():
    names = declared_functions()
    assert len(names) >= 15
    assert sorted(_lib.SIGNATURES) == names


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(re.findall(r" T (ms_\w+)", out.stdout))
    assert exported == set(declared_functions())


def test_library_is_gfx950_code_object():
    out = subprocess.run(
        ["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", _lib.LIB_PATH],
        capture_output=True,
        text=True,
    )
    text = out.stdout + out.stderr
    assert "gfx950" in text


def test_struct_sizes_match_header():
    assert _lib.NODE_REC.itemsize == 64
    assert _lib.POD_REC.itemsize == 40
    assert _lib.RESULT.itemsize == 24
    assert ctypes.sizeof(_lib.ms_config) == 32
    assert ctypes.sizeof(_lib.ms_info) == 56
    assert ctypes.sizeof(_lib.ms_comm_id) == _lib.COMM_ID_BYTES == 128
    assert _lib.POD_COMPACT.itemsize == _lib.RESULT_COMPACT.itemsize == 8
    # ms_pod_compact is the first 8 bytes of ms_pod_rec
    from minisched_amd import synth

    pr = synth.pods(50, seed=3, zones=True)
    assert _lib.compact_pods(pr).tobytes() == b"".join(r.tobytes()[:8] for r in pr)


def test_library_links_rccl():
    # the node-sharded cycles run their collectives in-library (ms_comm.cpp)
    out = subprocess.run(["readelf", "-d", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "librccl.so" in out


def test_abi_version_and_no_device_error_path():
    lib = _lib.load()
    assert lib.ms_abi_version() == 7  # round 5: NAM, label2 (5); two-pass TT shard calls (6); round 6: ext term sets (7)
    if _lib.device_count() > 0:
        pytest.skip("a device is visible; the no-device path is exercised on CPU hosts")
    cfg = _lib.ms_config(0, 0, 16, 0, 64, (ctypes.c_uint16 * 2)(), 1)
    h = ctypes.c_void_p()
    rc = lib.ms_create(ctypes.byref(cfg), ctypes.byref(h))
    assert rc == _lib.MS_E_NODEV
    assert b"device" in lib.ms_last_error(None)
    # argument validation happens before any device work
    bad = _lib.ms_config(0, 7, 16, 0, 64, (ctypes.c_uint16 * 2)(), 1)
    assert lib.ms_create(ctypes.byref(bad), ctypes.byref(h)) == _lib.MS_E_INVAL
    assert lib.ms_create(None, ctypes.byref(h)) == _lib.MS_E_INVAL
    assert lib.ms_destroy(None) == _lib.MS_E_INVAL
    assert lib.ms_schedule_batch(None, 0, None, 0, None) == _lib.MS_E_INVAL


def test_engine_refuses_without_device():
    if _lib.device_count() > 0:
        pytest.skip("device visible")
    with pytest.raises(_lib.MSError) as e:
        _lib.Engine(max_nodes=8)
    assert e.value.code == _lib.MS_E_NODEV


def hip_runtimes_mapped():
    libs = set()
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 6 and "libamdhip64" in parts[-1]:
                libs.add(os.path.realpath(parts[-1]))
    return libs


def test_single_hip_runtime_per_process():
    # torch and libminisched_gpu.so must share one HIP runtime (see _lib.load)
    import torch  # noqa: F401

    _lib.load()
    assert len(hip_runtimes_mapped()) == 1, hip_runtimes_mapped()


def test_comm_id_create_on_host():
    # ms_comm_id_create (ncclGetUniqueId) needs no device: rank 0 makes the id, every
    # rank receives its 128 bytes out of band (sharded.init_comm broadcasts them)
    a, b = _lib.comm_id_create(), _lib.comm_id_create()
    assert len(a) == len(b) == _lib.COMM_ID_BYTES and a != b


def test_loopback_build_is_test_only():
    # `make comm-loopback`: the same ABI with ms_comm.cpp's RCCL calls replaced by an
    # in-process rendezvous (tests/test_gpu_loopback.py); it links no RCCL, and the
    # product library exports none of its symbols
    assert os.path.exists(_lib.LOOPBACK_LIB_PATH), "make -C mini-kube-scheduler_amd comm-loopback"
    dyn = subprocess.run(["readelf", "-d", _lib.LOOPBACK_LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "librccl.so" not in dyn
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LOOPBACK_LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert set(re.findall(r" T (ms_\w+)", out)) == set(declared_functions())
    assert "lb_ncclReduceScatter" in out and "lb_collectives_issued" in out
    prod = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                          check=True).stdout
    assert "lb_" not in prod
    und = subprocess.run(["nm", "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert "ncclReduceScatter" in und and "ncclAllGather" in und
