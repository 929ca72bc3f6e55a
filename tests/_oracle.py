"""ctypes wrapper of oracle/libmsoracle.so — the CPU restatement (checker only).

Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "libmsoracle.so")

PLUGINS_NU_NN, PLUGINS_NU_NRF_NN_LA, PLUGINS_NU_NN_NA, PLUGINS_NU_TT_NN = 0, 1, 2, 3
MODE_BATCHED, MODE_SEQUENTIAL = 0, 1


class msor_nodes(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32)] + [
        (f, ctypes.c_void_p)
        for f in (
            "flags",
            "digit",
            "allowed_pods",
            "pod_count",
            "alloc_cpu",
            "alloc_mem",
            "req_cpu",
            "req_mem",
            "nz_cpu",
            "nz_mem",
            "zone",
            "taints",
            "label2",
        )
    ]


class msor_pods(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32)] + [
        (f, ctypes.c_void_p)
        for f in ("ordinal", "digit", "tol", "req_cpu", "req_mem", "nz_cpu", "nz_mem", "pref_zone", "pref_weight",
                  "tol_hard", "tol_soft")
    ]


_LIB = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(ORACLE_LIB):
            build()
        L = ctypes.CDLL(ORACLE_LIB)
        L.msor_fmix32.restype = ctypes.c_uint32
        L.msor_fmix32.argtypes = [ctypes.c_uint32]
        L.msor_h32.restype = ctypes.c_uint32
        L.msor_h32.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
        L.msor_key.restype = ctypes.c_uint64
        L.msor_key.argtypes = [ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint32]
        L.msor_least_requested.restype = ctypes.c_int64
        L.msor_least_requested.argtypes = [ctypes.c_int64, ctypes.c_int64]
        L.msor_schedule.restype = ctypes.c_int
        L.msor_schedule.argtypes = [
            ctypes.POINTER(msor_nodes),
            ctypes.POINTER(msor_pods),
            ctypes.c_int,
            ctypes.c_int,
            ctypes.c_uint64,
            ctypes.c_uint32,
        ] + [ctypes.c_void_p] * 5
        L.msor_schedule_nunn_omp.restype = ctypes.c_int
        L.msor_schedule_nunn_omp.argtypes = [
            ctypes.POINTER(msor_nodes),
            ctypes.POINTER(msor_pods),
            ctypes.c_uint64,
            ctypes.c_uint32,
            ctypes.c_int,
        ] + [ctypes.c_void_p] * 5
        L.msor_schedule_na.restype = ctypes.c_int
        L.msor_schedule_na.argtypes = [
            ctypes.POINTER(msor_nodes),
            ctypes.POINTER(msor_pods),
            ctypes.c_int64,
            ctypes.c_int64,
            ctypes.c_int,
            ctypes.c_uint64,
            ctypes.c_uint32,
        ] + [ctypes.c_void_p] * 5
        L.msor_schedule_tt.restype = ctypes.c_int
        L.msor_schedule_tt.argtypes = [
            ctypes.POINTER(msor_nodes),
            ctypes.POINTER(msor_pods),
            ctypes.c_int,
            ctypes.c_uint64,
            ctypes.c_uint32,
        ] + [ctypes.c_void_p] * 5
        L.msor_schedule_nam.restype = ctypes.c_int
        L.msor_schedule_nam.argtypes = [
            ctypes.POINTER(msor_nodes), ctypes.POINTER(msor_pods), ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int64, ctypes.c_int64,
            ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ]
        L.msor_schedule_nam_ext.restype = ctypes.c_int
        L.msor_schedule_nam_ext.argtypes = L.msor_schedule_nam.argtypes
        L.msor_nam_inloop.restype = ctypes.c_int
        L.msor_nam_inloop.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
        L.msor_tt_inloop.restype = ctypes.c_int
        L.msor_tt_inloop.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
        L.msor_default_normalize.restype = None
        L.msor_default_normalize.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32]
        L.msor_schedule_nunn_names.restype = ctypes.c_int
        L.msor_schedule_nunn_names.argtypes = [
            ctypes.POINTER(ctypes.c_char_p),
            ctypes.c_void_p,
            ctypes.c_uint32,
            ctypes.POINTER(ctypes.c_char_p),
            ctypes.c_void_p,
            ctypes.c_void_p,
            ctypes.c_uint32,
            ctypes.c_uint64,
        ] + [ctypes.c_void_p] * 4
        _LIB = L
    return _LIB


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _col(a, dtype):
    # always a private copy: a field view of a 1-row array is already contiguous
    # and ascontiguousarray would hand the oracle the caller's memory
    return np.array(a, dtype=dtype, copy=True, order="C")


def _node_view(recs):
    """Round-3 fixtures store the node records with `_pad1` where `taints` now
    sits (same bytes, always 0 there): read them as the current layout."""
    recs = np.asarray(recs)
    if recs.dtype.names and "taints" not in recs.dtype.names and recs.dtype.itemsize == 64:
        from minisched_amd import _lib

        recs = np.ascontiguousarray(recs).view(_lib.NODE_REC)
    return recs


class NodeCols:
    """SoA copy of node records (the oracle mutates resource columns in place)."""

    def __init__(self, recs):
        recs = _node_view(recs)
        self.flags = _col(np.where(recs["allowed_pods"] < 0, 0x80, 0) | (recs["unschedulable"] & 1), np.uint8)
        self.digit = _col(np.where(recs["name_digit"] <= 9, recs["name_digit"], 0xFF), np.uint8)
        self.allowed_pods = _col(recs["allowed_pods"], np.int32)
        self.pod_count = _col(recs["pod_count"], np.int32)
        self.alloc_cpu = _col(recs["alloc_milli_cpu"], np.int64)
        self.alloc_mem = _col(recs["alloc_memory"], np.int64)
        self.req_cpu = _col(recs["req_milli_cpu"], np.int64)
        self.req_mem = _col(recs["req_memory"], np.int64)
        self.nz_cpu = _col(recs["nonzero_milli_cpu"], np.int64)
        self.nz_mem = _col(recs["nonzero_memory"], np.int64)
        self.zone = _col(recs["zone"], np.uint8)
        self.taints = _col(recs["taints"], np.uint32)
        self.label2 = _col(recs["label2"], np.uint8)

    def struct(self):
        return msor_nodes(
            len(self.flags),
            *[
                _p(getattr(self, f))
                for f in (
                    "flags",
                    "digit",
                    "allowed_pods",
                    "pod_count",
                    "alloc_cpu",
                    "alloc_mem",
                    "req_cpu",
                    "req_mem",
                    "nz_cpu",
                    "nz_mem",
                    "zone",
                    "taints",
                    "label2",
                )
            ],
        )


def _pod_cols(pods):
    cols = dict(
        ordinal=_col(pods["ordinal"], np.uint32),
        digit=_col(pods["name_digit"], np.int8),
        tol=_col(pods["tolerates_unschedulable"], np.uint8),
        req_cpu=_col(pods["req_milli_cpu"], np.int64),
        req_mem=_col(pods["req_memory"], np.int64),
        nz_cpu=_col(pods["nonzero_milli_cpu"], np.int64),
        nz_mem=_col(pods["nonzero_memory"], np.int64),
        pref_zone=_col(pods["pref_zone"], np.uint8),
        pref_weight=_col(pods["pref_weight"], np.uint8),
        # (NU_TT_NN: the same two bytes carry the tolerated taint ids, minisched_gpu.h)
        tol_hard=_col(pods["pref_zone"], np.uint8),
        tol_soft=_col(pods["pref_weight"], np.uint8),
    )
    st = msor_pods(len(pods), *[_p(cols[k]) for k in ("ordinal", "digit", "tol", "req_cpu", "req_mem", "nz_cpu", "nz_mem",
                                                      "pref_zone", "pref_weight", "tol_hard", "tol_soft")])
    return cols, st


def _outs(n):
    return dict(
        node=np.empty(n, np.int32),
        score=np.empty(n, np.int64),
        code=np.empty(n, np.int32),
        mask=np.empty(n, np.uint32),
        key=np.empty(n, np.uint64),
    )


def schedule(node_recs, pods, plugin_set=PLUGINS_NU_NN, mode=MODE_BATCHED, seed=1, node_base=0, cols=None):
    """Runs the oracle; returns dict of outputs (+ 'cols', the node columns after)."""
    L = lib()
    cols = cols if cols is not None else NodeCols(node_recs)
    nst = cols.struct()
    pc, pst = _pod_cols(pods)
    o = _outs(len(pods))
    rc = L.msor_schedule(
        ctypes.byref(nst), ctypes.byref(pst), plugin_set, mode, seed, node_base,
        _p(o["node"]), _p(o["score"]), _p(o["code"]), _p(o["mask"]), _p(o["key"]),
    )
    assert rc == 0, "oracle rejected its arguments"
    o["cols"] = cols
    return o


def schedule_na(node_recs, pods, weights=(1, 1), literal=True, seed=1, node_base=0):
    """MSOR_PLUGINS_NU_NN_NA (batched): literal=True runs RunScorePlugins' in-loop
    NormalizeScore as written (O(F^2) per pod), False its closed form."""
    L = lib()
    cols = NodeCols(node_recs)
    nst = cols.struct()
    pc, pst = _pod_cols(pods)
    o = _outs(len(pods))
    rc = L.msor_schedule_na(
        ctypes.byref(nst), ctypes.byref(pst), int(weights[0]), int(weights[1]), 1 if literal else 0, seed, node_base,
        _p(o["node"]), _p(o["score"]), _p(o["code"]), _p(o["mask"]), _p(o["key"]),
    )
    assert rc == 0, "oracle rejected its arguments"
    return o


def schedule_nam(node_recs, pods, term_sets, weights=(1, 1), literal=True, seed=1, node_base=0):
    """MSOR_PLUGINS_NU_NN_NAM (batched): several preferred terms per pod (term set
    id = pref_zone | pref_weight << 8, term_sets uint8 (n, 16)); literal=True runs
    RunScorePlugins' in-loop NormalizeScore as written (O(F^2) per pod)."""
    L = lib()
    cols = NodeCols(node_recs)
    nst = cols.struct()
    pc, pst = _pod_cols(pods)
    ts = np.ascontiguousarray(np.asarray(term_sets, dtype=np.uint8).reshape(-1, 16))
    o = _outs(len(pods))
    rc = L.msor_schedule_nam(
        ctypes.byref(nst), ctypes.byref(pst), ts.ctypes.data if len(ts) else None, len(ts), int(weights[0]),
        int(weights[1]), 1 if literal else 0, seed, node_base,
        _p(o["node"]), _p(o["score"]), _p(o["code"]), _p(o["mask"]), _p(o["key"]),
    )
    assert rc == 0, "oracle rejected its arguments"
    return o


def schedule_nam_ext(node_recs, pods, term_sets_ext, weights=(1, 1), literal=True, seed=1, node_base=0):
    """msor_schedule_nam_ext: the same with general term sets (uint8 (n, 272)
    ms_nam_term_set_ext records, _lib.nam_term_sets_ext_array)."""
    L = lib()
    cols = NodeCols(node_recs)
    nst = cols.struct()
    pc, pst = _pod_cols(pods)
    ts = np.ascontiguousarray(np.asarray(term_sets_ext, dtype=np.uint8).reshape(-1, 272))
    o = _outs(len(pods))
    rc = L.msor_schedule_nam_ext(
        ctypes.byref(nst), ctypes.byref(pst), ts.ctypes.data if len(ts) else None, len(ts), int(weights[0]),
        int(weights[1]), 1 if literal else 0, seed, node_base,
        _p(o["node"]), _p(o["score"]), _p(o["code"]), _p(o["mask"]), _p(o["key"]),
    )
    assert rc == 0, "oracle rejected its arguments"
    return o


def nam_inloop(raw, literal=True):
    """msor_nam_inloop: the reverse=false in-loop hook on one raw-score list."""
    r = np.ascontiguousarray(raw, dtype=np.int64)
    out = np.zeros(len(r), dtype=np.int64)
    assert lib().msor_nam_inloop(_p(r), len(r), 1 if literal else 0, _p(out)) == 0
    return out


def schedule_tt(node_recs, pods, literal=True, seed=1, node_base=0):
    """MSOR_PLUGINS_NU_TT_NN (batched): literal=True runs RunScorePlugins' in-loop
    reverse NormalizeScore as written (O(F^2) per pod), False its closed form."""
    L = lib()
    cols = NodeCols(node_recs)
    nst = cols.struct()
    pc, pst = _pod_cols(pods)
    o = _outs(len(pods))
    rc = L.msor_schedule_tt(
        ctypes.byref(nst), ctypes.byref(pst), 1 if literal else 0, seed, node_base,
        _p(o["node"]), _p(o["score"]), _p(o["code"]), _p(o["mask"]), _p(o["key"]),
    )
    assert rc == 0, "oracle rejected its arguments"
    return o


def tt_inloop(counts, literal=True):
    """The TaintToleration list after the in-loop reverse normalise hook."""
    c = np.ascontiguousarray(counts, dtype=np.int64)
    out = np.zeros(max(1, len(c)), dtype=np.int64)
    assert lib().msor_tt_inloop(_p(c), len(c), 1 if literal else 0, _p(out)) == 0
    return out[: len(c)]


def default_normalize(scores, max_priority=100, reverse=False):
    a = np.ascontiguousarray(scores, dtype=np.int64).copy()
    lib().msor_default_normalize(max_priority, 1 if reverse else 0, _p(a), len(a))
    return a


def schedule_batched_commit(node_recs, pods, plugin_set, seed=1, node_base=0):
    """Batched semantics of the engine: decide every pod on the same state,
    then commit NodeInfo.AddPod for every SUCCESS (minisched_gpu.h MS_MODE_BATCHED)."""
    o = schedule(node_recs, pods, plugin_set, MODE_BATCHED, seed, node_base)
    cols = o["cols"]
    for j in np.nonzero(o["code"] == 0)[0]:
        i = int(o["node"][j]) - node_base
        cols.pod_count[i] += 1
        cols.req_cpu[i] += pods["req_milli_cpu"][j]
        cols.req_mem[i] += pods["req_memory"][j]
        cols.nz_cpu[i] += pods["nonzero_milli_cpu"][j]
        cols.nz_mem[i] += pods["nonzero_memory"][j]
    return o


def schedule_nunn_omp(node_recs, pods, seed=1, node_base=0, threads=0):
    L = lib()
    cols = NodeCols(node_recs)
    nst = cols.struct()
    pc, pst = _pod_cols(pods)
    o = _outs(len(pods))
    rc = L.msor_schedule_nunn_omp(
        ctypes.byref(nst), ctypes.byref(pst), seed, node_base, threads,
        _p(o["node"]), _p(o["score"]), _p(o["code"]), _p(o["mask"]), _p(o["key"]),
    )
    assert rc == 0
    return o


def schedule_nunn_names(node_names, node_flags, pod_names, pod_tol, pod_ordinal, seed=1):
    L = lib()
    nn = (ctypes.c_char_p * len(node_names))(*[s.encode() for s in node_names])
    pn = (ctypes.c_char_p * len(pod_names))(*[s.encode() for s in pod_names])
    nf = np.ascontiguousarray(node_flags, dtype=np.uint8)
    pt = np.ascontiguousarray(pod_tol, dtype=np.uint8)
    po = np.ascontiguousarray(pod_ordinal, dtype=np.uint32)
    n = len(pod_names)
    o = dict(node=np.empty(n, np.int32), score=np.empty(n, np.int64), code=np.empty(n, np.int32), mask=np.empty(n, np.uint32))
    rc = L.msor_schedule_nunn_names(
        nn, _p(nf), len(node_names), pn, _p(pt), _p(po), n, seed,
        _p(o["node"]), _p(o["score"]), _p(o["code"]), _p(o["mask"]),
    )
    assert rc == 0
    return o
