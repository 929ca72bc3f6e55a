"""ctypes binding of libminisched_gpu.so (include/minisched_gpu.h).

This is the Python twin of the cgo shim described in INTEGRATION.md: plain
pointers and sizes, numpy structured arrays that match the C structs byte for
byte. There is no CPU fallback: if the HIP library is missing the import of
`load()` raises, and every compute call needs a gfx950 device.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MINISCHED_LIB selects another build of the same ABI (e.g. the MS_STAMPS
# diagnostic library); the default is the production library.
LIB_PATH = os.environ.get("MINISCHED_LIB") or os.path.join(HERE, "libminisched_gpu.so")
# TEST-ONLY build (`make comm-loopback`): ms_comm.cpp's RCCL calls replaced by an
# in-process rendezvous, so G contexts driven by G host threads form a world-G
# communicator on one GPU (tests/test_gpu_loopback.py). Never the product path.
LOOPBACK_LIB_PATH = os.path.join(HERE, "libminisched_gpu_loopback.so")

# ---- constants (minisched_gpu.h) -------------------------------------------
MS_OK = 0
MS_E_INVAL, MS_E_HIP, MS_E_RCCL, MS_E_OOM, MS_E_CAPACITY, MS_E_NODEV = -1, -2, -3, -4, -5, -6
PLUGINS_NU_NN = 0
PLUGINS_NU_NRF_NN_LA = 1
PLUGINS_NU_NN_NA = 2
PLUGINS_NU_TT_NN = 3
PLUGINS_NU_NN_NAM = 4
MODE_BATCHED = 0
MODE_SEQUENTIAL = 1
CODE_SUCCESS, CODE_ERROR, CODE_UNSCHEDULABLE = 0, 1, 2
MASK_NODE_UNSCHEDULABLE = 1
MASK_NODE_RESOURCES_FIT = 2
MASK_TAINT_TOLERATION = 4
MAX_ORDINAL = 0xFFFFD  # keys 0 / 1 are reserved (no feasible node)

ERRNAMES = {
    MS_E_INVAL: "MS_E_INVAL",
    MS_E_HIP: "MS_E_HIP",
    MS_E_RCCL: "MS_E_RCCL",
    MS_E_OOM: "MS_E_OOM",
    MS_E_CAPACITY: "MS_E_CAPACITY",
    MS_E_NODEV: "MS_E_NODEV",
}

# ---- record layouts --------------------------------------------------------
NODE_REC = np.dtype(
    [
        ("unschedulable", "u1"),
        ("name_digit", "u1"),
        ("zone", "u1"),
        ("label2", "u1"),  # second node label value id (MS_PLUGINS_NU_NN_NAM term key 1)
        ("allowed_pods", "<i4"),
        ("pod_count", "<i4"),
        ("taints", "<u4"),  # MS_PLUGINS_NU_TT_NN: bits 0-7 NoSchedule/NoExecute ids, 8-15 PreferNoSchedule
        ("alloc_milli_cpu", "<i8"),
        ("alloc_memory", "<i8"),
        ("req_milli_cpu", "<i8"),
        ("req_memory", "<i8"),
        ("nonzero_milli_cpu", "<i8"),
        ("nonzero_memory", "<i8"),
    ]
)
POD_REC = np.dtype(
    [
        ("ordinal", "<u4"),
        ("name_digit", "i1"),
        ("tolerates_unschedulable", "u1"),
        ("pref_zone", "u1"),
        ("pref_weight", "u1"),
        ("req_milli_cpu", "<i8"),
        ("req_memory", "<i8"),
        ("nonzero_milli_cpu", "<i8"),
        ("nonzero_memory", "<i8"),
    ]
)
RESULT = np.dtype(
    [("node", "<i4"), ("code", "<i4"), ("score", "<i8"), ("plugin_mask", "<u4"), ("_pad", "<u4")]
)
# compact records (ms_schedule_batch_compact; NU+NN / NodeAffinity sets): 8 B each way
POD_COMPACT = np.dtype([("ordinal", "<u4"), ("name_digit", "i1"), ("tolerates_unschedulable", "u1"),
                        ("pref_zone", "u1"), ("pref_weight", "u1")])
RESULT_COMPACT = np.dtype([("node", "<i4"), ("score", "<u2"), ("code", "u1"), ("plugin_mask", "u1")])
# ms_seq_cand: a shard's speculative candidate with the node's record (node-sharded sequential mode)
SEQ_CAND = np.dtype(
    [
        ("key", "<u8"),
        ("alloc_milli_cpu", "<i8"),
        ("alloc_memory", "<i8"),
        ("req_milli_cpu", "<i8"),
        ("req_memory", "<i8"),
        ("nonzero_milli_cpu", "<i8"),
        ("nonzero_memory", "<i8"),
        ("allowed_pods", "<i4"),
        ("pod_count", "<i4"),
        ("flags_digit", "<u4"),
        ("_pad", "<u4"),
    ]
)
SEQ_TOPK = 4
TT_SUMMARY_BYTES = 192  # MS_TT_SUMMARY_BYTES
TT_CENSUS_BYTES = 32  # MS_TT_CENSUS_BYTES
NAM_SEG_BYTES = 104  # MS_NAM_SEG_BYTES
NAM_TERMS = 4  # MS_NAM_TERMS


NAM_TERM_EXT_BYTES = 68  # ms_pref_term_ext
NAM_SET_EXT_BYTES = NAM_TERMS * NAM_TERM_EXT_BYTES  # ms_nam_term_set_ext
_ALL_IDS = (1 << 256) - 1


def nam_term_sets_ext_array(sets):
    """ms_nam_term_set_ext records (uint8 (n, 272)) from a list of term lists
    [(weight 0..100, zone id set, label2 id set), ...] (at most MS_NAM_TERMS
    each); an id set is a Python int whose bit v holds value id v (0..255; bit 0:
    the label is absent), e.g. encode.NamTerms builds them from requirements."""
    out = np.zeros((len(sets), NAM_SET_EXT_BYTES), dtype=np.uint8)
    for i, terms in enumerate(sets):
        if len(terms) > NAM_TERMS:
            raise ValueError(f"at most {NAM_TERMS} preferred terms per set")
        for k, (weight, zmask, lmask) in enumerate(terms):
            if not 0 <= weight <= 100 or not 0 <= zmask <= _ALL_IDS or not 0 <= lmask <= _ALL_IDS:
                raise ValueError("term: weight 0..100, id sets within 256 bits")
            b = k * NAM_TERM_EXT_BYTES
            out[i, b:b + 32] = np.frombuffer(int(zmask).to_bytes(32, "little"), dtype=np.uint8)
            out[i, b + 32:b + 64] = np.frombuffer(int(lmask).to_bytes(32, "little"), dtype=np.uint8)
            out[i, b + 64] = weight
    return out


def nam_term_sets_to_ext(sets16):
    """The 16-B form (nam_term_sets_array: {key, value, weight, 0} x 4, In [value] or
    Exists = 0xFF on one key) as ms_nam_term_set_ext records: that key's set is
    {value} or every id but 0, the other key's all ids (the library's own conversion)."""
    a = np.asarray(sets16, dtype=np.uint8).reshape(-1, NAM_TERMS, 4)
    sets = []
    for row in a:
        terms = []
        for key, value, weight, _ in row:
            key, value, weight = int(key), int(value), int(weight)
            if weight == 0 or value == 0:
                terms.append((0, 0, 0))
                continue
            m = (_ALL_IDS & ~1) if value == 0xFF else 1 << value
            terms.append((weight, m, _ALL_IDS) if key == 0 else (weight, _ALL_IDS, m))
        sets.append(terms)
    return nam_term_sets_ext_array(sets)


def nam_term_sets_array(sets):
    """ms_nam_term_set records (uint8 (n, 16)) from a list of term lists
    [(label key 0|1, value id 1..254 or 0xFF for Exists, weight 1..100), ...]
    (at most MS_NAM_TERMS each). Set i of the list is term set id i + 1."""
    out = np.zeros((len(sets), 16), dtype=np.uint8)
    for i, terms in enumerate(sets):
        if len(terms) > NAM_TERMS:
            raise ValueError(f"at most {NAM_TERMS} preferred terms per set")
        for k, (key, value, weight) in enumerate(terms):
            if key not in (0, 1) or not 1 <= value <= 255 or not 0 <= weight <= 100:
                raise ValueError("term: key 0/1, value 1..254 or 0xFF, weight 0..100")
            out[i, 4 * k:4 * k + 3] = (key, value, weight)
    return out
SEQ_SHARD_BATCH_MAX = 256
SEQ_MAX_SHARDS = 16
assert NODE_REC.itemsize == 64 and POD_REC.itemsize == 40 and RESULT.itemsize == 24 and SEQ_CAND.itemsize == 72
assert POD_COMPACT.itemsize == 8 and RESULT_COMPACT.itemsize == 8


def compact_pods(pods: np.ndarray) -> np.ndarray:
    """ms_pod_compact of pod records (their first 8 bytes)."""
    p = np.ascontiguousarray(pods, dtype=POD_REC)
    out = np.empty(len(p), dtype=POD_COMPACT)
    for f in POD_COMPACT.names:
        out[f] = p[f]
    return out


class ms_config(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int32),
        ("plugin_set", ctypes.c_int32),
        ("max_nodes", ctypes.c_uint32),
        ("node_base", ctypes.c_uint32),
        ("max_batch", ctypes.c_uint32),
        ("score_weight", ctypes.c_uint16 * 2),
        ("seed", ctypes.c_uint64),
    ]


CALL_PHASES = ("total", "lock_flush", "stage_in", "launch", "stage_out", "wait", "alloc", "chunks")  # MS_PH_*


class ms_call_profile(ctypes.Structure):
    _fields_ = [("ns", ctypes.c_uint64 * len(CALL_PHASES))]


class ms_info(ctypes.Structure):
    _fields_ = [
        ("max_nodes", ctypes.c_uint32),
        ("node_base", ctypes.c_uint32),
        ("present_nodes", ctypes.c_uint32),
        ("pending_deltas", ctypes.c_uint32),
        ("device", ctypes.c_int32),
        ("plugin_set", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("seq_pods", ctypes.c_uint32),
        ("seq_resweep_tiles", ctypes.c_uint32),
        ("seq_recomputes", ctypes.c_uint32),
        ("_pad", ctypes.c_uint32),
        ("comm_rank", ctypes.c_int32),
        ("comm_world", ctypes.c_int32),
    ]


COMM_ID_BYTES = 128  # MS_COMM_ID_BYTES (an ncclUniqueId)


class ms_comm_id(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * COMM_ID_BYTES)]


# Every function the header declares, with its ctypes signature.
_vp, _u32, _i32, _u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64
SIGNATURES = {
    "ms_abi_version": (ctypes.c_int, []),
    "ms_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "ms_create": (ctypes.c_int, [ctypes.POINTER(ms_config), ctypes.POINTER(_vp)]),
    "ms_destroy": (ctypes.c_int, [_vp]),
    "ms_last_error": (ctypes.c_char_p, [_vp]),
    "ms_get_info": (ctypes.c_int, [_vp, ctypes.POINTER(ms_info)]),
    "ms_last_call_profile": (ctypes.c_int, [_vp, ctypes.POINTER(ms_call_profile)]),
    "ms_nodes_upsert": (ctypes.c_int, [_vp, _u32, _vp, _vp]),
    "ms_nodes_delete": (ctypes.c_int, [_vp, _u32, _vp]),
    "ms_nodes_flush": (ctypes.c_int, [_vp]),
    "ms_nodes_read": (ctypes.c_int, [_vp, _u32, _u32, _vp]),
    "ms_schedule_batch": (ctypes.c_int, [_vp, _u32, _vp, _i32, _vp]),
    "ms_schedule_batch_compact": (ctypes.c_int, [_vp, _u32, _vp, _i32, _vp]),
    "ms_commit_bind": (ctypes.c_int, [_vp, _u32, _vp]),
    "ms_uncommit_bind": (ctypes.c_int, [_vp, _u32, _vp]),
    "ms_sweep_device": (ctypes.c_int, [_vp, _u32, _vp, _vp, _vp, _vp]),
    "ms_decode_device": (ctypes.c_int, [_vp, _u32, _vp, _vp, _vp, _u32, _vp, _vp]),
    "ms_decode_device_jobs": (ctypes.c_int, [_vp, _u32, _vp, _u32, _vp]),
    "ms_apply_binds_device": (ctypes.c_int, [_vp, _u32, _vp, _vp, _vp]),
    "ms_schedule_sequential_device": (ctypes.c_int, [_vp, _u32, _vp, _vp, _vp]),
    "ms_select_batch_device": (ctypes.c_int, [_vp, _u32, _vp, _vp, _vp]),
    "ms_seq_candidates_device": (ctypes.c_int, [_vp, _u32, _vp, _vp, _vp, _vp]),
    "ms_seq_validate_device": (ctypes.c_int, [_vp, _u32, _vp, _u32, _vp, _vp, _vp, _vp, _vp]),
    "ms_tt_summaries_device": (ctypes.c_int, [_vp, _u32, _vp, _vp, _vp]),
    "ms_tt_decode_device": (ctypes.c_int, [_vp, _u32, _vp, _u32, _vp, _vp, _vp]),
    "ms_tt_census_device": (ctypes.c_int, [_vp, _u32, _vp, _vp, _vp]),
    "ms_tt_pick_device": (ctypes.c_int, [_vp, _u32, _vp, _u32, _u32, _vp, _vp, _vp]),
    "ms_tt_final_device": (ctypes.c_int, [_vp, _u32, _vp, _u32, _vp, _vp, _vp, _vp]),
    "ms_nam_term_sets": (ctypes.c_int, [_vp, _u32, _vp]),
    "ms_nam_term_sets_ext": (ctypes.c_int, [_vp, _u32, _vp]),
    "ms_nam_segment_device": (ctypes.c_int, [_vp, _u32, _vp, _vp, _vp]),
    "ms_nam_keys_device": (ctypes.c_int, [_vp, _u32, _vp, _u32, _u32, _vp, _vp, _vp]),
    "ms_comm_id_create": (ctypes.c_int, [ctypes.POINTER(ms_comm_id)]),
    "ms_comm_init": (ctypes.c_int, [_vp, ctypes.POINTER(ms_comm_id), _i32, _i32]),
    "ms_sharded_slice": (ctypes.c_int, [_vp, _u32, ctypes.POINTER(_u32), ctypes.POINTER(_u32)]),
    "ms_sharded_submit": (ctypes.c_int, [_vp, _u32, _vp, _vp, _vp]),
    "ms_sharded_drain": (ctypes.c_int, [_vp, _vp]),
}

DECODE_MAX_JOBS = 8  # MS_DECODE_MAX_JOBS


class DecodeJob(ctypes.Structure):  # ms_decode_job
    _fields_ = [("pods", ctypes.c_void_p), ("keys", ctypes.c_void_p), ("flags", ctypes.c_void_p),
                ("results", ctypes.c_void_p), ("n_pods", ctypes.c_uint32), ("_pad", ctypes.c_uint32)]


assert ctypes.sizeof(DecodeJob) == 40

_LIBS: dict = {}


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Loads the HIP library (fails loudly when it was not built). Each path is
    its own handle (RTLD_LOCAL), so a test can hold the product library and the
    loopback build side by side."""
    if path in _LIBS:
        return _LIBS[path]
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} is missing: build it with `make -C mini-kube-scheduler_amd` "
            "(there is no CPU fallback for the scheduling path)"
        )
    # One HIP runtime per process. torch bundles its own libamdhip64.so.7 and
    # links it by a different NEEDED name than ours, so loading our library
    # first would map /opt/rocm's runtime beside torch's (two HSA runtimes: the
    # second sees no GPU). Loading torch first makes our NEEDED
    # libamdhip64.so.7 resolve to the runtime torch already mapped.
    if os.environ.get("MINISCHED_NO_TORCH", "0") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if hasattr(lib, "lb_collectives_issued"):  # the loopback build only
        lib.lb_collectives_issued.restype = ctypes.c_ulonglong
        lib.lb_collectives_issued.argtypes = []
    _LIBS[path] = lib
    return lib


class MSError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} -> {ERRNAMES.get(code, code)}: {msg}")
        self.code = code


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def comm_id_create(lib: Optional[ctypes.CDLL] = None) -> bytes:
    """A new communicator id (rank 0 creates it and ships the bytes to every rank)."""
    out = ms_comm_id()
    lib = lib or load()
    rc = lib.ms_comm_id_create(ctypes.byref(out))
    if rc != MS_OK:
        raise MSError("ms_comm_id_create", rc, lib.ms_last_error(None).decode())
    return ctypes.string_at(ctypes.addressof(out), COMM_ID_BYTES)  # (.internal stops at a NUL)


def device_count() -> int:
    n = ctypes.c_int(0)
    load().ms_device_count(ctypes.byref(n))
    return n.value


class Engine:
    """One context = one device and one contiguous range of node ordinals."""

    def __init__(
        self,
        max_nodes: int,
        plugin_set: int = PLUGINS_NU_NN,
        node_base: int = 0,
        seed: int = 1,
        device: int = 0,
        max_batch: int = 1 << 16,
        score_weights=(0, 0),
        lib: Optional[ctypes.CDLL] = None,
    ):
        self.lib = lib or load()
        cfg = ms_config(device, plugin_set, max_nodes, node_base, max_batch, (ctypes.c_uint16 * 2)(*score_weights), seed)
        h = ctypes.c_void_p()
        rc = self.lib.ms_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc != MS_OK:
            raise MSError("ms_create", rc, self.lib.ms_last_error(None).decode())
        self.h = h
        self.max_nodes, self.node_base, self.plugin_set, self.seed = max_nodes, node_base, plugin_set, seed

    def _check(self, fn: str, rc: int):
        if rc != MS_OK:
            raise MSError(fn, rc, self.lib.ms_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None):
            self.lib.ms_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def info(self) -> ms_info:
        out = ms_info()
        self._check("ms_get_info", self.lib.ms_get_info(self.h, ctypes.byref(out)))
        return out

    def last_call_profile(self) -> dict:
        """Host phase times of the last ms_schedule_batch(_compact) call: microseconds
        per MS_PH_* phase (chunks: a count)."""
        out = ms_call_profile()
        self._check("ms_last_call_profile", self.lib.ms_last_call_profile(self.h, ctypes.byref(out)))
        return {k: (int(out.ns[i]) if k == "chunks" else out.ns[i] * 1e-3) for i, k in enumerate(CALL_PHASES)}

    def upsert(self, ordinals: np.ndarray, recs: np.ndarray):
        o = np.ascontiguousarray(ordinals, dtype=np.uint32)
        recs = np.asarray(recs)
        if recs.dtype.names and "_pad1" in recs.dtype.names and recs.dtype.itemsize == NODE_REC.itemsize:
            recs = np.ascontiguousarray(recs).view(NODE_REC)  # (ABI 3 records: `taints` was `_pad1`)
        r = np.ascontiguousarray(recs, dtype=NODE_REC)
        assert len(o) == len(r)
        self._check("ms_nodes_upsert", self.lib.ms_nodes_upsert(self.h, len(o), _ptr(o), _ptr(r)))

    def delete(self, ordinals: np.ndarray):
        o = np.ascontiguousarray(ordinals, dtype=np.uint32)
        self._check("ms_nodes_delete", self.lib.ms_nodes_delete(self.h, len(o), _ptr(o)))

    def flush(self):
        self._check("ms_nodes_flush", self.lib.ms_nodes_flush(self.h))

    def read(self, first: int, n: int) -> np.ndarray:
        out = np.zeros(n, dtype=NODE_REC)
        self._check("ms_nodes_read", self.lib.ms_nodes_read(self.h, first, n, _ptr(out)))
        return out

    def schedule(self, pods: np.ndarray, mode: int = MODE_BATCHED, out: Optional[np.ndarray] = None) -> np.ndarray:
        """ms_schedule_batch. out: a reusable RESULT array of len(pods) (the
        caller's buffer, as a cgo caller would pass it)."""
        p = np.ascontiguousarray(pods, dtype=POD_REC)
        if out is None:
            out = np.zeros(len(p), dtype=RESULT)
        elif out.dtype != RESULT or len(out) != len(p) or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous RESULT array of len(pods)")
        self._check("ms_schedule_batch", self.lib.ms_schedule_batch(self.h, len(p), _ptr(p), mode, _ptr(out)))
        return out

    def schedule_compact(self, pods: np.ndarray, mode: int = MODE_BATCHED,
                         out: Optional[np.ndarray] = None) -> np.ndarray:
        """ms_schedule_batch_compact: POD_COMPACT in, RESULT_COMPACT out (8 B each way)."""
        p = np.ascontiguousarray(pods, dtype=POD_COMPACT)
        if out is None:
            out = np.zeros(len(p), dtype=RESULT_COMPACT)
        elif out.dtype != RESULT_COMPACT or len(out) != len(p) or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous RESULT_COMPACT array of len(pods)")
        self._check("ms_schedule_batch_compact",
                    self.lib.ms_schedule_batch_compact(self.h, len(p), _ptr(p), mode, _ptr(out)))
        return out

    def commit_bind(self, ordinal: int, pod: np.ndarray):
        p = np.ascontiguousarray(pod, dtype=POD_REC).reshape(1)
        self._check("ms_commit_bind", self.lib.ms_commit_bind(self.h, ordinal, _ptr(p)))

    def uncommit_bind(self, ordinal: int, pod: np.ndarray):
        p = np.ascontiguousarray(pod, dtype=POD_REC).reshape(1)
        self._check("ms_uncommit_bind", self.lib.ms_uncommit_bind(self.h, ordinal, _ptr(p)))

    # ---- device-resident entry points (raw device pointers as ints) --------
    def sweep_device(self, n_pods: int, pods_dev: int, keys_dev: int, flags_dev: int = 0, stream: int = 0):
        self._check(
            "ms_sweep_device",
            self.lib.ms_sweep_device(self.h, n_pods, pods_dev, keys_dev, flags_dev or None, stream or None),
        )

    def decode_device(self, n_pods, pods_dev, keys_dev, flags_dev, present_nodes, results_dev, stream=0):
        self._check(
            "ms_decode_device",
            self.lib.ms_decode_device(
                self.h, n_pods, pods_dev, keys_dev, flags_dev or None, present_nodes, results_dev, stream or None
            ),
        )

    def decode_device_jobs(self, jobs, present_nodes, stream=0):
        """jobs: [(n_pods, pods_dev, keys_dev, flags_dev or 0, results_dev)], at most
        DECODE_MAX_JOBS; one launch decodes them all (ms_decode_device_jobs)."""
        arr = (DecodeJob * max(1, len(jobs)))()
        for i, (n, pods, keys, flags, res) in enumerate(jobs):
            arr[i] = DecodeJob(pods, keys, flags or None, res, n, 0)
        self._check("ms_decode_device_jobs",
                    self.lib.ms_decode_device_jobs(self.h, len(jobs), arr, present_nodes, stream or None))

    def apply_binds_device(self, n_pods, pods_dev, results_dev, stream=0):
        self._check(
            "ms_apply_binds_device",
            self.lib.ms_apply_binds_device(self.h, n_pods, pods_dev, results_dev, stream or None),
        )

    def select_batch_device(self, n_pods, pods_dev, results_dev, stream=0):
        """Stateless batched cycle on a single-shard context (no bind commit)."""
        self._check(
            "ms_select_batch_device",
            self.lib.ms_select_batch_device(self.h, n_pods, pods_dev, results_dev, stream or None),
        )

    def seq_candidates_device(self, n_pods, pods_dev, cands_dev, flags_dev, stream=0):
        """Node-sharded sequential mode, step 1: this shard's top-4 candidates + flags."""
        self._check("ms_seq_candidates_device",
                    self.lib.ms_seq_candidates_device(self.h, n_pods, pods_dev, cands_dev, flags_dev, stream or None))

    def seq_validate_device(self, n_pods, pods_dev, n_shards, cands_all_dev, flags_all_dev, results_dev, n_done_dev,
                            stream=0):
        """Node-sharded sequential mode, step 3: replicated in-order validation + owned binds."""
        self._check("ms_seq_validate_device",
                    self.lib.ms_seq_validate_device(self.h, n_pods, pods_dev, n_shards, cands_all_dev, flags_all_dev,
                                                    results_dev, n_done_dev, stream or None))

    def tt_summaries_device(self, n_pods, pods_dev, summaries_dev, stream=0):
        """Node-sharded TaintToleration set, step 1: this shard's per-pod summaries."""
        self._check("ms_tt_summaries_device",
                    self.lib.ms_tt_summaries_device(self.h, n_pods, pods_dev, summaries_dev, stream or None))

    def tt_decode_device(self, n_pods, pods_dev, n_shards, summaries_all_dev, results_dev, stream=0):
        """Step 3: merge the shards' summaries (shard-major, LIST order) and decode."""
        self._check("ms_tt_decode_device",
                    self.lib.ms_tt_decode_device(self.h, n_pods, pods_dev, n_shards, summaries_all_dev, results_dev,
                                                 stream or None))

    def tt_census_device(self, n_pods, pods_dev, census_dev, stream=0):
        """Node-sharded TaintToleration, two-pass form, step 1: this shard's census."""
        self._check("ms_tt_census_device", self.lib.ms_tt_census_device(self.h, n_pods, pods_dev, census_dev,
                                                                        stream or None))

    def tt_pick_device(self, n_pods, pods_dev, n_shards, shard_index, census_all_dev, keys_dev, stream=0):
        """Step 3: this shard's keys under the plan of every shard's census (shard-major)."""
        self._check("ms_tt_pick_device",
                    self.lib.ms_tt_pick_device(self.h, n_pods, pods_dev, n_shards, shard_index, census_all_dev,
                                               keys_dev, stream or None))

    def tt_final_device(self, n_pods, pods_dev, n_shards, census_all_dev, keys_max_dev, results_dev, stream=0):
        """Step 5: results from every shard's census and the uint64 MAX of the shards' keys."""
        self._check("ms_tt_final_device",
                    self.lib.ms_tt_final_device(self.h, n_pods, pods_dev, n_shards, census_all_dev, keys_max_dev,
                                                results_dev, stream or None))

    def nam_term_sets(self, sets):
        """MS_PLUGINS_NU_NN_NAM: registers the term sets (uint8 array (n, 4, 4) of
        {key, value, weight, 0} per term, or a NAM_TERM_SET-compatible (n, 16)
        array); pod term set id s is row s - 1."""
        raw = np.ascontiguousarray(np.asarray(sets, dtype=np.uint8).reshape(-1, 16))
        self._check("ms_nam_term_sets", self.lib.ms_nam_term_sets(self.h, len(raw), raw.ctypes.data if len(raw) else None))

    def nam_term_sets_ext(self, sets):
        """The general form (ABI 7): uint8 (n, 272) ms_nam_term_set_ext records
        (nam_term_sets_ext_array)."""
        raw = np.ascontiguousarray(np.asarray(sets, dtype=np.uint8).reshape(-1, NAM_SET_EXT_BYTES))
        self._check("ms_nam_term_sets_ext",
                    self.lib.ms_nam_term_sets_ext(self.h, len(raw), raw.ctypes.data if len(raw) else None))

    def nam_segment_device(self, n_pods, pods_dev, seg_dev, stream=0):
        """Node-sharded multi-term NodeAffinity, step 1: this shard's rescale record per pod."""
        self._check("ms_nam_segment_device",
                    self.lib.ms_nam_segment_device(self.h, n_pods, pods_dev, seg_dev, stream or None))

    def nam_keys_device(self, n_pods, pods_dev, n_shards, shard_index, segs_all_dev, keys_dev, stream=0):
        """Step 3: this shard's packed keys under every shard's records (shard-major);
        the uint64 MAX over the shards decodes with decode_device (flags 0)."""
        self._check("ms_nam_keys_device",
                    self.lib.ms_nam_keys_device(self.h, n_pods, pods_dev, n_shards, shard_index, segs_all_dev, keys_dev,
                                                stream or None))

    # ---- in-library multi-GPU (a communicator per job) -------------------------
    def comm_init(self, comm_id: bytes, rank: int, world: int):
        """Joins this context (one node shard) to the job's RCCL communicator
        (collective over the ranks)."""
        if len(comm_id) != COMM_ID_BYTES:
            raise ValueError("comm_id must be MS_COMM_ID_BYTES bytes")
        cid = ms_comm_id()
        ctypes.memmove(ctypes.addressof(cid), comm_id, COMM_ID_BYTES)
        self._check("ms_comm_init", self.lib.ms_comm_init(self.h, ctypes.byref(cid), rank, world))

    def sharded_slice(self, n_pods: int):
        """(first, count): the pod slice of an n_pods batch this rank decodes."""
        a, b = ctypes.c_uint32(), ctypes.c_uint32()
        self._check("ms_sharded_slice", self.lib.ms_sharded_slice(self.h, n_pods, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def sharded_submit(self, n_pods, pods_dev, results_dev, stream=0):
        self._check("ms_sharded_submit",
                    self.lib.ms_sharded_submit(self.h, n_pods, pods_dev, results_dev or None, stream or None))

    def sharded_drain(self, stream=0):
        self._check("ms_sharded_drain", self.lib.ms_sharded_drain(self.h, stream or None))

    def schedule_sequential_device(self, n_pods, pods_dev, results_dev, stream=0):
        self._check(
            "ms_schedule_sequential_device",
            self.lib.ms_schedule_sequential_device(self.h, n_pods, pods_dev, results_dev, stream or None),
        )
