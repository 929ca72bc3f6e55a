"""CPU stand-ins for the node-sharded exact sequential protocol (test infrastructure).

They restate, in numpy, what each rank's HIP kernels do in
minisched_gpu.h's ms_seq_candidates_device / ms_seq_validate_device, so that
the distribution protocol (per-shard top-4 + records, all-gather, replicated
in-order validation with truncation, binds routed to their owner) can run
under gloo on CPU and be compared with the single-process sequential oracle.
Semantics follow oracle/ms_oracle.c (minisched.go:115-199,304-325 + upstream
NodeResourcesFit / LeastAllocated / NodeInfo.AddPod).
"""
import numpy as np

M32 = np.uint64(0xFFFFFFFF)
TOPK = 4


def _fmix32(h):
    h = h ^ (h >> np.uint64(16))
    h = (h * np.uint64(0x85EBCA6B)) & M32
    h = h ^ (h >> np.uint64(13))
    h = (h * np.uint64(0xC2B2AE35)) & M32
    return h ^ (h >> np.uint64(16))


def _mix32(x):
    x = x ^ (x >> np.uint64(16))
    x = (x * np.uint64(0x85EBCA6B)) & M32
    x = x ^ (x >> np.uint64(16))
    return (x * np.uint64(0xC2B2AE35)) & M32


def _lr(requested, capacity):
    with np.errstate(divide="ignore", invalid="ignore"):
        v = np.where(capacity > 0, (capacity - requested) * 100 // np.maximum(capacity, 1), 0)
    return np.where((capacity == 0) | (requested > capacity), 0, v)


class Shard:
    """One rank's node columns (global ordinals [base, base + n))."""

    def __init__(self, recs, base):
        self.base = base
        self.n = len(recs)
        self.absent = recs["allowed_pods"] < 0
        self.unsched = recs["unschedulable"].astype(bool)
        self.digit = np.where(recs["name_digit"] <= 9, recs["name_digit"], 0xFF).astype(np.int64)
        self.allowed = recs["allowed_pods"].astype(np.int64)
        self.cnt = recs["pod_count"].astype(np.int64)
        self.alloc_cpu = recs["alloc_milli_cpu"].astype(np.int64)
        self.alloc_mem = recs["alloc_memory"].astype(np.int64)
        self.req_cpu = recs["req_milli_cpu"].astype(np.int64)
        self.req_mem = recs["req_memory"].astype(np.int64)
        self.nz_cpu = recs["nonzero_milli_cpu"].astype(np.int64)
        self.nz_mem = recs["nonzero_memory"].astype(np.int64)
        self.ords = np.arange(base, base + self.n, dtype=np.uint64)

    def candidates(self, pods, seed):
        """Per pod: top-4 (key, record) over this shard and the filter flags (bit0 NU, bit8 NRF)."""
        P = len(pods)
        cands = np.zeros((P, TOPK, 11), dtype=np.int64)  # key, 6 resources, allowed, cnt, flags_digit
        flags = np.zeros(P, dtype=np.int64)
        s32 = np.uint64((seed ^ (seed >> 32)) & 0xFFFFFFFF)
        for j in range(P):
            pr = pods[j]
            tol = bool(pr["tolerates_unschedulable"])
            nu = ~self.absent & self.unsched & (not tol)
            rc, rm = int(pr["req_milli_cpu"]), int(pr["req_memory"])
            bad = self.cnt + 1 > self.allowed
            if not (rc == 0 and rm == 0):
                bad = bad | (rc > self.alloc_cpu - self.req_cpu) | (rm > self.alloc_mem - self.req_mem)
            nrf = ~self.absent & ~nu & bad
            feas = ~self.absent & ~nu & ~nrf
            flags[j] = (1 if nu.any() else 0) | (0x100 if nrf.any() else 0)
            la = (_lr(self.nz_cpu + int(pr["nonzero_milli_cpu"]), self.alloc_cpu) +
                  _lr(self.nz_mem + int(pr["nonzero_memory"]), self.alloc_mem)) // 2
            nn = np.where(self.digit == int(pr["name_digit"]), 10, 0)
            score = (nn + la).astype(np.uint64)
            A = _fmix32(np.array([s32 ^ np.uint64(int(pr["ordinal"]))], dtype=np.uint64))[0]
            h = _mix32((A + self.ords * np.uint64(0x9E3779)) & M32)
            keys = (score << np.uint64(52)) | (h << np.uint64(20)) | (np.uint64(0xFFFFF) - self.ords)
            keys = np.where(feas, keys, np.uint64(0))
            order = np.argsort(keys)[::-1][:TOPK]
            for r, i in enumerate(order):
                if keys[i] == 0:
                    break
                cands[j, r] = [np.int64(keys[i].astype(np.int64)), self.alloc_cpu[i], self.alloc_mem[i], self.req_cpu[i],
                               self.req_mem[i], self.nz_cpu[i], self.nz_mem[i], self.allowed[i], self.cnt[i],
                               (1 if self.unsched[i] else 0) | (int(self.digit[i]) << 8), 0]
        return cands, flags

    def commit(self, ordinal, rec):
        """Write back a bound node's live record (only this shard's own nodes)."""
        if not (self.base <= ordinal < self.base + self.n):
            return False
        i = ordinal - self.base
        self.req_cpu[i], self.req_mem[i], self.nz_cpu[i], self.nz_mem[i], self.cnt[i] = rec
        return True


def _eval(rec, ordinal, pr, seed):
    """Packed key of (pod, node) against a candidate record (0 = filtered out)."""
    key, acpu, amem, rcpu, rmem, ncpu, nmem, allowed, cnt, fd = [int(x) for x in rec[:10]]
    if (fd & 1) and not pr["tolerates_unschedulable"]:
        return 0
    rc, rm = int(pr["req_milli_cpu"]), int(pr["req_memory"])
    if cnt + 1 > allowed:
        return 0
    if not (rc == 0 and rm == 0) and (rc > acpu - rcpu or rm > amem - rmem):
        return 0

    def lr(req, cap):
        return 0 if cap == 0 or req > cap else (cap - req) * 100 // cap

    la = (lr(ncpu + int(pr["nonzero_milli_cpu"]), acpu) + lr(nmem + int(pr["nonzero_memory"]), amem)) // 2
    nn = 10 if (fd >> 8) == int(pr["name_digit"]) else 0
    s32 = (seed ^ (seed >> 32)) & 0xFFFFFFFF
    A = int(_fmix32(np.array([s32 ^ int(pr["ordinal"])], dtype=np.uint64))[0])
    h = int(_mix32(np.array([(A + ordinal * 0x9E3779) & 0xFFFFFFFF], dtype=np.uint64))[0])
    return ((nn + la) << 52) | (h << 20) | (0xFFFFF - ordinal)


def validate(pods, cands_all, flags_all, seed):
    """The replicated validation over the gathered lists: cands_all [G][P][4][11],
    flags_all [G][P]. Returns (n_done, results [(code, node, score, mask)], bound
    {ordinal: (req_cpu, req_mem, nz_cpu, nz_mem, pod_count)})."""
    G, P = cands_all.shape[0], cands_all.shape[1]
    merged = []
    for j in range(P):
        ents = [cands_all[s, j, r] for s in range(G) for r in range(TOPK) if cands_all[s, j, r, 0] != 0]
        ents.sort(key=lambda e: int(e[0]), reverse=True)  # keys < 2^63: the int64 order is the u64 order
        merged.append([e.copy() for e in ents[:TOPK]])
    live = {}  # ordinal -> record (list of 11 ints), bound in this batch
    out = []
    for j in range(P):
        pr = pods[j]
        lst = merged[j]
        f = next((r for r, e in enumerate(lst) if (0xFFFFF - (int(e[0]) & 0xFFFFF)) not in live), None)
        if f is None and len(lst) == TOPK:
            return j, out, live
        best, best_ord, best_rec = 0, -1, None
        upto = len(lst) if f is None else f
        for r in range(upto):
            o = 0xFFFFF - (int(lst[r][0]) & 0xFFFFF)
            v = _eval(live[o], o, pr, seed)
            if v > best:
                best, best_ord, best_rec = v, o, None
        if f is not None:
            e = lst[f]
            v = int(e[0]) & 0xFFFFFFFFFFFFFFFF
            if v > best:
                best, best_ord, best_rec = v, 0xFFFFF - (v & 0xFFFFF), e
        fm = int(np.bitwise_or.reduce(flags_all[:, j]))
        if best == 0:
            if lst:
                fm |= 0x100
            out.append((2, -1, 0, (1 if fm & 0xFF else 0) | (2 if fm & 0xFF00 else 0)))
        elif pr["name_digit"] < 0:
            out.append((1, -1, 0, 0))
        else:
            out.append((0, best_ord, best >> 52, 0))
            rec = live.get(best_ord)
            if rec is None:
                rec = [int(x) for x in best_rec]
                live[best_ord] = rec
            rec[3] += int(pr["req_milli_cpu"])
            rec[4] += int(pr["req_memory"])
            rec[5] += int(pr["nonzero_milli_cpu"])
            rec[6] += int(pr["nonzero_memory"])
            rec[8] += 1
    return P, out, live
