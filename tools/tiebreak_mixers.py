#!/usr/bin/env python3
"""Tie uniformity of candidate tie-break mixers.

For many pods (A = fmix32(seed32 ^ pod)) and a tie set of T nodes at a given
ordinal stride, every node should win the argmax of the hash about 1/T of the
time. Prints chi-square / (dof + 5 sqrt(2 dof)) per case: above 1 fails the
5-sigma bound tests/test_oracle_kat.py uses. Rule r3 (the shipped one) passes
every case; the cheaper forms that fold one multiply into the node term fail
some stride.
"""
import numpy as np

M = np.uint64(0xFFFFFFFF)
C = np.uint64(0x9E3779)
P = 200_000
CASES = [(2, 1), (3, 1), (10, 1), (64, 1), (16, 10), (32, 1000), (2, 10), (3, 10), (2, 100), (2, 1000),
         (4, 1 << 16), (2, 1 << 18), (2, 3 << 17), (2, 1 << 19)]


def fmix32(h):
    h = h ^ (h >> np.uint64(16))
    h = (h * np.uint64(0x85EBCA6B)) & M
    h = h ^ (h >> np.uint64(13))
    h = (h * np.uint64(0xC2B2AE35)) & M
    return h ^ (h >> np.uint64(16))


def r3(a, ords):
    x = (a[:, None] + ords[None, :] * C) & M
    x = x ^ (x >> np.uint64(16))
    x = (x * np.uint64(0x85EBCA6B)) & M
    x = x ^ (x >> np.uint64(16))
    return (x * np.uint64(0xC2B2AE35)) & M


def folded(k1, k2):
    def f(a, ords):  # (A + ord*C)*k1 = A*k1 + ord*(C*k1): one mad, then xor-shift + multiply
        x = ((a[:, None] * np.uint64(k1)) + ords[None, :] * ((C * np.uint64(k1)) & M)) & M
        x = x ^ (x >> np.uint64(16))
        return (x * np.uint64(k2)) & M
    return f


def main():
    with np.errstate(over="ignore"):
        A = fmix32(np.arange(10**6, 10**6 + P, dtype=np.uint64) ^ np.uint64(1))
        for name, mx in (("r3", r3), ("fold 85ebca6b/c2b2ae35", folded(0x85EBCA6B, 0xC2B2AE35)),
                         ("fold c2b2ae35/85ebca6b", folded(0xC2B2AE35, 0x85EBCA6B)),
                         ("fold 9e3779b1/c2b2ae35", folded(0x9E3779B1, 0xC2B2AE35))):
            res = []
            for T, stride in CASES:
                ords = np.arange(T, dtype=np.uint64) * np.uint64(stride)
                w = np.bincount(np.argmax(mx(A, ords), axis=1), minlength=T)
                exp = P / T
                chi, dof = ((w - exp) ** 2 / exp).sum(), T - 1
                res.append(f"T{T}/s{stride}:{chi / (dof + 5 * np.sqrt(2 * dof)):.2f}")
            print(f"{name:24s}", " ".join(res))


if __name__ == "__main__":
    main()
