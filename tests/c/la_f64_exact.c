/* Exactness of the binary64 LeastAllocated fast form used by the config-E sweep
 * (ms_kernels.hip, la_fast): for 0 <= cap < 2^41, av <= cap, 0 <= n < 2^53,
 *   r  = RN(100 / cap)            (0 when cap <= 0)
 *   a2 = RN(RN(av * r) + 2^-43)
 *   x  = RN(-n * r + a2)          (one fused multiply-add)
 *   q  = x <= 0 ? 0 : trunc(x)    (v_cvt_u32_f64 saturates negatives to 0)
 * equals the reference's leastRequestedScore(cap - av + n, cap):
 *   requested > capacity -> 0, capacity == 0 -> 0, else (cap - req) * 100 / cap,
 * i.e. floor(100 (av - n) / cap) for av >= n, else 0 (k8s v1.22
 * noderesources/least_allocated.go, restated in oracle/ms_oracle.c).
 * Error bound: |x - (X + eps)| <= 402 u, u = 2^-53, so the
 * result is floor(X) while eps > 402 u and eps + 402 u < 1/cap.
 * Build: cc -O2 -ffp-contract=off la_f64_exact.c -lm; prints the case count. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t sm;
static uint64_t next(void) {
    uint64_t z = (sm += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static const double kEps = 0x1p-43;

static uint32_t fast(int64_t cap, int64_t av, int64_t n) {
    const double r = cap > 0 ? 100.0 / (double)cap : 0.0;
    const double a = (double)av * r;
    const double a2 = a + kEps;
    const double x = fma(-(double)n, r, a2);
    if (!(x > 0.0)) return 0;
    return (uint32_t)x;
}

static uint32_t exact(int64_t cap, int64_t av, int64_t n) {
    if (cap <= 0) return 0;
    const __int128 t = (__int128)av - n;
    if (t < 0) return 0;
    return (uint32_t)((t * 100) / cap);
}

static int64_t pick_cap(void) {
    const uint64_t u = next();
    switch (u % 8) {
        case 0: return (int64_t)(1 + next() % 64) * 1000;                 /* millicores */
        case 1: return (int64_t)(1 + next() % 4096) << 20;                /* MiB multiples */
        case 2: return (int64_t)1 << (next() % 41);                       /* powers of two */
        case 3: return (int64_t)((1ull << 41) - 1 - next() % 1000);       /* top of the range */
        case 4: return (int64_t)(1 + next() % 1000);                      /* tiny */
        default: return (int64_t)(1 + next() % ((1ull << 41) - 1));       /* anything */
    }
}

int main(int argc, char **argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 20000000L;
    sm = 12345;
    long bad = 0, cases = 0;
    for (long i = 0; i < iters; ++i) {
        const int64_t cap = pick_cap();
        /* t = av - n near every k * cap / 100 boundary (exact integers and their neighbours) */
        const int64_t k = (int64_t)(next() % 101);
        const int64_t base = (int64_t)(((__int128)k * cap) / 100);
        const int64_t d = (int64_t)(next() % 5) - 2;
        int64_t t = base + d;
        if (next() % 8 == 0) t = (int64_t)(next() % (uint64_t)(cap + 1)) - (int64_t)(next() % 3);
        if (t > cap) t = cap;
        const int64_t room = cap - (t > 0 ? t : 0); /* n <= cap - t keeps av = t + n <= cap */
        int64_t n = room > 0 ? (int64_t)(next() % (uint64_t)(room + 1)) : 0;
        if (next() % 4 == 0) n = 0;
        int64_t av = t + n;
        if (av > cap) { av = cap; n = av - t; if (n < 0) continue; }
        ++cases;
        const uint32_t f = fast(cap, av, n), e = exact(cap, av, n);
        if (f != e) {
            if (bad < 10) printf("MISMATCH cap=%lld av=%lld n=%lld fast=%u exact=%u\n", (long long)cap, (long long)av,
                                 (long long)n, f, e);
            ++bad;
        }
    }
    /* overcommitted nodes (av < 0) and huge pod requests */
    for (long i = 0; i < iters / 10; ++i) {
        const int64_t cap = pick_cap();
        const int64_t av = -(int64_t)(next() % ((1ull << 53) - 1));
        const int64_t n = (int64_t)(next() % (1ull << 53));
        ++cases;
        if (fast(cap, av, n) != exact(cap, av, n)) ++bad;
        const int64_t av2 = (int64_t)(next() % (uint64_t)(cap + 1));
        ++cases;
        if (fast(cap, av2, n) != exact(cap, av2, n)) ++bad;
    }
    printf("cases=%ld mismatches=%ld\n", cases, bad);
    return bad != 0;
}
