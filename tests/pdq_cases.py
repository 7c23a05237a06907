"""Seeded TargetClustersList inputs for Go sort.Sort (pdqsort) emulation tests.

The shapes cover every branch of the pdqsort loop: insertion sort (n <= 12),
partialInsertionSort (nearly sorted, the shape the Aggregated cut sees: input in
sortClusters order, so nearly descending by replicas), the decreasing hint
(ascending input reversed), partitionEqual (many duplicates), breakPatterns and
the heapsort fallback (adversarial, imbalanced partitions).
"""
import random

SIZES = [0, 1, 2, 5, 12, 13, 24, 25, 49, 50, 51, 63, 64, 65, 100, 129, 500, 777, 2048, 3000, 5000]


def case(rng, n, kind):
    if kind == "random":
        return [rng.randint(0, 2**31 - 1) for _ in range(n)]
    if kind == "few":
        k = rng.choice([1, 2, 3, 5, 8])
        return [rng.randint(0, k) for _ in range(n)]
    if kind == "desc":
        v = sorted((rng.randint(0, 50) for _ in range(n)), reverse=True)
        return v
    if kind == "desc_perturbed":
        v = sorted((rng.randint(0, 1000) for _ in range(n)), reverse=True)
        for _ in range(rng.randint(1, 7)):
            if n >= 2:
                i, j = rng.randrange(n), rng.randrange(n)
                v[i], v[j] = v[j], v[i]
        return v
    if kind == "asc":
        return sorted(rng.randint(0, 50) for _ in range(n))
    if kind == "two_classes":  # score-100 block then score-0 block, each descending
        k = rng.randint(0, n)
        a = sorted((rng.randint(0, 300) for _ in range(k)), reverse=True)
        b = sorted((rng.randint(0, 300) for _ in range(n - k)), reverse=True)
        return a + b
    if kind == "organ":
        h = n // 2
        return list(range(h)) + list(range(n - h, 0, -1))
    if kind == "sawtooth":
        p = rng.randint(2, 40)
        return [i % p for i in range(n)]
    if kind == "equal":
        return [7] * n
    raise ValueError(kind)


KINDS = ["random", "few", "desc", "desc_perturbed", "asc", "two_classes", "organ", "sawtooth", "equal"]


def cases(seed, sizes=SIZES, kinds=KINDS):
    rng = random.Random(seed)
    for n in sizes:
        for kind in kinds:
            yield n, kind, case(rng, n, kind)
