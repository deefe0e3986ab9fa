"""Model of the BVH build's chunked rank sort (rt_kernels.hip, bvh_build_kernel, n_inst <=
1024): per-64-entry chunk sort, then rank = lane + the entry's rank in every other sorted
chunk by a 6-step branchless binary search (<= against earlier chunks, < against later
ones).  It must give thrust's stable sort_by_key order (bvh.cu:86), i.e. (key, index)
order, with ties and ~0 (degenerate-box) keys.  The device kernel itself is checked by
the GPU parity tests (hit ids and BVH counters equal the oracle's); their scenes have no
tied Morton keys, hence this model test of the tie rules."""
import random

ONES = 2 ** 64 - 1


def chunked_rank_sort(keys):
    m = len(keys)
    nch = (m + 63) // 64
    chunks = [sorted((keys[t] if t < m else ONES, t) for t in range(64 * c, 64 * c + 64)) for c in range(nch)]
    S = [[k for k, _ in ch] for ch in chunks]
    out = [None] * m
    for c in range(nch):
        for lane, (k, x) in enumerate(chunks[c]):
            if x >= m:
                continue
            pos = lane
            for cc in range(nch):
                if cc == c:
                    continue
                pred = (lambda v: v <= k) if cc < c else (lambda v: v < k)
                p = 0
                for sp in (32, 16, 8, 4, 2, 1):
                    if pred(S[cc][p + sp - 1]):
                        p += sp
                pos += p + (1 if (p == 63 and pred(S[cc][63])) else 0)
            assert out[pos] is None
            out[pos] = (k, x)
    return out


def test_chunked_rank_sort_matches_stable_sort():
    rng = random.Random(7)
    for _ in range(200):
        m = rng.randint(1, 1024)
        r = rng.choice([0, 3, 50, 2 ** 40, ONES - 1])
        keys = [rng.randint(0, r) for _ in range(m)]
        if rng.random() < 0.3:
            keys = [k if rng.random() < 0.8 else ONES for k in keys]
        assert chunked_rank_sort(keys) == sorted((k, i) for i, k in enumerate(keys))
