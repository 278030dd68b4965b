"""NumPy model of tools/os_sort_bench.hip's record sort, checked against a stable argsort on the CPU
before the kernel's first GPU run.  It follows the kernel step by step: the pass plan (passes,
digit width, the last pass's narrower digit), the all-pass histogram, each tile's per-wave stable
ranks (64 keys at a time, a lane's rank = earlier equal-digit lanes of its 64 + the wave's running
count), the waves' offsets inside the tile, the tiles' exclusive per-digit prefixes (what the
decoupled look-back computes), and the scatter position dbase[d] + wave offset + rank.

    python tools/os_sort_model.py        (exits non-zero on the first mismatch)
"""
import sys

import numpy as np

THREADS, ITEMS = 256, 16
WAVE_ITEMS, TILE = 64 * ITEMS, THREADS * ITEMS
MAX_BITS, MAX_PASSES = 12, 4


def plan(end_bit):
    passes = (end_bit + MAX_BITS - 1) // MAX_BITS
    dbits = (end_bit + passes - 1) // passes
    return passes, dbits, [(p * dbits, min(dbits, end_bit - p * dbits)) for p in range(passes)]


def one_pass(keys, vals, shift, nbits, ghist):
    n = len(keys)
    B = 1 << nbits
    digit = ((keys >> np.uint64(shift)) & np.uint64(B - 1)).astype(np.int64)
    dbase = np.concatenate([[0], np.cumsum(ghist[:B])[:-1]]).astype(np.int64)
    ntiles = (n + TILE - 1) // TILE
    pos = np.empty(n, np.int64)
    prefix = np.zeros(B, np.int64)  # per digit: keys of the tiles before (the look-back's result)
    for t in range(ntiles):
        wc = np.zeros((4, B), np.int64)
        rank = {}
        for w in range(4):
            base = t * TILE + w * WAVE_ITEMS
            for i in range(ITEMS):
                lo = base + i * 64
                idx = np.arange(lo, min(lo + 64, n))
                if len(idx) == 0:
                    continue
                d = digit[idx]
                # earlier lanes of these 64 with the same digit (the ballot-built peer mask)
                order = np.argsort(d, kind="stable")
                ds = d[order]
                first = np.searchsorted(ds, ds, side="left")
                within = np.empty(len(idx), np.int64)
                within[order] = np.arange(len(idx)) - first
                r = wc[w][d] + within
                for j, q in enumerate(idx):
                    rank[q] = (w, r[j])
                np.add.at(wc[w], d, 1)
        off = np.zeros((4, B), np.int64)
        off[1] = wc[0]
        off[2] = wc[0] + wc[1]
        off[3] = wc[0] + wc[1] + wc[2]
        cnt = wc.sum(axis=0)
        for q, (w, r) in rank.items():
            d = digit[q]
            pos[q] = dbase[d] + prefix[d] + off[w][d] + r
        prefix += cnt
    out_k = np.empty_like(keys)
    out_v = np.empty_like(vals)
    assert np.array_equal(np.sort(pos), np.arange(n)), "positions are not a permutation"
    out_k[pos] = keys
    out_v[pos] = vals
    return out_k, out_v


def model_sort(keys, vals, end_bit):
    passes, dbits, steps = plan(end_bit)
    assert passes <= MAX_PASSES
    hists = []
    for shift, nb in steps:
        d = ((keys >> np.uint64(shift)) & np.uint64((1 << nb) - 1)).astype(np.int64)
        hists.append(np.bincount(d, minlength=1 << nb))
    k, v = keys, vals
    for (shift, nb), h in zip(steps, hists):
        k, v = one_pass(k, v, shift, nb, h)
    return k, v


def check(n, bits, hot, seed):
    rng = np.random.default_rng(seed)
    mask = np.uint64((1 << bits) - 1)
    keys = rng.integers(0, 1 << 63, size=n, dtype=np.uint64) & mask
    hot_keys = rng.integers(0, 1 << 63, size=4, dtype=np.uint64) & mask
    h = rng.random(n) < hot
    keys[h] = hot_keys[(np.arange(n)[h] // 64) % 4]
    vals = np.arange(n, dtype=np.uint64)
    k, v = model_sort(keys, vals, bits)
    order = np.argsort(keys & mask, kind="stable")
    ok = np.array_equal(k, keys[order]) and np.array_equal(v, vals[order])
    print(f"n={n} bits={bits} hot={hot} passes={plan(bits)[0]}: {'ok' if ok else 'MISMATCH'}", flush=True)
    return ok


def main():
    cases = [(5000, 30, 0.5), (4096, 12, 0.0), (9000, 35, 0.5), (12289, 36, 0.3), (3000, 1, 0.0), (7000, 13, 0.9),
             (8200, 48, 0.2), (100, 7, 0.5)]
    ok = all(check(n, b, h, i) for i, (n, b, h) in enumerate(cases))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
