"""Synthetic graph fixtures shared by the tests (numpy; test infrastructure).

R-MAT here is the definition the product's generator (ge_rmat_csr in
graph-embed_amd/csrc/ge_graph.cpp) must reproduce bit for bit:

  h(e, l)   = splitmix64(splitmix64(seed) + 64*e + l)       (uint64, wrapping)
  u(e, l)   = (h >> 11) * 2**-53
  quadrant  = 0 if u < a, 1 if u < a+b, 2 if u < a+b+c, else 3
  src, dst  = MSB-first bits (quadrant >> 1, quadrant & 1) over `scale` levels
  keep      = src < n and dst < n and src != dst
  A         = symmetrised, deduplicated, unit weights, rows/cols ascending

(Graph500 R-MAT parameters (a, b, c) = (0.57, 0.19, 0.19).)
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def rmat_edges(n, m, seed, a=0.57, b=0.19, c=0.19):
    scale = max(1, int(np.ceil(np.log2(max(n, 2)))))
    e = np.arange(m, dtype=np.uint64)
    base = splitmix64(np.uint64(seed))
    src = np.zeros(m, dtype=np.int64)
    dst = np.zeros(m, dtype=np.int64)
    for lvl in range(scale):
        with np.errstate(over="ignore"):
            h = splitmix64(base + e * np.uint64(64) + np.uint64(lvl))
        u = (h >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
        q = np.where(u < a, 0, np.where(u < a + b, 1, np.where(u < a + b + c, 2, 3)))
        src = (src << 1) | (q >> 1)
        dst = (dst << 1) | (q & 1)
    keep = (src < n) & (dst < n) & (src != dst)
    return src[keep], dst[keep]


def csr_from_edges(n, src, dst):
    r = np.concatenate([src, dst])
    c = np.concatenate([dst, src])
    key = np.unique(r.astype(np.int64) * n + c)
    rows = (key // n).astype(np.int64)
    cols = (key % n).astype(np.int32)
    ip = np.zeros(n + 1, dtype=np.int64)
    np.add.at(ip, rows + 1, 1)
    ip = np.cumsum(ip).astype(np.int32)
    return ip, cols, np.ones(len(cols), dtype=np.float64)


def rmat(n, m, seed=12345):
    s, d = rmat_edges(n, m, seed)
    return csr_from_edges(n, s, d)


def largest_component(A):
    """LCC as examples/embedder.cpp:35-93: components labelled in vertex order,
    the first largest wins, vertices kept in ascending order."""
    ip, ix, dx = A
    n = len(ip) - 1
    comp = -np.ones(n, dtype=np.int64)
    c = 0
    for s in range(n):
        if comp[s] != -1:
            continue
        comp[s] = c
        stack = [s]
        while stack:
            v = stack.pop()
            for w in ix[ip[v]:ip[v + 1]]:
                if comp[w] == -1:
                    comp[w] = c
                    stack.append(w)
        c += 1
    counts = np.bincount(comp, minlength=c)
    keep = np.flatnonzero(comp == int(np.argmax(counts)))
    return submatrix(A, keep)


def submatrix(A, keep):
    ip, ix, dx = A
    n = len(ip) - 1
    newid = -np.ones(n, dtype=np.int64)
    newid[keep] = np.arange(len(keep))
    rows, cols, vals = [], [], []
    nip = [0]
    for r in keep:
        seg = ix[ip[r]:ip[r + 1]]
        w = dx[ip[r]:ip[r + 1]]
        m = newid[seg] >= 0
        cols.append(newid[seg[m]])
        vals.append(w[m])
        nip.append(nip[-1] + int(m.sum()))
    cols = np.concatenate(cols) if cols else np.zeros(0)
    vals = np.concatenate(vals) if vals else np.zeros(0)
    return (np.array(nip, dtype=np.int32), cols.astype(np.int32), vals.astype(np.float64))


def erdos_renyi(n, p, seed=42):
    """G(n, p): upper-triangle Bernoulli from numpy RandomState(seed), symmetrised."""
    rs = np.random.RandomState(seed)
    iu, ju = np.triu_indices(n, 1)
    keep = rs.random_sample(len(iu)) < p
    return csr_from_edges(n, iu[keep].astype(np.int64), ju[keep].astype(np.int64))


def random_coords(n, dim, seed=7):
    return np.random.RandomState(seed).uniform(-1.0, 1.0, size=(n, dim))


def as_lists(A):
    ip, ix, dx = A
    return [int(x) for x in ip], [int(x) for x in ix], [float(x) for x in dx]


def with_hubs(A, hubs, seed=0):
    """A plus stars: hub h joined to k distinct random vertices for (h, k) in
    hubs (csr_from_edges symmetrises; unit weights).  Makes rows longer than one LDS chunk."""
    n = len(A[0]) - 1
    rows = np.repeat(np.arange(n), np.diff(A[0]))
    src, dst = [rows], [A[1].astype(np.int64)]
    rs = np.random.RandomState(seed)
    for h, k in hubs:
        nb = rs.choice(np.setdiff1d(np.arange(n), [h]), size=k, replace=False)
        src.append(np.full(k, h))
        dst.append(nb)
    return csr_from_edges(n, np.concatenate(src), np.concatenate(dst))


def with_degrees(A, targets, seed=0):
    """A plus edges so that vertex v has exactly targets[v] neighbours (each
    added edge goes to a random non-neighbour; unit weights, symmetric).
    Targets are applied in order; a later star may raise an earlier vertex's
    degree by one, so keep target vertices apart from each other's stars."""
    n = len(A[0]) - 1
    rs = np.random.RandomState(seed)
    src = np.repeat(np.arange(n), np.diff(A[0])).astype(np.int64)
    dst = A[1].astype(np.int64)
    protect = np.array(list(targets.keys()))
    for v, k in targets.items():
        nbrs = set(dst[src == v].tolist())
        need = k - len(nbrs)
        assert need >= 0, (v, k, len(nbrs))
        pool = np.setdiff1d(np.arange(n), np.concatenate([[v], list(nbrs), protect]))
        nb = rs.choice(pool, size=need, replace=False)
        src = np.concatenate([src, np.full(need, v), nb])
        dst = np.concatenate([dst, nb, np.full(need, v)])
    return csr_from_edges(n, src, dst)
