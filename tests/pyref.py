"""Second, independent restatement of graph-embed's hot path in pure Python.

Test infrastructure only.  Python floats are IEEE binary64 with every operation
rounded separately (no FMA), so evaluating the reference's expressions in the
reference's order reproduces the reference bit for bit.  It is used on small
cases to cross-check oracle/ge_oracle.cpp, which in turn checks the HIP path.

Each function cites the reference (include/forceatlas.hpp, src/partitioner.cpp,
src/embed.cpp) lines it follows.
"""
import math

EPS = 0.00001  # include/forceatlas.hpp:110, :337


class MT19937:
    """std::mt19937 (32-bit Mersenne Twister, init_genrand seeding)."""

    def __init__(self, seed):
        self.mt = [0] * 624
        self.mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            prev = self.mt[i - 1]
            self.mt[i] = (1812433253 * (prev ^ (prev >> 30)) + i) & 0xFFFFFFFF
        self.idx = 624

    def _twist(self):
        mt = self.mt
        for i in range(624):
            y = (mt[i] & 0x80000000) | (mt[(i + 1) % 624] & 0x7FFFFFFF)
            v = mt[(i + 397) % 624] ^ (y >> 1)
            if y & 1:
                v ^= 0x9908B0DF
            mt[i] = v
        self.idx = 0

    def __call__(self):
        if self.idx >= 624:
            self._twist()
        y = self.mt[self.idx]
        self.idx += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF


def uniform_m1_p1(gen):
    """libstdc++ uniform_real_distribution<double>(-1, 1): generate_canonical
    with two 32-bit draws, then canonical * (b - a) + a."""
    s = float(gen())
    s += float(gen()) * 4294967296.0
    c = s / 18446744073709551616.0
    if c >= 1.0:
        c = math.nextafter(1.0, 0.0)
    return c * 2.0 + (-1.0)


def _dist(u, v):
    acc = 0.0
    for a, b in zip(u, v):
        t = b - a
        acc += t * t
    return math.sqrt(acc)


def _mag(u):
    acc = 0.0
    for a in u:
        acc += a * a
    return math.sqrt(acc)


def force_atlas(indptr, indices, data, dim, coords=None, iterations=100000, seed=None,
                ks=0.1, ksmax=1.0, repel=1.0, attract=1.0, gravity=1.0):
    """forceAtlas with useWeights, no linlog/nohubs, delta 1, tolerate 1
    (include/forceatlas.hpp:89-270)."""
    n = len(indptr) - 1
    if coords is None:
        g = MT19937(seed)
        coords = [[uniform_m1_p1(g) for _ in range(dim)] for _ in range(n)]
    else:
        coords = [list(r) for r in coords]
    deg = []
    for i in range(n):
        s = 0.0
        for e in range(indptr[i], indptr[i + 1]):
            s += data[e]
        deg.append(s)
    prev = [[0.0] * dim for _ in range(n)]
    for _ in range(iterations):
        forces = []
        for i in range(n):
            f = [0.0] * dim
            di = deg[i] + 1
            xi = coords[i]
            for j in range(n):
                if j == i:
                    continue
                xj = coords[j]
                d = _dist(xi, xj)
                if d < EPS:
                    d = EPS
                val = di * (deg[j] + 1) * repel / (d * d)
                for k in range(dim):
                    f[k] += (-(xj[k] - xi[k]) / d) * val
            for e in range(indptr[i], indptr[i + 1]):
                xj = coords[indices[e]]
                d = _dist(xi, xj)
                if d < EPS:
                    d = EPS
                fa = attract * (d * data[e])
                for k in range(dim):
                    f[k] += ((xj[k] - xi[k]) / d) * fa
            m = _mag(xi)
            forces.append([f[k] + (-xi[k] / m) * gravity * di for k in range(dim)])
        for i in range(n):
            sw = _dist(forces[i], prev[i])
            tot = _mag(forces[i])
            sp = ks * 1.0 / (1 + 1.0 * math.sqrt(sw))
            cap = ksmax / tot
            if sp > cap:
                sp = cap
            for k in range(dim):
                coords[i][k] = forces[i][k] * sp + coords[i][k]
        prev = forces
    return coords


def force_atlas_ml(indptr, indices, data, pt_indptr, pt_indices, vertex_A, coords_A, r_A,
                   dim, iterations, seed, ks=0.1, ksmax=1.0, repel=1.0, attract=1.0,
                   gravity=1.0):
    """forceAtlasMultilevel in the single-thread draw order
    (include/forceatlas.hpp:314-574)."""
    n = len(indptr) - 1
    m = len(pt_indptr) - 1
    g = MT19937(seed)
    X = [[0.0] * dim for _ in range(n)]
    for a in range(m):
        v = pt_indices[pt_indptr[a]:pt_indptr[a + 1]]
        s = len(v)
        for vi in v:
            for k in range(dim):
                X[vi][k] = uniform_m1_p1(g)
        deg = []
        for vi in v:
            t = 0.0
            for e in range(indptr[vi], indptr[vi + 1]):
                if vertex_A[indices[e]] == a:
                    t += data[e]
            deg.append(t)
        prev = [[0.0] * dim for _ in range(s)]
        ca = coords_A[a]
        for _ in range(iterations):
            forces = []
            for i in range(s):
                f = [0.0] * dim
                di = deg[i] + 1
                xi = X[v[i]]
                for j in range(s):
                    if j == i:
                        continue
                    xj = X[v[j]]
                    d = _dist(xi, xj)
                    if d < EPS:
                        d = EPS
                    val = di * (deg[j] + 1) * repel / (d * d)
                    for k in range(dim):
                        f[k] += (-(xj[k] - xi[k]) / d) * val
                mg = _mag(xi)
                if mg < EPS:
                    mg = EPS
                for e in range(indptr[v[i]], indptr[v[i] + 1]):
                    j = indices[e]
                    if vertex_A[j] == a and j != i:
                        xj = X[j]
                        d = _dist(xi, xj)
                        if d < EPS:
                            d = EPS
                        fa = attract * (d * data[e])
                        for k in range(dim):
                            f[k] += ((xj[k] - xi[k]) / d) * fa
                    else:
                        cb = coords_A[vertex_A[j]]
                        d = _dist(ca, cb)
                        if d < EPS:
                            d = EPS
                        for k in range(dim):
                            f[k] += ((cb[k] - ca[k]) / d) * 100.0 / mg
                forces.append([f[k] + (-xi[k] / mg) * gravity * di for k in range(dim)])
            for i in range(s):
                acc = 0.0
                for k in range(dim):
                    t = forces[i][k] - prev[i][k]
                    acc += t * t
                sw = math.sqrt(acc)
                if sw < EPS:
                    sw = EPS
                tot = _mag(forces[i])
                sp = ks * 1.0 / (1 + 1.0 * math.sqrt(sw))
                cap = ksmax / tot
                if sp > cap:
                    sp = cap
                for k in range(dim):
                    X[v[i]][k] = forces[i][k] * sp + X[v[i]][k]
            prev = forces
        avg = [0.0] * dim
        for vi in v:
            for k in range(dim):
                avg[k] = avg[k] + X[vi][k]
        avg = [a_ / s for a_ in avg]
        for vi in v:
            for k in range(dim):
                X[vi][k] -= avg[k]
        big = 0.0
        for vi in v:
            mm = _mag(X[vi])
            if mm > big:
                big = mm
        if big < EPS:
            big = EPS
        for vi in v:
            for k in range(dim):
                X[vi][k] = ca[k] + r_A[a] * (X[vi][k] / big)
    return X


def partition(indptr, indices, data, cf, positive_merging=True, stall=1.0, matching=2):
    """Hierarchy partitioner (src/partitioner.cpp:1550-1893), mergeLeaves off.
    Returns a list of P_T as (indptr, indices, rows, cols)."""
    inf = float("inf")
    n = len(indptr) - 1
    nbr = [dict() for _ in range(n)]
    alpha = [0.0] * n
    T = 0.0
    for i in range(n):
        s = 0.0
        for e in range(indptr[i], indptr[i + 1]):
            if indices[e] != i:
                nbr[i].setdefault(indices[e], data[e])
            s += data[e]
        alpha[i] = s
    for i in range(n):
        for e in range(indptr[i], indptr[i + 1]):
            T += data[e]
    alpha = [x / T for x in alpha]
    basis = list(range(n))
    alive = list(range(n))
    where = list(range(n))
    up = list(range(n))
    best = [-inf] * n
    arg = [0] * n
    busy = [False] * n
    N = M = n
    out = []

    def root(x):
        r = x
        while up[r] != r:
            r = up[r]
        while up[x] != r:
            up[x], x = r, up[x]
        return r

    def snap():
        groups = [[] for _ in range(M)]
        for y, b in enumerate(basis):
            groups[where[root(b)]].append(y)
        ip, ix = [0], []
        for gr in groups:
            ix.extend(gr)
            ip.append(len(ix))
        out.append((ip, ix, M, N))

    while True:
        merged = []
        for _ in range(matching):
            for i in alive:
                if not busy[i] or best[i] == -inf:
                    b, bj = -inf, -1
                    for j in sorted(nbr[i]):
                        if not busy[j]:
                            eta = 2 * (nbr[i][j] / T - alpha[i] * alpha[j])
                            if eta > b:
                                b, bj = eta, j
                    best[i], arg[i] = b, bj
            for i in alive:
                if busy[i]:
                    continue
                j = arg[i]
                if j != -1 and not busy[j] and not (best[i] < best[j]):
                    if (not positive_merging) or best[i] > 0:
                        if len(nbr[i]) < len(nbr[j]):
                            merged.append((j, i))
                        else:
                            merged.append((i, j))
                        busy[i] = busy[j] = True
        for keep, gone in merged:
            for k in sorted(nbr[gone]):
                w = nbr[gone][k]
                del nbr[k][gone]
                best[k] = -inf
                if k == keep:
                    alpha[keep] = alpha[keep] + alpha[gone]
                else:
                    nbr[keep][k] = nbr[keep].get(k, 0.0) + w
                    nbr[k][keep] = nbr[k].get(keep, 0.0) + w
        M_prev = M
        if 1.0 * M / N <= cf:
            snap()
            basis = list(alive)
            N = M
        for keep, gone in merged:
            slot = where[gone]
            last = alive[-1]
            alive[slot], alive[-1] = alive[-1], alive[slot]
            alive.pop()
            where[last] = slot
            up[gone] = keep
            busy[keep] = False
            M -= 1
        if not (1.0 * M / M_prev < stall):
            break
    snap()
    return out
