"""Independent numpy restatement of the spec.  TEST INFRASTRUCTURE.

Written separately from oracle/acs_oracle.c (vectorised over receivers, numpy's own sort, no
shared code) so that agreement between the two pins the C oracle.  Each function cites the §A
rule it follows.  numpy performs every fp64 / fp32 operation as a single IEEE-rounded op (no
FMA); fp32 mode runs the same code on float32 arrays and float32 constants.
"""
from __future__ import annotations

import numpy as np

MASK32 = np.uint64(0xFFFFFFFF)
M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)

HONEST = 0xFFFFFFFF
BYZ = 0xFFFFFFFE

INIT, DROP, FAULTSET, CRASH_ROUND, CRASH_PARTIAL, BYZS, GRAPH, DELAY = range(8)


def philox(c0, c1, c2, c3, k0, k1):
    """§A.1 Philox4x32-10 on broadcastable uint arrays; returns 4 uint32 arrays."""
    c0, c1, c2, c3 = (np.asarray(v, dtype=np.uint64) & MASK32 for v in (c0, c1, c2, c3))
    k0 = np.asarray(k0, dtype=np.uint64) & MASK32
    k1 = np.asarray(k1, dtype=np.uint64) & MASK32
    for rnd in range(10):
        if rnd:
            k0 = (k0 + W0) & MASK32
            k1 = (k1 + W1) & MASK32
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & MASK32,
                          (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & MASK32)
    return tuple(v.astype(np.uint32) for v in (c0, c1, c2, c3))


def key_of(seed: int):
    return seed & 0xFFFFFFFF, seed >> 32


def draw(seed, stream, b, r, s):
    """§A.1 draw(stream, b, r, s) = philox((s>>2, r, b, stream), key(seed))[s & 3]."""
    s_arr = np.asarray(s, dtype=np.uint64)
    scalar = s_arr.ndim == 0
    s1 = np.atleast_1d(s_arr)
    k0, k1 = key_of(seed)
    w = philox(s1 >> np.uint64(2), r, b, stream, k0, k1)
    W = np.stack(np.broadcast_arrays(*w), axis=0)
    sel = np.broadcast_to((s1 & np.uint64(3)).astype(np.intp), W.shape[1:])
    out = np.take_along_axis(W, sel[None], axis=0)[0]
    return out[0] if scalar else out


def u53(w0, w1):
    """§A.1 u53 = ((w0>>5)·2^26 + (w1>>6)) · 2^-53 (exact)."""
    w0 = np.asarray(w0, dtype=np.uint64)
    w1 = np.asarray(w1, dtype=np.uint64)
    m = ((w0 >> np.uint64(5)) << np.uint64(26)) | (w1 >> np.uint64(6))
    return m.astype(np.float64) * 2.0 ** -53


def feistel(n: int, graph_seed: int, k: int, v, inverse: bool = False):
    """§A.3 π_k (or π_k^-1) of [0,n): 4-round Feistel on an even bit width, cycle walking."""
    mb = max(2, int(n - 1).bit_length())
    mb += mb & 1
    h = mb // 2
    mask = np.uint64((1 << h) - 1)
    hh = np.uint64(h)
    k0, k1 = key_of(graph_seed)
    v = np.array(v, dtype=np.uint64, copy=True)
    todo = np.ones(v.shape, dtype=bool)
    first = True
    while first or todo.any():
        first = False
        cur = v[todo]
        L, R = cur >> hh, cur & mask
        if not inverse:
            for j in range(4):
                f = philox(R, j, k, GRAPH, k0, k1)[0].astype(np.uint64) & mask
                L, R = R, L ^ f
        else:
            for j in (3, 2, 1, 0):
                f = philox(L, j, k, GRAPH, k0, k1)[0].astype(np.uint64) & mask
                L, R = R ^ f, L
        cur = (L << hh) | R
        v[todo] = cur
        todo = v >= np.uint64(n)
    return v


def drop_threshold(p: float) -> int:
    """§A.5 thr = (u32) floor(p · 2^32) in fp64."""
    return int(min(max(np.floor(p * 4294967296.0), 0.0), 4294967295.0))


def tree_sum_rows(a: np.ndarray) -> np.ndarray:
    """§A.7 tree_sum of every row: pad with +0.0 to a power of two, stride-halving adds."""
    a = np.asarray(a)
    n = a.shape[-1]
    P = 1
    while P < n:
        P *= 2
    w = np.zeros(a.shape[:-1] + (P,), dtype=a.dtype)
    w[..., :n] = a
    s = P // 2
    while s >= 1:
        w[..., :s] = w[..., :s] + w[..., s:2 * s]
        s //= 2
    return w[..., 0]


def apply_rule(rule: int, t: int, S: np.ndarray, xi=None) -> np.ndarray:
    """§A.7 on rows of S (entry order preserved for AVERAGE); xi = receivers' own values (W-MSR)."""
    m = S.shape[1]
    ft = S.dtype.type
    if rule == 0:
        return tree_sum_rows(S) / ft(m)
    if rule == 4:
        # W-MSR: drop min(t, #below x_i) smallest and min(t, #above x_i) largest;
        # zero padding past the window leaves the stride-halving sum unchanged (no -0.0 values)
        Ss = np.sort(S, axis=1)
        xi = np.asarray(xi, dtype=S.dtype)[:, None]
        lo = np.minimum(t, (Ss < xi).sum(axis=1))
        hi = np.minimum(t, (Ss > xi).sum(axis=1))
        nw = m - lo - hi
        k = np.arange(m)[None, :]
        idx = np.minimum(lo[:, None] + k, m - 1)
        W = np.where(k < nw[:, None], np.take_along_axis(Ss, idx, axis=1), ft(0))
        return tree_sum_rows(W) / nw.astype(S.dtype)
    R = np.sort(S, axis=1)[:, t:m - t]
    if rule == 1:
        return tree_sum_rows(R) / ft(R.shape[1])
    if rule == 2:
        return (R[:, 0] + R[:, -1]) * ft(0.5)
    Q = R[:, ::t]
    return tree_sum_rows(Q) / ft(Q.shape[1])


def apply_rule_omit(rule: int, t: int, S: np.ndarray, miss: np.ndarray, xi) -> np.ndarray:
    """DESIGN.md §9 missing_policy = OMIT, rows of S with a missing-entry mask (self never
    missing): AVERAGE sums the entry-order row with +0.0 in the missing places and divides by
    m' = #present; the other rules see only the present entries, and TRIMMED / MIDPOINT / DLPSW
    keep x_i when m' <= 2t.  Written with +inf fillers (they sort last) and masked windows
    (zero padding past a window leaves the stride-halving sum unchanged)."""
    ft = S.dtype.type
    m = S.shape[1]
    mp = m - miss.sum(axis=1)
    xi = np.asarray(xi, dtype=S.dtype)
    if rule == 0:
        return tree_sum_rows(np.where(miss, ft(0), S)) / mp.astype(S.dtype)
    Ss = np.sort(np.where(miss, ft(np.inf), S), axis=1)
    k = np.arange(m)[None, :]
    if rule == 4:
        lo = np.minimum(t, (Ss < xi[:, None]).sum(axis=1))
        hi = np.minimum(t, (Ss > xi[:, None]).sum(axis=1) - miss.sum(axis=1))
        nw = mp - lo - hi
        idx = np.minimum(lo[:, None] + k, m - 1)
        W = np.where(k < nw[:, None], np.take_along_axis(Ss, idx, axis=1), ft(0))
        return tree_sum_rows(W) / nw.astype(S.dtype)
    ok = mp > 2 * t
    nr = np.where(ok, mp - 2 * t, 1)
    rows = np.arange(S.shape[0])
    if rule == 2:
        res = (Ss[:, t] + Ss[rows, np.where(ok, mp - t - 1, t)]) * ft(0.5)
    else:
        step = t if rule == 3 else 1
        cnt = (nr + step - 1) // step
        width = (m - 2 * t + step - 1) // step
        kk = np.arange(width)[None, :]
        idx = np.minimum(t + kk * step, m - 1)
        W = np.where(kk < cnt[:, None], np.take_along_axis(Ss, np.broadcast_to(idx, (S.shape[0], width)), axis=1), ft(0))
        res = tree_sum_rows(W) / cnt.astype(S.dtype)
    return np.where(ok, res, xi)


class NpSim:
    """Vectorised restatement of one configuration (attribute names as acsim.Config)."""

    def __init__(self, cfg, csr=None):
        from acsim.config import _enum
        if csr is not None:
            self.rowptr = np.asarray(csr[0], dtype=np.int64)
            self.colidx = np.asarray(csr[1], dtype=np.int64)
        self.cfg = cfg
        self.N = N = int(cfg.n_nodes)
        self.B = int(cfg.n_instances)
        self.topo = _enum("topology", cfg.topology)
        self.rule = _enum("rule", cfg.rule)
        self.fault = _enum("fault_model", cfg.fault_model)
        self.byz = _enum("byz_strategy", cfg.byz_strategy)
        self.term = _enum("termination", cfg.termination)
        self.t = int(cfg.trim)
        self.d = int(cfg.degree)
        self.seed = int(cfg.seed)
        gseed = int(cfg.graph_seed) or self.seed
        self.thr = drop_threshold(cfg.loss_p)
        self.m = N if self.topo == 0 else self.d + 1
        if self.topo == 1:
            i = np.arange(N, dtype=np.uint64)
            cols = []
            for t in range(self.d):
                cols.append(feistel(N, gseed, t >> 1, i, inverse=bool(t & 1)))
            self.nbr = np.stack(cols, axis=1).astype(np.int64)
        self.f32 = _enum("dtype", getattr(cfg, "dtype", "f64")) == 1
        self.ft = np.float32 if self.f32 else np.float64
        self.x = np.empty((self.B, N), dtype=self.ft)
        self.status = np.full((self.B, N), HONEST, dtype=np.uint64)
        self.gb = [int(cfg.instance_offset) + lb for lb in range(self.B)]
        idx = np.arange(N, dtype=np.uint64)
        for lb, b in enumerate(self.gb):
            w = draw(self.seed, INIT, b, 0, 2 * idx), draw(self.seed, INIT, b, 0, 2 * idx + 1)
            if self.f32:   # (draw(INIT,b,0,2i) >> 8) * 2^-24
                self.x[lb] = (w[0] >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)
            else:
                self.x[lb] = u53(*w)
            f = int(cfg.n_faulty)
            if self.fault and f:
                keys = (draw(self.seed, FAULTSET, b, 0, idx).astype(np.uint64) << np.uint64(32)) | idx
                fv = (np.sort(keys)[:f] & MASK32).astype(np.int64)
                if self.fault == 2:
                    self.status[lb, fv] = BYZ
                else:
                    cr = draw(self.seed, CRASH_ROUND, b, 0, fv.astype(np.uint64)).astype(np.uint64)
                    self.status[lb, fv] = cr % np.uint64(cfg.crash_window)
        self.rounds = np.zeros(self.B, dtype=np.int64)
        # bounded-delay rounds: every past x^q, q = 0..r
        self.D = int(getattr(cfg, "delay_max", 0))
        self.omit = _enum("missing_policy", getattr(cfg, "missing_policy", "self")) == 1
        self.hist = [[self.x[lb].copy()] for lb in range(self.B)]
        self.trace = [[] for _ in range(self.B)]
        self.lo = np.zeros(self.B, dtype=self.ft)
        self.hi = np.zeros(self.B, dtype=self.ft)
        self.done = np.zeros(self.B, dtype=bool)
        self.converged = np.zeros(self.B, dtype=bool)
        for lb in range(self.B):
            self._after(lb)

    def _after(self, lb):
        h = self.status[lb] == HONEST
        xs = self.x[lb][h]
        self.lo[lb], self.hi[lb] = xs.min(), xs.max()
        sp = float(self.hi[lb] - self.lo[lb])
        self.trace[lb].append(sp)
        self.converged[lb] = sp <= self.cfg.eps
        self.done[lb] = (self.term == 0 and sp <= self.cfg.eps) or self.rounds[lb] >= self.cfg.max_rounds

    def _step(self, lb):
        cfg = self.cfg
        b = self.gb[lb]
        G = int(cfg.mask_group)
        bG = b - b % G
        r = int(self.rounds[lb])
        x = self.x[lb]
        st = self.status[lb]
        N = self.N
        lo, hi = self.lo[lb], self.hi[lb]
        crash_node = (st != HONEST) & (st != BYZ)
        active = (st == HONEST) | (crash_node & (np.uint64(r) < st))
        A = np.nonzero(active)[0]
        xn = x.copy()
        if A.size and self.topo == 2:
            # CSR (§8(f) row 1): m_i varies, so receivers are resolved one row at a time
            for i in A:
                rp, re_ = int(self.rowptr[i]), int(self.rowptr[i + 1])
                J = np.concatenate([[i], self.colidx[rp:re_]])[None, :]
                slots = np.concatenate([[0], np.arange(rp, re_)]).astype(np.uint64)[None, :]
                selfm = np.zeros(J.shape, dtype=bool)
                selfm[0, 0] = True
                V, miss = self._values(np.array([i]), J, slots, selfm, r, b, bG, x, st, lo, hi)
                xn[i] = self._rule(V, miss, x[[i]])[0]
        elif A.size:
            if self.topo == 0:
                J = np.broadcast_to(np.arange(N), (A.size, N))
                slots = A[:, None].astype(np.uint64) * np.uint64(N) + J.astype(np.uint64)
                selfm = J == A[:, None]
            else:
                J = np.concatenate([A[:, None], self.nbr[A]], axis=1)
                tt = np.arange(self.d, dtype=np.uint64)
                slots = np.concatenate(
                    [np.zeros((A.size, 1), np.uint64),
                     A[:, None].astype(np.uint64) * np.uint64(self.d) + tt[None, :]], axis=1)
                selfm = np.zeros(J.shape, dtype=bool)
                selfm[:, 0] = True
            V, miss = self._values(A, J, slots, selfm, r, b, bG, x, st, lo, hi)
            xn[A] = self._rule(V, miss, x[A])
        self.x[lb] = xn
        self.hist[lb].append(xn.copy())
        self.rounds[lb] = r + 1
        self._after(lb)

    def _rule(self, V, miss, xi):
        if self.omit:
            return apply_rule_omit(self.rule, self.t, V, miss, xi)
        return apply_rule(self.rule, self.t, V, xi)

    def _values(self, A, J, slots, selfm, r, b, bG, x, st, lo, hi):
        """§A.6 resolution of the entry matrix (rows = receivers A, columns = entries)."""
        cfg = self.cfg
        if True:
            sj = st[J]
            cj = (sj != HONEST) & (sj != BYZ) & ~selfm
            missing = cj & (np.uint64(r) > sj)
            eq = cj & (np.uint64(r) == sj)
            if eq.any():
                missing[eq] = draw(self.seed, CRASH_PARTIAL, b, r, slots[eq]) >= np.uint32(0x80000000)
            if self.thr > 0:
                cand = ~missing & ~selfm
                missing[cand] = draw(self.seed, DROP, bG, r, slots[cand]) < np.uint32(self.thr)
            V = x[J].copy()
            if self.D:
                # delivered value x_j^{r - delta}, delta = min(r, draw(DELAY, b, r, s) mod (D + 1))
                lb = b - int(cfg.instance_offset)
                dl = (draw(self.seed, DELAY, b, r, slots) % np.uint32(self.D + 1)).astype(np.int64)
                dl = np.minimum(dl, r)
                for dv in range(1, self.D + 1):
                    mk = (dl == dv) & ~selfm
                    if mk.any():
                        V[mk] = self.hist[lb][r - dv][J[mk]]
            byzm = (sj == BYZ) & ~selfm & ~missing
            if byzm.any():
                ft = self.ft
                d = ft(cfg.byz_delta)
                lo, hi = ft(lo), ft(hi)
                if self.byz == 0:
                    rowv = np.where((A % 2) == 0, hi + d, lo - d)
                    V[byzm] = np.broadcast_to(rowv[:, None], V.shape)[byzm]
                elif self.byz == 2:
                    V[byzm] = ft(cfg.byz_const) + ft(0)
                else:
                    s2 = slots[byzm] * np.uint64(2)
                    if self.f32:   # u24 = (draw(BYZ,b,r,2s) >> 8) * 2^-24
                        u = (draw(self.seed, BYZS, b, r, s2) >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)
                    else:
                        u = u53(draw(self.seed, BYZS, b, r, s2), draw(self.seed, BYZS, b, r, s2 + np.uint64(1)))
                    V[byzm] = (lo - d) + u * ((hi - lo) + ft(2) * d)
            V[missing | selfm] = np.broadcast_to(x[A][:, None], V.shape)[missing | selfm]
        return V, missing & ~selfm

    def round(self, k=1):
        for lb in range(self.B):
            for _ in range(k):
                if self.done[lb]:
                    break
                self._step(lb)

    def run(self):
        for lb in range(self.B):
            while not self.done[lb]:
                self._step(lb)
