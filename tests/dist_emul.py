"""numpy replay of the distributed preconditioner apply and SpMVs, driven by the plans the
library exports (cpk_analysis_plan).  It follows the device algorithm step for step -- local
forward sweep, separator payload, allgather, redundant separator solve, local backward sweep --
in the exported factor's accumulation order, so it must equal the oracle's apply bit for bit.
Test infrastructure only."""
import numpy as np


def seq_rowsum(ptr, prod):
    """Row sums of CSR products, each row summed left to right from 0.0 (the device order)."""
    nr = len(ptr) - 1
    lens = np.diff(ptr)
    acc = np.zeros(nr)
    for k in range(int(lens.max()) if nr and len(prod) else 0):
        rows = np.nonzero(lens > k)[0]
        acc[rows] += prod[ptr[rows] + k]
    return acc


def _fwd_rows(pl):
    """Forward rows of the local factor with entries ordered by ascending key."""
    Lp, Li, Lx, key = pl["fsub_Lp"], pl["fsub_Li"], pl["fsub_Lx"], pl["fsub_key"]
    rows = [[] for _ in range(pl["nsub"])]
    for j in range(pl["nsub"]):
        for p in range(Lp[j], Lp[j + 1]):
            rows[Li[p]].append((key[j], j, Lx[p]))
    return [sorted(r) for r in rows]


def _bwd_rows(pl):
    """Backward rows (columns of L) including separator extras, ordered by descending key."""
    Lp, Li, Lx, key = pl["fsub_Lp"], pl["fsub_Li"], pl["fsub_Lx"], pl["fsub_key"]
    ep, ec, ek, ev = pl["extra_ptr"], pl["extra_col"], pl["extra_key"], pl["extra_val"]
    out = []
    for j in range(pl["nsub"]):
        r = [(key[Li[p]], Li[p], Lx[p]) for p in range(Lp[j], Lp[j + 1])]
        r += [(ek[p], ec[p], ev[p]) for p in range(ep[j], ep[j + 1])]
        out.append(sorted(r, reverse=True))
    return out


class RankApply:
    def __init__(self, pl):
        self.pl = pl
        self.fr = _fwd_rows(pl)
        self.br = _bwd_rows(pl)

    def phase1(self, x, neg_from):
        """local forward sweep; returns (w, payload of length kt)"""
        pl = self.pl
        nsub, nT, kt = pl["nsub"], pl["nT"], pl["kt"]
        perm = pl["fsub_perm"]
        w = np.zeros(nsub + nT)
        for i in range(nsub):
            s = perm[i]
            acc = -x[s] if s >= neg_from else x[s]
            for _, j, v in self.fr[i]:
                acc -= v * w[j]
            w[i] = acc
        pay = np.zeros(kt)
        ts = pl["tsend"]
        pay[:len(ts)] = w[ts]
        for t, d in enumerate(pl["tdof"]):  # rank 0 only
            pay[len(ts) + t] = -x[d] if d >= neg_from else x[d]
        return w, pay

    def phase2(self, w, recv):
        """separator solve (redundant) + local backward sweep; returns y (local)"""
        pl = self.pl
        nsub, nT = pl["nsub"], pl["nT"]
        tf_ptr, tf_col, tf_val, tf_src = pl["tf_ptr"], pl["tf_col"], pl["tf_val"], pl["tf_src"]
        tb_ptr, tb_col, tb_val, DT = pl["tb_ptr"], pl["tb_col"], pl["tb_val"], pl["DT"]
        lp, lr = pl["tlev_ptr"], pl["tlev_rows"]
        wT = w[nsub:]
        for lev in range(len(lp) - 1):
            for t in lr[lp[lev]:lp[lev + 1]]:
                acc = recv[tf_src[t]]
                for e in range(tf_ptr[t], tf_ptr[t + 1]):
                    c = tf_col[e]
                    acc -= tf_val[e] * (recv[c] if c >= 0 else wT[-c - 1])
                wT[t] = acc
        for lev in range(len(lp) - 2, -1, -1):
            for t in lr[lp[lev]:lp[lev + 1]]:
                acc = wT[t] / DT[t]
                for e in range(tb_ptr[t], tb_ptr[t + 1]):
                    acc -= tb_val[e] * wT[tb_col[e]]
                wT[t] = acc
        y = np.zeros(pl["N_loc"])
        for t, d in enumerate(pl["tdof"]):
            y[d] = wT[t]
        D, perm = pl["fsub_D"], pl["fsub_perm"]
        for i in range(nsub - 1, -1, -1):
            acc = w[i] / D[i]
            for _, j, v in self.br[i]:
                acc -= v * w[j]
            w[i] = acc
            y[perm[i]] = acc
        return y


def dist_spmv(pl, kind, xloc, recv):
    """local rows of K*x with ghosts read from the allgathered halo buffer"""
    ptr, col, val = pl[kind + "_ptr"], pl[kind + "_col"], pl[kind + "_val"]
    nloc = pl["N_loc"]
    xv = np.where(col < nloc, xloc[np.minimum(col, nloc - 1)], recv[np.maximum(col - nloc, 0)])
    return seq_rowsum(ptr, val * xv)


def halo_payload(pl, kind, xloc):
    k = pl[kind + "_kmax"]
    pay = np.zeros(k)
    s = pl[kind + "_send"]
    pay[:len(s)] = xloc[s]
    return pay
