// precond.cpp -- the constraint preconditioner M = opLDL2(G, B, -C) on the device.
//
// Construction replaces opLDL2's constructor (ops/opLDL2.m:60-92): assemble Kp = [A B'; B C],
// choose a fill-reducing ordering, factor P'*Kp*P = L*D*L' on the host, cut the elimination
// tree into the sweep schedule, and upload Kp, L, L', D and P to HBM.
// apply() replaces opLDL2.multiply (ops/opLDL2.m:161-188) with the effective semantics of the
// reference: Spot operators are value objects, so the residual-update state (Aty, Cy) written
// inside multiply never survives the call and the branch subtracts zeros -- it is skipped here
// (a functional no-op).  With force_itref the residual norms do not influence the loop and
// the residual after the last refinement step is never read, so neither is computed.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <memory>

#include "dev.hpp"

namespace cpk {

SweepConfig sweep_config() {
    SweepConfig cfg;
    if (const char *e = getenv("CPK_SWEEP")) {
        int v[7] = {0, 0, 0, 0, 0, 0, 0};
        const int got = sscanf(e, "%d,%d,%d,%d,%d,%d,%d", &v[0], &v[1], &v[2], &v[3], &v[4], &v[5], &v[6]);
        if (got == 3) v[3] = v[0], v[4] = v[1], v[5] = v[2];
        auto ok = [](int r, int c, int t) {
            return r > 0 && r <= 16384 && c > 0 && c <= 16384 && (t == 64 || t == 128 || t == 256 || t == 512) &&
                   sweep_lds_bytes(r, c) <= 160 * 1024;
        };
        if ((got == 3 || got == 6 || got == 7) && ok(v[0], v[1], v[2]) && ok(v[3], v[4], v[5])) {
            for (int i = 0; i < 2; i++) cfg.rows[i] = v[3 * i], cfg.cap[i] = v[3 * i + 1], cfg.threads[i] = v[3 * i + 2];
            cfg.sub0 = got == 7 ? v[6] : 0;
        }
    }
    return cfg;
}

Analysis analyze(const HCsr &A11, const HCsr &B, const HCsr &C22) {
    auto t0 = std::chrono::steady_clock::now();
    Analysis an;
    an.Kp = assemble_kp(A11, B, C22);  // dimension checks of opLDL2.m:61-75
    an.n = A11.nrows, an.m = C22.nrows, an.N = an.n + an.m;
    std::vector<int32_t> perm = order_kp(an.Kp, an.n, &an.ordering);
    Factor f0 = ldl_factor(an.Kp, perm, 1);
    an.sweep = sweep_config();
    an.S = build_schedule(f0, an.sweep.rows[0], an.sweep.cap[0], an.sweep.rows[1], an.sweep.cap[1], an.sweep.sub0);
    an.F = relabel(f0, an.S);
    an.F0 = std::move(f0);
    an.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return an;
}

Precond *precond_create(Ctx &c, Analysis &&an) {
    auto t0 = std::chrono::steady_clock::now();
    auto pc = std::make_unique<Precond>();
    pc->ctx = &c;
    pc->n = an.n, pc->m = an.m, pc->N = an.N;
    pc->ordering = an.ordering;
    pc->Kp = std::move(an.Kp);
    pc->S = std::move(an.S);
    make_dmat(pc->Kp, pc->dKp);
    {
        const std::vector<int64_t> key(pc->S.order.begin(), pc->S.order.end());
        make_dfactor(an.F, pc->S, pc->dF, &key);
    }
    an.F = Factor();
    pc->F = std::move(an.F0);
    for (int i = 0; i < 2; i++)
        pc->dF.sweep_rows[i] = an.sweep.rows[i], pc->dF.sweep_cap[i] = an.sweep.cap[i],
        pc->dF.sweep_threads[i] = an.sweep.threads[i];
    pc->w.alloc(pc->N);
    pc->r.alloc(pc->N);
    pc->active.alloc(1);
    c.ensure_partials(std::max<size_t>(pc->dKp.nblk * 2, 4096));
    CPK_HIP(hipDeviceSynchronize());
    pc->ptime = an.seconds + std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return pc.release();
}

Precond *precond_create(Ctx &c, const HCsr &A11, const HCsr &B, const HCsr &C22) {
    return precond_create(c, analyze(A11, B, C22));
}

void Precond::apply(const double *x, int64_t neg_from, double *y, const int *run) {
    Ctx &c = *ctx;
    // y = op.LDL * x   (opLDL2.m:165-167)
    launch_sptrsv_fwd(c, dF, x, neg_from, w.p, run, nullptr);
    launch_sptrsv_bwd(c, dF, w.p, y, false, run, nullptr);
    if (nitref <= 0) return;
    const int64_t steps = (int64_t)nitref;
    if (force_itref != 0) {
        // every step runs; rNorm/xNorm and the final residual are dead
        for (int64_t s = 0; s < steps; s++) {
            launch_spmv_resid(c, dKp, x, neg_from, y, r.p, run, nullptr);  // r = x - op.A*y
            launch_sptrsv_fwd(c, dF, r.p, N, w.p, run, nullptr);         // dy = op.LDL*r
            launch_sptrsv_bwd(c, dF, w.p, y, true, run, nullptr);        // y = y + dy
        }
        return;
    }
    // data-dependent refinement: the predicate lives on the device, kernels test it
    launch_spmv_resid_norm(c, dKp, x, neg_from, y, r.p, itref_tol, active.p, run, nullptr);
    for (int64_t s = 0; s < steps; s++) {
        launch_sptrsv_fwd(c, dF, r.p, N, w.p, run, active.p);
        launch_sptrsv_bwd(c, dF, w.p, y, true, run, active.p);
        if (s + 1 < steps) launch_spmv_resid_norm(c, dKp, x, neg_from, y, r.p, itref_tol, active.p, run, active.p);
    }
}

double Precond::apply_bytes() const {
    // SpTRSV sweep over the strict factor (l entries): 12*l + 4*(N+1) + 16*N (vector in/out)
    // + 4*N (perm) ; backward adds D (8*N) and the scatter (8*N, +8*N when accumulating).
    const double l = (double)dF.nnz, Nn = (double)N;
    const double fwd = 12 * l + 4 * (Nn + 1) + 16 * Nn + 4 * Nn;
    const double bwd = 12 * l + 4 * (Nn + 1) + 16 * Nn + 4 * Nn + 8 * Nn + 8 * Nn;
    const double kp = 12 * (double)dKp.nnz + 4 * (Nn + 1) + 8 * Nn /*y*/ + 8 * Nn /*x*/ + 8 * Nn /*r*/;
    double b = fwd + bwd;
    const int64_t steps = nitref > 0 ? (int64_t)nitref : 0;
    b += steps * (kp + fwd + bwd + 8 * Nn);
    return b;
}

}  // namespace cpk
