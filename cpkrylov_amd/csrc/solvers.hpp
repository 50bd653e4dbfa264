// solvers.hpp -- host entry points of the device solvers (solvers.hip).
#pragma once
#include "dev.hpp"

namespace cpk {
// [x, y, stats, flag] = method(b, A, C, M, opts): d_b (n), d_xy (N), AC = blkdiag(A, C)
void method_solve_device(Ctx &c, int method, const double *d_b, const DMat &AC, Precond &M, const cpk_opts *opts,
                         double *d_xy, cpk_stats *stats);
// reg_cpkrylov's shift + method + recovery (reg_cpkrylov.m:150-175): d_b (N), d_x (N)
// The shift's products: rows < n of Arows*xy0 (= A*xy0(1:n)) and of Btrows*xy0 restricted to
// columns >= bt_colmin (= B'*xy0(n+1:N)).
void reg_solve_device(Ctx &c, int method, const double *d_b, const DMat &AC, const DMat &Arows, const DMat &Btrows,
                      int64_t bt_colmin, Precond &M, const cpk_opts *opts, double *d_x, cpk_stats *stats);
int reg_shift_device(Ctx &c, const double *d_b, const DMat &Arows, const DMat &Btrows, int64_t bt_colmin, Precond &M,
                     double *d_b1, double *d_xy0);
void profile_kernels(Ctx &c, const DMat &AC, Precond &M, int reps, cpk_profile *out);
double method_bytes(int method, const DMat &AC, const Precond &M, int64_t iters, const cpk_opts *opts);
}  // namespace cpk
