function [x, stats, flag] = reg_cpkrylov_gpu(method, b, A, B, C, G, opts)
%REG_CPKRYLOV_GPU  reg_cpkrylov (reg_cpkrylov.m:1-180) with the factorization, the shift,
%   the Krylov loop and the recovery all on the MI355X (libcpk through cpk_mex).
%   method is a function handle (@cpminres, ...) or its name; arguments and outputs are
%   those of reg_cpkrylov.  For the operator-only drop-in (MATLAB loops, GPU M*z), replace
%   opLDL2 by opCpkLDL2 at reg_cpkrylov.m:131 instead.
   if nargin < 6
      error('reg_cpkrylov: not enough inputs');
   end
   if nargin < 7
      opts = struct();
   end
   [x, stats, flag] = cpk_mex('reg_solve', method, full(b), sparse(A), sparse(B), sparse(C), ...
                              sparse(G), opts);
end
