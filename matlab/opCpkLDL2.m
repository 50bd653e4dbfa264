classdef opCpkLDL2 < opSpot
%OPCPKLDL2  Drop-in for opLDL2 (ops/opLDL2.m) whose factorization and apply run on an
%           MI355X through libcpk (cpk_mex.c).
%
%   M = opCpkLDL2(A, B, C) represents inv([A B'; B C]) exactly as opLDL2(A, B, C) does:
%   same public properties (nitref, itref_tol, force_itref, residual_update), same setter
%   semantics (opLDL2.m:97-115), same multiply (opLDL2.m:161-188) and divide (:193-195).
%   The factor lives in HBM; M*z costs one PCIe round trip of z.
%
%   Spot operators are value objects.  The properties are therefore sent with every
%   multiply, so copies keep independent settings as they do with opLDL2.

   properties( SetAccess = private )
      nA            % leading block dimension
      nC            % trailing block dimension
      h             % cpkHandle: owns the device-side factorization
   end

   properties( SetAccess = public )
      nitref = 3
      itref_tol = 1.0e-8
      force_itref = false
      residual_update = false
   end

   methods
      function op = opCpkLDL2(A, B, C)
         if nargin ~= 3
            error('Invalid number of arguments.');
         end
         nA = size(A,1);  nC = size(C,1);
         if nA ~= size(A,2) || nC ~= size(C,2)
            error('First and last arguments must be square.');
         end
         if size(B,2) ~= nA || size(B,1) ~= nC
            error('Incompatible dimensions.');
         end
         op = op@opSpot('CpkLDL2', nA + nC, nA + nC);
         op.nA = nA;  op.nC = nC;
         op.h = cpkHandle(cpk_mex('pc_create', sparse(A), sparse(B), sparse(C)));
         op.sweepflag = true;
      end

      % setter semantics of opLDL2.m:97-115 (itref_tol has no setter there: the `sef` typo)
      function op = set.nitref(op, val)
         op.nitref = max(0, round(val));
      end
      function op = set.force_itref(op, val)
         if val ~= false && val ~= true
            op.force_itref = false;
         else
            op.force_itref = val;
         end
      end

      function opOut = transpose(op)
         opOut = op;
      end
      % conj / ctranspose (opLDL2.m:127-137): P*inv(conj(L)')*inv(conj(D))*inv(conj(L))*P'.  The
      % factors are real (complex systems are out of scope, opLDL2.m:80's cflag), so conj of the
      % operator is the operator and its conjugate transpose is its transpose: itself
      function opOut = conj(op)
         opOut = op;
      end
      function opOut = ctranspose(op)
         opOut = op;
      end
      % double (opLDL2.m:138-149): the dense matrix, one column op * e_i at a time -- the same
      % products the reference forms (each a device apply with the current properties)
      function x = double(op)
         n = op.nA + op.nC;
         e = zeros(n, 1);
         x = zeros(n);
         for i = 1 : n
            e(i) = 1;
            x(:, i) = op * e;
            e(i) = 0;
         end
      end
   end

   methods( Access = protected )
      function y = multiply(op, x, mode) %#ok<INUSD>
         cpk_mex('pc_set', op.h.id, struct('nitref', op.nitref, 'itref_tol', op.itref_tol, ...
                 'force_itref', double(op.force_itref), 'residual_update', double(op.residual_update)));
         y = cpk_mex('pc_apply', op.h.id, full(x));
      end
      function x = divide(op, b, mode) %#ok<INUSD>
         x = cpk_mex('pc_divide', op.h.id, full(b));
      end
   end
end
