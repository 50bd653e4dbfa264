classdef cpkHandle < handle
%CPKHANDLE  Owner of a libcpk preconditioner handle; frees it when the last copy of the
%           opCpkLDL2 value object that holds it goes away.
   properties( SetAccess = private )
      id
   end
   methods
      function obj = cpkHandle(id)
         obj.id = id;
      end
      function delete(obj)
         if ~isempty(obj.id)
            cpk_mex('pc_destroy', obj.id);
         end
      end
   end
end
