function SS = tci_ssfun(construct, data, x)
%TCI_SSFUN Drop-in replacement for SumofSquaresFunction_TranscriptionCycleMCMC on an MI355X.
%   SS = TCI_SSFUN(construct, data, x) has the signature, arguments and result of
%   SumofSquaresFunction_TranscriptionCycleMCMC(construct,data,x)
%   (src/SumofSquaresFunction_TranscriptionCycleMCMC.m:1): data.xdata is the time vector,
%   data.ydata = [MS2, PP7], x = [v,tau,ton,MS2_basal,PP7_basal,A,R,dR]. The SS is computed by the
%   HIP kernel behind tci_mex (matlab/tci_mex.cpp -> include/tci.h).
%
%   Use it exactly where TranscriptionCycleMCMC.m:186 builds the mcmcstat handle:
%       ssfun = @(x,data) tci_ssfun(construct,data,x);
%
%   A device context is created once per distinct (construct, data) in each MATLAB process
%   (parfor workers are separate processes and each keep their own) and reused for every
%   later call with the same data, which is what mcmcstat does.
persistent cache
if isempty(cache)
    cache = containers.Map('KeyType', 'char', 'ValueType', 'any');
end
t = data.xdata(:)';
y = data.ydata(:)';
n = numel(t);
key = sprintf('%s|%d|%s', construct, n, sprintf('%bx', [sum(t), sum(t .* (1:n)), ...
    sum(y(~isnan(y))), sum(isnan(y))]));
if isKey(cache, key)
    h = cache(key);
else
    cell_data = struct('time', t, 'MS2', y(1:n), 'PP7', y(n+1:end));
    h = tci_mex('create', cell_data, construct, 0);
    cache(key) = h;
end
SS = tci_mex('ss', h, 1, x);
end
