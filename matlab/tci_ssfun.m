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
%   later call with the same data, which is what mcmcstat does. The cache is keyed by a SHA-1
%   of the exact bytes of [t, y] (as the Python twin ssfun.py does) and a hit is confirmed by
%   comparing the stored bytes, so two cells never share a context. At most MAX_CTX contexts
%   are kept; the least recently used one is destroyed beyond that.
%   TCI_SSFUN() with no arguments destroys every cached context.
MAX_CTX = 64;
persistent cache stamp
if isempty(cache)
    cache = containers.Map('KeyType', 'char', 'ValueType', 'any');
    stamp = 0;
end
if nargin == 0
    ks = keys(cache);
    for i = 1:numel(ks)
        e = cache(ks{i});
        tci_mex('destroy', e.h);
    end
    cache = containers.Map('KeyType', 'char', 'ValueType', 'any');
    SS = [];
    return
end
t = double(data.xdata(:)');
y = double(data.ydata(:)');
n = numel(t);
bytes = typecast([t, y], 'uint8');
md = java.security.MessageDigest.getInstance('SHA-1');
md.update(bytes);
key = [construct, '|', sprintf('%d|', n), sprintf('%02x', typecast(md.digest(), 'uint8'))];
stamp = stamp + 1;
hit = false;
if isKey(cache, key)
    e = cache(key);               % containers.Map allows one level of indexing only
    hit = isequal(e.bytes, bytes);
    if ~hit                       % a SHA-1 collision: never reuse another cell's context
        tci_mex('destroy', e.h);
        remove(cache, key);
    end
end
if hit
    e.used = stamp;
    cache(key) = e;
else
    if cache.Count >= MAX_CTX     % evict the least recently used context
        ks = keys(cache);
        vals = values(cache, ks);
        used = cellfun(@(v) v.used, vals);
        [~, i] = min(used);
        old = cache(ks{i});
        tci_mex('destroy', old.h);
        remove(cache, ks{i});
    end
    cell_data = struct('time', t, 'MS2', y(1:n), 'PP7', y(n+1:end));
    e = struct('h', tci_mex('create', cell_data, construct, 0), 'bytes', bytes, 'used', stamp);
    cache(key) = e;
end
SS = tci_mex('ss', e.h, 1, x);
end
