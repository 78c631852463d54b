function [MCMCresults, MCMCplot, MCMCchain] = tci_fit(data, varargin)
%TCI_FIT One dataset of TranscriptionCycleMCMC on an MI355X: every cell's DRAM chain in one launch.
%   [MCMCresults, MCMCplot, MCMCchain] = TCI_FIT(data, Name, Value, ...) replaces the body of the
%   parfor over cells of src/TranscriptionCycleMCMC.m:161-357 and the pruning of skipped cells
%   (:359-369) for ONE dataset. data is the dataset's struct array (fields time, MS2, PP7, name;
%   README.md:11-16), i.e. data_all(k).data at :146. The three outputs are the reference's structs
%   with the reference's fields, one element per fitted cell in cell order; save them as :371-378 do.
%
%   Where the reference runs one mcmcrun per cell in a parfor worker, with a MATLAB ssfun handle,
%   TCI_FIT sets every cell up exactly as :163-270 do, then makes ONE tci_mex('dram', ...) call:
%   mcmcstat's DRAM (proposals, bounds rejection, delayed rejection, covariance adaptation, the
%   Gaussian dR priors and the sigma^2 Gibbs update) for all cells at once on the GPU, every ssfun
%   evaluation a HIP kernel (matlab/tci_mex.cpp -> include/tci.h tci_dram_run). The summaries
%   (:276-303) come back reduced on the device; the forward model at the means (:307-309) is
%   tci_mex('forward', ..., 'raw').
%
%   Name-value options -- the reference's names and defaults (:36-45, :57-77):
%     'n_burn' (10000), 'n_steps' (20000), 'ratePriorWidth' (50), 't_start' (0), 't_end' (Inf),
%     'construct' ('P2P-MS2v5-LacZ-PP7v4', or a struct: see tci_mex 'create'),
%     'previous' ([]: no loadPrevious; else the MCMCresults struct array of an earlier fit -- the
%        hierarchical fit of :84-107, v fixed to previous mean_v +- 1e-5 (:193-198, :217-241),
%        ApprovedFits carried over (:345-347), cells without an entry skipped (:196-198))
%   and the GPU's own:
%     'device' (0), 'cells' (all: 1-based cell numbers to fit -- one GPU's share of a dataset),
%     'thin' (1 = every chain row, as the reference keeps them; k keeps rows 1, 1+k, ...; 0 keeps none
%        and MCMCchain is empty), 'seed' (0), 'engine' ('auto'), 'adapt_pmax' (0; see include/tci.h).
%
%   x0 is drawn from MATLAB's global RNG exactly as :200-208 draw it (rand, normrnd); the chains use
%   the device's Philox streams keyed by (seed, cell number), so a cell's chain does not depend on
%   which other cells are fitted with it or on which GPU. Sampling follows mcmcstat's published
%   algorithm, so a fit reproduces the reference's posterior, not MATLAB's random draws.
%
%   Spreading a dataset over the GPUs of a node (one MATLAB worker per GPU, e.g. spmd):
%       share = labindex:numlabs:numel(data);
%       [r, p, c] = tci_fit(data, 'cells', share, 'device', labindex - 1);
%   then concatenate the workers' outputs and sort them by cell_index.

p = inputParser;
p.addParameter('n_burn', 10000);
p.addParameter('n_steps', 20000);
p.addParameter('ratePriorWidth', 50);
p.addParameter('t_start', 0);
p.addParameter('t_end', Inf);
p.addParameter('construct', 'P2P-MS2v5-LacZ-PP7v4');
p.addParameter('previous', []);
p.addParameter('device', 0);
p.addParameter('cells', []);
p.addParameter('thin', 1);
p.addParameter('seed', 0);
p.addParameter('engine', 'auto');
p.addParameter('adapt_pmax', 0);
p.parse(varargin{:});
o = p.Results;
n_burn = o.n_burn;
n_steps = o.n_steps;
loadPrevious = ~isempty(o.previous);
N = length(data);                                   % :146
cellNums = o.cells;
if isempty(cellNums)
    cellNums = 1:N;
end

% ---- per-cell setup, as the parfor body does it (:163-255) --------------------------------------
setup = struct('cellNum', {}, 't', {}, 'MS2', {}, 'PP7', {}, 'x0', {}, 'lb', {}, 'ub', {}, 'mu', {}, ...
    'sig', {}, 'J0', {}, 'approved', {});
for cellNum = cellNums(:)'
    t = data(cellNum).time;                         % :163-167
    MS2 = data(cellNum).MS2;
    PP7 = data(cellNum).PP7;
    indStart = find(t >= o.t_start, 1, 'first');    % :170-175
    indEnd = find(t < o.t_end, 1, 'last');
    t = t(indStart:indEnd);
    MS2 = MS2(indStart:indEnd);
    PP7 = PP7(indStart:indEnd);
    approved = 0;                                   % :349
    if loadPrevious                                 % :193-198
        cellToload = find([o.previous.cell_index] == cellNum, 1);
        if isempty(cellToload) || isempty(o.previous(cellToload).mean_v) || ...
                ~isfinite(o.previous(cellToload).mean_v)
            continue
        end
        v0 = o.previous(cellToload).mean_v;
        approved = o.previous(cellToload).ApprovedFits;   % :345-347
    else
        v0 = 1+2*rand;                              % :200
    end
    ton0 = 4*rand;                                  % :202-208
    A0 = rand;
    tau0 = 4*rand;
    MS2_basal0 = 10;
    PP7_basal0 = 5;
    R0 = 15;
    dR0 = normrnd(0,3,1,length(t));
    x0 = [v0,tau0,ton0,MS2_basal0,PP7_basal0,A0,R0,dR0];   % :210
    if loadPrevious                                 % :217-221
        v_step = 0.0000001;
        v_lower = v0-0.00001;                       % :235-241
        v_upper = v0+0.00001;
    else
        v_step = 0.05;
        v_lower = 0;
        v_upper = 10;
    end
    ton_step = t(end)-t(end-1);                     % :222-231: diag(J0)
    J0 = [v_step, 0.1, ton_step, 1, 1, 0.05, 0.5, 0.5*ones(size(dR0))];
    n = length(t);                                  % :242-255: params {name, x0, lower, upper, mu, sig}
    lb = [v_lower, 0, 0, 0, 0, 0, 0, -30*ones(1,n)];
    ub = [v_upper, 20, 10, 50, 50, 1, 40, 30*ones(1,n)];
    mu = zeros(1, 7+n);
    sig = [Inf(1,7), o.ratePriorWidth*ones(1,n)];
    setup(end+1) = struct('cellNum', cellNum, 't', t, 'MS2', MS2, 'PP7', PP7, 'x0', x0, 'lb', lb, ...
        'ub', ub, 'mu', mu, 'sig', sig, 'J0', J0, 'approved', approved); %#ok<AGROW>
end
MCMCresults = struct('mean_v',{},'sigma_v',{},'mean_ton',{},'sigma_ton',{},...   % :149-157
    'mean_A',{},'sigma_A',{},'mean_tau',{},'sigma_tau',{},...
    'mean_MS2_basal',{},'sigma_MS2_basal',{},'mean_PP7_basal',{},'sigma_PP7_basal',{},'mean_R',{},...
    'sigma_R',{},'mean_dR',{},'sigma_dR',{},'mean_sigma',{},'sigma_sigma',{},...
    'cell_index',{},'ApprovedFits',{});
MCMCplot = struct('t_plot',{},'MS2_plot',{},'PP7_plot',{},'simMS2',{},'simPP7',{});
MCMCchain = struct('v_chain',{},'ton_chain',{},'A_chain',{},'tau_chain',{},...
    'MS2_basal_chain',{},'PP7_basal_chain',{},'R_chain',{},'dR_chain',{},'s2chain',{});
nc = numel(setup);
if nc == 0
    return
end

% ---- one context over the fitted cells, one column per chain (padding past a chain's 7 + N) -------
cellData = struct('time', {setup.t}, 'MS2', {setup.MS2}, 'PP7', {setup.PP7});
h = tci_mex('create', cellData, o.construct, o.device);
cleanup = onCleanup(@() tci_mex('destroy', h));
P = 7 + max(arrayfun(@(f) numel(f.t), setup));
X0 = zeros(P, nc); LB = -Inf(P, nc); UB = Inf(P, nc); MU = zeros(P, nc); SIG = Inf(P, nc); J0 = ones(P, nc);
for k = 1:nc
    m = numel(setup(k).x0);
    X0(1:m, k) = setup(k).x0;
    LB(1:m, k) = setup(k).lb;
    UB(1:m, k) = setup(k).ub;
    MU(1:m, k) = setup(k).mu;
    SIG(1:m, k) = setup(k).sig;
    J0(1:m, k) = setup(k).J0;
end
sigma2_0 = 1;                                       % :212, :259
options = struct('nsimu', n_steps, 'burnintime', n_burn, 'adaptint', 100, 'method', 'dram', ...  % :263-270
    'updatesigma', 1, 'verbosity', 0, 'stats_from', max(n_burn, 1), 'thin', o.thin, ...
    'seed', o.seed*1000003 + 20201028, 'engine', o.engine, 'adapt_pmax', o.adapt_pmax, ...
    'chain_keys', [setup.cellNum] - 1);
if o.thin > 0
    [results, chain, s2chain] = tci_mex('dram', h, 1:nc, X0, LB, UB, MU, SIG, J0, sigma2_0, options);  % :273
    rows = 1 + o.thin*(0:size(chain, 3)-1);         % chain rows kept: 1, 1+thin, ...
    sel = rows >= max(n_burn, 1);                   % chain(n_burn:end, :) (:276-283)
else
    results = tci_mex('dram', h, 1:nc, X0, LB, UB, MU, SIG, J0, sigma2_0, options);
end

% ---- summaries, forward model at the means, the three structs (:276-356) -------------------------
for k = 1:nc
    n = numel(setup(k).t);
    th = results.mean(1:7+n, k)';
    sd = results.std(1:7+n, k)';
    r.mean_v = th(1);          r.sigma_v = sd(1);   % :286-301 (std(., 1))
    r.mean_ton = th(3);        r.sigma_ton = sd(3);
    r.mean_A = th(6);          r.sigma_A = sd(6);
    r.mean_tau = th(2);        r.sigma_tau = sd(2);
    r.mean_MS2_basal = th(4);  r.sigma_MS2_basal = sd(4);
    r.mean_PP7_basal = th(5);  r.sigma_PP7_basal = sd(5);
    r.mean_R = th(7);          r.sigma_R = sd(7);
    r.mean_dR = th(8:end);     r.sigma_dR = sd(8:end);
    r.mean_sigma = results.sigma_mean(k);           % :302-303
    r.sigma_sigma = results.sigma_std(k);
    r.cell_index = setup(k).cellNum;                  % :343
    r.ApprovedFits = setup(k).approved;               % :345-350
    MCMCresults(k) = r;
    [simMS2, simPP7] = tci_mex('forward', h, k, th, 'raw');   % :307-309 (x mean_A inside)
    MCMCplot(k) = struct('t_plot', setup(k).t, 'MS2_plot', setup(k).MS2, 'PP7_plot', setup(k).PP7, ...
        'simMS2', simMS2, 'simPP7', simPP7);
    if o.thin > 0
        c = reshape(chain(1:7+n, k, sel), 7+n, [])';   % rows x P
        MCMCchain(k) = struct('v_chain', c(:,1), 'ton_chain', c(:,3), 'A_chain', c(:,6), ...
            'tau_chain', c(:,2), 'MS2_basal_chain', c(:,4), 'PP7_basal_chain', c(:,5), ...
            'R_chain', c(:,7), 'dR_chain', c(:,8:end), 's2chain', s2chain(k, :)');   % :315-323
    else
        MCMCchain(k) = struct('v_chain', [], 'ton_chain', [], 'A_chain', [], 'tau_chain', [], ...
            'MS2_basal_chain', [], 'PP7_basal_chain', [], 'R_chain', [], 'dR_chain', [], 's2chain', []);
    end
end
end
