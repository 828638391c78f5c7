"""DGP_RF — mirror of the reference's models/dgp.py:8-304 on the MI355X engine.

Same constructor, properties and methods; the state the reference keeps in tf.Variables lives in
one packed HBM engine (dgprf.Engine) and the layer/kernel objects hold views into it, so
`model.BNN.layers[1].W`, `model.W_mcmc`, `kernel.log_amplitude`, ... are live device tensors.
Compute (forward, likelihood, analytic backward, SGHMC/SGLD update, predictive scoring,
RMSprop preconditioner statistics) runs in libdgprf.so.
"""
import numpy as np
import torch

from dgprf import _native as N
from dgprf import engine as E
from dgprf.module import Module, rebind
from kernels import ARCKernel, RBFKernel
from layers import ARCLayer, GPLayer, RBFLayer
from likelihoods import Gaussian, Softmax
from utils import BNN_from_list, BNN_from_list_input_cat, log_gaussian


def whole_dataset(ds):
    """(X, Y) of an in-order, single-pass DeviceDataset (experiments/utils_dataset.py), else None.
    Rows of the DGP forward are independent, so scoring such a dataset batch by batch
    (models/regression_model.py:33-50, classification_model.py:49-60) and concatenating equals ONE
    forward over all its rows: one launch instead of one per batch (1e5 test rows at the driver's
    B = 200: 500 launches)."""
    from experiments.utils_dataset import DeviceDataset
    if isinstance(ds, DeviceDataset) and not ds.shuffled and not ds.repeated:
        B = ds.batch_size
        if not ds.drop_remainder or not B:
            return ds.X, ds.Y
        n = ds.n // B * B  # the batches drop the remainder rows
        return ds.X[:n], ds.Y[:n]
    return None


def _per_layer(v, L, what):
    """Scalar -> [v]*L, list -> list (models/dgp.py:34-43)."""
    if np.ndim(v) == 0:
        out = [int(v)] * L
    else:
        out = [int(x) for x in np.asarray(v).reshape(-1)]
    assert len(out) == L, f"Error in #{what}!"
    return out


class DGP_RF(Module):
    def __init__(self, d_in, d_out, n_hidden_layers=1, n_rf=20, n_gp=2, likelihood=Softmax(),
                 kernel_type_list=None, kernel_trainable=True, random_fixed=True, input_cat=False,
                 set_nonzero_mean=False, name=None):
        """
        :param d_in: Input dim
        :param d_out: Output dim
        :param n_hidden_layers: Number of hidden layers
        :param n_rf: Number of random features
        :param n_gp: Number of latent GPs in each layer
        :param likelihood: Likelihood class in the last layer
        :param kernel_type_list: kernel type list, set is_ard default True
        :param kernel_trainable: fix the trainable variables or not
        :param random_fixed: z fixed or not when feeding forward
        :param input_cat: concatenate input to each hidden layer except the final layer
        """
        super().__init__(name=name)
        self.d_in = d_in
        self.d_out = d_out
        self.n_hidden_layers = n_hidden_layers
        self.random_fixed = random_fixed
        self.input_cat = input_cat
        self.set_nonzero_mean = set_nonzero_mean
        self.kernel_trainable = kernel_trainable
        self.likelihood = likelihood
        self.n_rf = _per_layer(n_rf, n_hidden_layers, "random feature layers")
        self.n_gp = _per_layer(n_gp, n_hidden_layers, "hidden GP layers")
        if kernel_type_list is None:
            self.kernel_type_list = ['RBF' for _ in range(n_hidden_layers)]
        else:
            assert len(kernel_type_list) == n_hidden_layers, "Kernel type list's length does not match!"
            self.kernel_type_list = kernel_type_list
        self.kernel_list = self.transform_kernel_list()
        self.BNN = self.transformed_BNN()
        self._bind_engine()

    # ------------------------------------------------------------------ construction
    def transform_kernel_list(self):
        """models/dgp.py:74-91."""
        kernel_list = []
        if not self.input_cat:
            before_n_rf = [self.d_in] + self.n_gp[:-1]
        else:
            before_n_rf = [self.d_in] + [g + self.d_in for g in self.n_gp[:-1]]
        for i, kernel_type in enumerate(self.kernel_type_list):
            if kernel_type == 'RBF':
                kernel = RBFKernel(n_feature=before_n_rf[i], trainable=self.kernel_trainable,
                                   is_ard=True, length_scale=None)
            elif kernel_type == 'ARC':
                kernel = ARCKernel(n_feature=before_n_rf[i], trainable=self.kernel_trainable,
                                   is_ard=True, length_scale=None)
            else:
                raise NotImplementedError
            kernel_list.append(kernel)
        return kernel_list

    def transformed_BNN(self):
        """models/dgp.py:93-115."""
        bnn = []
        for l in range(self.n_hidden_layers):
            kernel_tmp = self.kernel_list[l]
            if kernel_tmp.kernel_type == "RBF":
                layer_Omega = RBFLayer(kernel_tmp, self.n_rf[l], random_fixed=self.random_fixed,
                                       set_nonzero_mean=self.set_nonzero_mean)
                layer_GP = GPLayer(2 * self.n_rf[l], self.n_gp[l])
            elif kernel_tmp.kernel_type == "ARC":
                layer_Omega = ARCLayer(kernel_tmp, self.n_rf[l], random_fixed=self.random_fixed,
                                       set_nonzero_mean=self.set_nonzero_mean)
                layer_GP = GPLayer(self.n_rf[l], self.n_gp[l])
            else:
                raise NotImplementedError
            bnn.extend([layer_Omega, layer_GP])
        if not self.input_cat:
            return BNN_from_list(bnn)
        return BNN_from_list_input_cat(bnn)

    def _lik_code(self):
        if isinstance(self.likelihood, Gaussian):
            return N.LIK_GAUSSIAN
        if isinstance(self.likelihood, Softmax):
            return N.LIK_SOFTMAX
        raise NotImplementedError  # models/dgp.py:158-159

    def _bind_engine(self):
        """Pack every layer's state into one Engine and rebind the objects to views of it."""
        kinds = [N.RBF if k == 'RBF' else N.ARC for k in self.kernel_type_list]
        # trainable hyper-parameter groups of full_bayesian=True (models/dgp.py:175-181)
        flags = 0
        if self.kernel_trainable:
            flags |= N.HYP_KERNEL
        if self.set_nonzero_mean:
            flags |= N.HYP_MEAN
        if isinstance(self.likelihood, Gaussian) and \
                getattr(self.likelihood.lik_log_var, "trainable", True):
            flags |= N.HYP_LIK
        spec = E.ModelSpec(self.d_in, self.d_out, kinds, self.n_rf, self.n_gp, self.input_cat,
                           self._lik_code(), hyp_flags=flags,
                           ard=[int(k.is_ard) for k in self.kernel_list])
        eng = E.Engine(spec, n_chains=1)
        for l in range(self.n_hidden_layers):
            rf, gp, k = self.BNN.layers[2 * l], self.BNN.layers[2 * l + 1], self.kernel_list[l]
            gp.W = rebind(gp.W, eng.W_view(l))
            k.log_amplitude = rebind(k.log_amplitude, eng.log_amp_view(l))
            k.log_inv_length_scale = rebind(k.log_inv_length_scale, eng.lis_view(l))
            rf.mean = rebind(rf.mean, eng.mean_view(l).view(-1, 1))
        self._engine = eng
        self._rebind_z()
        if isinstance(self.likelihood, Gaussian):
            # bound to its engine slot: full_bayesian=True updates it on the device
            self.likelihood.lik_log_var = rebind(self.likelihood.lik_log_var,
                                                 eng.lik_log_var_view())
            eng.lik_log_var_source = lambda: self.likelihood.lik_log_var
        self.BNN._model = self

    def _rebind_z(self):
        eng = self._engine
        for l in range(self.n_hidden_layers):
            rf = self.BNN.layers[2 * l]
            if hasattr(rf, "z") and rf.z.data_ptr() != eng.z_view(l).data_ptr():
                rf.z = rebind(rf.z, eng.z_view(l))
                rf.z.trainable = False

    # ------------------------------------------------------------------ properties
    @property
    def Likelihood_hyperparams(self):
        return list(self.likelihood.trainable_variables)

    @property
    def Omega_hyperparams(self):
        params = []
        for l in range(self.n_hidden_layers):
            params.extend(list(self.BNN.layers[2 * l].trainable_variables))
        return params

    @property
    def W_mcmc(self):
        return [self.BNN.layers[2 * l + 1].W for l in range(self.n_hidden_layers)]

    def assign_W(self, W_value_list):
        for gp_layer, W_value in zip(self.BNN.gp_layers, W_value_list):
            gp_layer.assign_W(W_value)

    # ------------------------------------------------------------------ device helpers
    def _omega_for_call(self):
        """Build Omega for this call; layers with random_fixed=False get fresh z (rf_layers.py:39-41)."""
        eng = self._engine
        fresh = [l for l in range(self.n_hidden_layers) if not self.BNN.layers[2 * l].random_fixed]
        if not fresh:
            # fixed z: Omega / c / sigma^2 only when z or a hyper-parameter changed since the last
            # build (engine version keys), as the graph path does
            eng.build_omega_if_stale()
            return None
        z = eng.z.clone()
        for l in fresh:
            pl = eng.layout
            o, n = pl.omega_off[l], pl.d[l] * pl.n_rf[l]
            E.normal(None, N.RNG_Z, out=z[o:o + n])
        om = torch.empty_like(eng.omega)
        eng.build_omega(z=z, omega=om)
        return om

    def _omega_and_z_for_call(self):
        """Like _omega_for_call, also returning the z that built Omega (full_bayesian=True
        differentiates through Omega = exp(lis) z + mean with that z)."""
        eng = self._engine
        fresh = [l for l in range(self.n_hidden_layers) if not self.BNN.layers[2 * l].random_fixed]
        if not fresh:
            eng.build_omega_if_stale()
            return None, None
        z = eng.z.clone()
        for l in fresh:
            pl = eng.layout
            o, n = pl.omega_off[l], pl.d[l] * pl.n_rf[l]
            E.normal(None, N.RNG_Z, out=z[o:o + n])
        om = torch.empty_like(eng.omega)
        eng.build_omega(z=z, omega=om)
        return om, z

    def _fused_forward(self, X):
        om = self._omega_for_call()
        out = self._engine.forward(X, f_out=True, omega=om, build=False)
        return out["F"][0][0]

    # ------------------------------------------------------------------ potential
    def log_likelihood(self, X, Y, allow_gradient_from_W=True):
        """log p(Y | X, all params) per row [N] (models/dgp.py:118-127)."""
        om = self._omega_for_call()
        return self._engine.forward(X, Y, logp=True, omega=om, build=False)["logp"][0]

    def prior_W(self):
        """log p(W) ~ N(0, I) (models/dgp.py:129-136)."""
        return self._engine.prior_w()[0]

    def prior_kernel_params(self):
        """models/dgp.py:138-147."""
        log_p = 0.
        for l in range(self.n_hidden_layers):
            k = self.BNN.layers[2 * l].kernel
            log_p = log_p + torch.sum(log_gaussian(k.log_amplitude, mean=0., var=1.))
            log_p = log_p + torch.sum(log_gaussian(k.log_inv_length_scale, mean=0., var=1.))
        return log_p

    def prior_likelihood_params(self):
        """models/dgp.py:149-159."""
        if isinstance(self.likelihood, Softmax):
            return 0.
        elif isinstance(self.likelihood, Gaussian):
            log_p = 0.
            for var in self.likelihood.trainable_variables:
                log_p = log_p + torch.sum(log_gaussian(var, mean=0., var=1.))
            return log_p
        else:
            raise NotImplementedError

    def U(self, X_batch, Y_batch, data_size, full_bayesian=False, allow_gradient_from_W=True):
        """Minibatch potential -(1/B) sum log p(y|x,w) - (1/N) log p(w)  (models/dgp.py:161-182)."""
        B = float(np.shape(X_batch)[0])
        N_ = float(data_size)
        ll = torch.sum(self.log_likelihood(X_batch, Y_batch)) / B
        if not full_bayesian:
            prior = self.prior_W() / N_ if allow_gradient_from_W else 0.
        else:
            assert allow_gradient_from_W == True, "Full Bayes should allow gradients from W!"  # noqa: E712
            prior = 0.
            for param in self.trainable_variables:
                prior = prior + torch.sum(log_gaussian(param, mean=0., var=1.)) / N_
        return -(prior + ll)

    # ------------------------------------------------------------------ sampler
    def _check_moments(self, full_bayesian=False):
        eng = self._engine
        if not eng.moments_ready or (full_bayesian and not eng.hyper_moments_ready):
            raise AssertionError("Trainable Params do not have attr moments!")  # dgp.py:208

    def _hyper_vars(self):
        """(variable, hmass slot, hyp offset, length) of every trainable hyper-parameter."""
        eng = self._engine
        by_off = {}
        for l in range(self.n_hidden_layers):
            k, rf = self.kernel_list[l], self.BNN.layers[2 * l]
            by_off[l] = k.log_amplitude
            by_off[eng.layout.lis_off[l]] = k.log_inv_length_scale
            by_off[eng.layout.mean_off[l]] = rf.mean
        if isinstance(self.likelihood, Gaussian):
            by_off[self.n_hidden_layers] = self.likelihood.lik_log_var
        return [(by_off[o], slot, o, n) for slot, o, n in eng.hyper_slots()]

    def _attach_sampler_attrs(self, full_bayesian=False):
        eng = self._engine
        for l, W in enumerate(self.W_mcmc):
            W.moments = eng.mom_view(l)
            W.M = eng.mass[0, l]
        if full_bayesian:
            for v, slot, o, n in self._hyper_vars():
                v.moments = eng.hmom[0, o:o + n].view(v.shape)
                v.M = eng.hmass[0, slot]

    def sgmcmc_update(self, X_batch, Y_batch, data_size, lr=0.01, momentum_decay=0.95,
                      resample_moments=False, temperature=1., full_bayesian=False):
        """One SGHMC (SGLD when momentum_decay = 0) step for W (models/dgp.py:184-216):
        m <- b m - h N dU/dW + sqrt(2(1-b) T M) xi,  W <- W + h m / M,  h = sqrt(lr / N).
        Runs as one fused forward/backward/update sequence of HIP kernels."""
        self._check_moments(full_bayesian)
        om, z = self._omega_and_z_for_call()
        self._engine.step(X_batch, Y_batch, data_size, lr, momentum_decay, temperature,
                          bool(resample_moments), build=False, omega=om, z=z,
                          full_bayes=bool(full_bayesian))

    def precond_update(self, ds, data_size, K_batches=32, full_bayesian=False,
                       precond_type='rmsprop', second_moment_centered=False):
        """Preconditioner M per W_l from K minibatch gradients (models/dgp.py:218-299):
        Welford mean/M2 on the device, mass = sqrt(mean(E[g^2]) + 1e-7) (or the centred
        variance), normalised by the smallest mass; momenta rescaled by sqrt(M)."""
        eng = self._engine
        if not eng.moments_ready:
            eng.init_moments()
            self._attach_sampler_attrs()
        if full_bayesian and not eng.hyper_moments_ready:
            eng.init_hyper_moments()  # vars = self.trainable_variables (models/dgp.py:230-240)
            self._attach_sampler_attrs(full_bayesian=True)
        if precond_type == 'identity':
            return None
        elif precond_type == 'rmsprop':
            L = self.n_hidden_layers
            hv = self._hyper_vars() if full_bayesian else []
            m_c = [torch.rsqrt(eng.mass[0, l]) * eng.mom_view(l) for l in range(L)]
            m_ch = [torch.rsqrt(eng.hmass[0, slot]) * eng.hmom[0, o:o + n]
                    for _, slot, o, n in hv]
            n_all = eng.layout.w_total + (eng.layout.hyp_total if full_bayesian else 0)
            mean = torch.zeros(eng.C, n_all, dtype=torch.float32, device=eng.dev)
            m2 = torch.zeros_like(mean)
            om, z = self._omega_and_z_for_call()
            k = 0
            for X_batch, Y_batch in ds:
                g = eng.grad(X_batch, Y_batch, data_size, build=False, omega=om, z=z,
                             full_bayes=bool(full_bayesian))
                k = k + 1
                eng.welford(g, mean, m2, k, full_bayes=bool(full_bayesian))
                if k == K_batches:
                    break
            assert k == K_batches, \
                f"Estimating M ends before we use {K_batches} batches, we actually use {k} batches!"
            est = eng.mass_estimate(mean, m2, K_batches, second_moment_centered,
                                    full_bayes=bool(full_bayesian))
            mass_est, hmass_est = (est if full_bayesian else (est, None))
            self._mass_estimate = mass_est[0]
            # scale the minimum estimated mass (over every variable) to one (dgp.py:289-296)
            mass_min = torch.min(mass_est[0])
            if hv:
                slots = torch.tensor([slot for _, slot, _, _ in hv], device=eng.dev)
                mass_min = torch.minimum(mass_min, torch.min(hmass_est[0, slots]))
            eng.mass.copy_(mass_est / mass_min)
            for l in range(L):
                eng.mom_view(l).copy_(torch.sqrt(eng.mass[0, l]) * m_c[l])
            for (_, slot, o, n), mc in zip(hv, m_ch):
                eng.hmass[0, slot] = hmass_est[0, slot] / mass_min
                eng.hmom[0, o:o + n] = torch.sqrt(eng.hmass[0, slot]) * mc
            return None
        else:
            raise NotImplementedError

    # ------------------------------------------------------------------ MCEM M-step
    def hyper_variables(self):
        """The variables MCEM_Q_maximizer watches: Omega_hyperparams + Likelihood_hyperparams
        (experiments/utils_training.py:342), in that order."""
        return list(self.Omega_hyperparams) + list(self.Likelihood_hyperparams)

    def Q_and_hyper_grads(self, W_samples, X_batch, Y_batch, data_size):
        """Q = (1/S) sum_s -U(W_s; full_bayesian=False, allow_gradient_from_W=False) and
        d(-Q)/d(hyper) for hyper_variables() (experiments/utils_training.py:339-358).

        -U without the W prior is the minibatch log-likelihood, so d(-Q)/d(hyper) is the device
        full-Bayes hyper-parameter gradient (k_step_bwd<FB> + the hyper reduction) minus its prior
        term hyper/N, averaged over the samples.  Each sample is assign_W'd first; the model is
        left holding the last one, like the reference's loop.  Returns (Q, grads)."""
        eng = self._engine
        pl = eng.layout
        X_batch = E.as_device(X_batch, eng.dev)
        Y_batch = E.as_device(Y_batch, eng.dev)
        B = float(X_batch.shape[0])
        acc = torch.zeros(pl.hyp_total, dtype=torch.float32, device=eng.dev)
        Q = torch.zeros((), dtype=torch.float32, device=eng.dev)
        S = 0
        for W_model_list in W_samples:
            self.assign_W(W_model_list)
            om, z = self._omega_and_z_for_call()
            g = eng.grad(X_batch, Y_batch, data_size, build=False, omega=om, z=z,
                         full_bayes=True)
            acc += g[0, pl.w_total:]
            Q += torch.sum(eng.forward(X_batch, Y_batch, logp=True, omega=om,
                                       build=False)["logp"][0]) / B
            S += 1
        acc /= S
        by_var = {id(v): (o, n) for v, _, o, n in self._hyper_vars()}
        grads = []
        for v in self.hyper_variables():
            o, n = by_var[id(v)]
            grads.append(acc[o:o + n].view(v.shape) - v.detach() / float(data_size))
        return Q / S, grads

    def collect_W(self):
        """{'W_l': copy of GP layer l's W} — the helper experiments/utils_training_demo.py:57,140
        calls (absent from the reference's models/)."""
        return {'W_' + str(i): W.detach().clone() for i, W in enumerate(self.W_mcmc)}

    def save(self, path):
        """Checkpoint the sampler: an .npz of every W, the momenta and masses, z, the
        kernel / likelihood hyper-parameters with their momenta and masses, the device step counter
        and the Philox key — the state the reference keeps only as live tf.Variable aliases
        (experiments/utils_training.py:226,306).  Resuming from it continues the chain bit-exactly."""
        np.savez(path, **self._engine.state_arrays())

    def load(self, path):
        """Restore a checkpoint written by save() into a model of the same construction."""
        with np.load(path, allow_pickle=False) as st:
            self._engine.load_state_arrays({k: st[k] for k in st.files})
        eng = self._engine
        if eng.moments_ready:
            self._attach_sampler_attrs(full_bayesian=eng.hyper_moments_ready)

    def set_random_fixed(self, state):
        for l in range(self.n_hidden_layers):
            self.BNN.layers[2 * l].set_random_fixed(state)
        self._rebind_z()

    # ------------------------------------------------------------------ engine-path sampling
    def run_sgmcmc(self, X_all, Y_all, data_size, n_steps, batch_size=200, lr=0.01,
                   momentum_decay=0.9, temperature=1., steps_per_graph=50, perm_seed=0,
                   schedule=None, start_step=0, cycle_length=1, resample_in_cycle_head=False,
                   full_bayesian=False):
        """Run n_steps sgmcmc_update steps with device-resident data: per-epoch shuffled,
        drop-remainder minibatches (experiments/utils_dataset.py:38-42) drawn on the device and
        `steps_per_graph` steps per hipGraph replay.  schedule='cyclical' applies the driver's
        burn-in + cosine schedule on the device (experiments/utils_training.py:41-61).
        full_bayesian=True also samples the trainable hyper-parameters (models/dgp.py:199-204)."""
        plan = self.sgmcmc_graphs(X_all, Y_all, data_size, n_steps, batch_size, lr,
                                  momentum_decay, temperature, steps_per_graph, perm_seed,
                                  schedule, start_step, cycle_length, resample_in_cycle_head,
                                  full_bayesian)
        for g, reps in plan:
            for _ in range(reps):
                g.launch()

    def sgmcmc_graphs(self, X_all, Y_all, data_size, n_steps, batch_size=200, lr=0.01,
                      momentum_decay=0.9, temperature=1., steps_per_graph=50, perm_seed=0,
                      schedule=None, start_step=0, cycle_length=1, resample_in_cycle_head=False,
                      full_bayesian=False):
        """The hipGraphs run_sgmcmc replays for these arguments, as [(graph, replays)]: a graph of
        spg = min(steps_per_graph, n_steps) steps replayed n_steps // spg times, then one graph of
        the remaining n_steps % spg steps.  Graphs are cached on the engine, so a caller that
        times run_sgmcmc captures them here first and the timed call only replays.  Omega, c and
        sigma^2 are built from the current hyper-parameters, so the graphs can be launched as they
        are returned."""
        self._check_moments(full_bayesian)
        eng = self._engine
        # random_fixed=False layers redraw z on every call (layers/rf_layers.py:39-41): on the
        # device, from the step's Philox counter, inside the graph
        fresh = sum(1 << l for l in range(self.n_hidden_layers)
                    if not self.BNN.layers[2 * l].random_fixed)
        if fresh and full_bayesian:
            raise NotImplementedError("run_sgmcmc with random_fixed=False needs full_bayesian=False")
        if full_bayesian:
            eng.hyper_epoch += 1  # these graphs rewrite hyp / Omega on the device
        X_all = E.as_device(X_all, eng.dev)
        Y_all = E.as_device(Y_all, eng.dev)
        if Y_all.dim() == 1:
            Y_all = Y_all[:, None]
        sched = N.SCHED_CYCLICAL if schedule == 'cyclical' else N.SCHED_CONST
        spg = max(1, min(int(steps_per_graph), int(n_steps)))
        mk = lambda k: eng.graph(X_all, Y_all, batch_size, data_size, lr, momentum_decay,
                                 temperature, k, sched, start_step, cycle_length,
                                 resample_in_cycle_head, perm_seed, full_bayes=bool(full_bayesian),
                                 fresh_z=fresh)
        # Omega, c, sigma^2 only when a hyper-parameter or z changed since the last build (and
        # with them a wide first layer's resident dataset projection, before graphs capture it)
        eng.build_omega_if_stale()
        full, rest = divmod(int(n_steps), spg)
        plan = [(mk(spg), full)] if full else []
        if rest:
            plan.append((mk(rest), 1))
        return plan
