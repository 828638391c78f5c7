"""RegressionDGP — mirror of the reference's models/regression_model.py:6-50."""
import torch

from likelihoods import Gaussian
from models.dgp import DGP_RF, whole_dataset


class RegressionDGP(DGP_RF):
    def __init__(self, d_in, d_out, n_hidden_layers=1, n_rf=20, n_gp=2, likelihood=Gaussian(),
                 kernel_type_list=None, kernel_trainable=True,
                 random_fixed=True, input_cat=False, set_nonzero_mean=False, name=None):
        super(RegressionDGP, self).__init__(d_in, d_out, n_hidden_layers=n_hidden_layers,
                                            n_rf=n_rf, n_gp=n_gp, likelihood=likelihood,
                                            kernel_type_list=kernel_type_list,
                                            kernel_trainable=kernel_trainable,
                                            random_fixed=random_fixed,
                                            input_cat=input_cat, set_nonzero_mean=set_nonzero_mean,
                                            name=name)

    def feed_forward(self, ds):
        """Output of the last batch before the likelihood (:16-22)."""
        y_batch_before_likelihood = None
        for x_batch, y_batch in ds:
            y_batch_before_likelihood = self.BNN(x_batch)
        return y_batch_before_likelihood

    def feed_forward_all_layers(self, X):
        """Every GP layer's output (:24-31).  The reference calls the layers sequentially without
        the input concatenation, which only type-checks when input_cat=False."""
        if self.input_cat:
            raise ValueError("feed_forward_all_layers does not apply input concatenation "
                             "(models/regression_model.py:24-31); use BNN(X)")
        om = self._omega_for_call()
        out = self._engine.forward(X, f_out="all", omega=om, build=False)
        return [F[0] for F in out["F"]]

    def eval_log_likelihood_and_se(self, ds):
        """
        :param ds: iterable X: [N, D_in]; Y: [N, D_out];
        :return: log likelihood log p(Y|F) [N] and square errors [N] (:33-50), one fused
                 forward + likelihood kernel per batch (one over the whole set for an in-order
                 DeviceDataset).
        """
        assert isinstance(self.likelihood, Gaussian), "The likelihood of the model is not Gaussian!"
        om = self._omega_for_call()
        whole = whole_dataset(ds)
        if whole is not None:  # every row in one fused launch (same rows, same order)
            out = self._engine.forward(*whole, logp=True, se=True, omega=om, build=False)
            return out["logp"][0], out["se"][0]
        log_p_all_data, se_all_data = [], []
        for x_batch, y_batch in ds:
            out = self._engine.forward(x_batch, y_batch, logp=True, se=True, omega=om, build=False)
            log_p_all_data.append(out["logp"][0])
            se_all_data.append(out["se"][0])
        return torch.cat(log_p_all_data, dim=0), torch.cat(se_all_data, dim=0)
