"""ClassificationDGP — mirror of the reference's models/classification_model.py:7-60."""
import torch

from likelihoods import Softmax
from models.dgp import DGP_RF, whole_dataset


class ClassificationDGP(DGP_RF):
    def __init__(self, d_in, d_out, n_hidden_layers=1, n_rf=30, n_gp=10, likelihood=Softmax(),
                 kernel_type_list=None, random_fixed=True, input_cat=False,
                 kernel_trainable=True, set_nonzero_mean=False, name=None):
        super(ClassificationDGP, self).__init__(d_in, d_out, n_hidden_layers=n_hidden_layers,
                                                n_rf=n_rf, n_gp=n_gp, likelihood=likelihood,
                                                kernel_type_list=kernel_type_list,
                                                input_cat=input_cat, random_fixed=random_fixed,
                                                kernel_trainable=kernel_trainable,
                                                set_nonzero_mean=set_nonzero_mean, name=name)

    def eval_batch_accuracy(self, X_batch, Y_batch):
        """Accuracy of one sample of the params on a batch (:17-30)."""
        out = self.BNN(X_batch)
        out = self.likelihood.predict_full(out)
        predicts = torch.argmax(out, dim=-1).to(torch.float32)
        labels = torch.as_tensor(Y_batch, dtype=torch.float32, device=out.device).reshape(-1)
        right = torch.sum((predicts == labels).to(torch.float32))
        return right / float(out.shape[0])

    def eval_all_accuracy(self, ds_test):
        right = 0.
        test_size = 0.
        for img_batch, label_batch in ds_test:
            batch_size = float(len(img_batch))
            right += self.eval_batch_accuracy(img_batch, label_batch) * batch_size
            test_size += batch_size
        return right / test_size

    def eval_test_free_random(self, ds_test):
        self.BNN.set_random_fixed(False)
        acc = self.eval_all_accuracy(ds_test)
        self.BNN.set_random_fixed(True)
        return acc

    def eval_log_likelihood(self, ds):
        """log p(Y|F) per test point [N] (:49-60), fused forward + softmax likelihood kernel."""
        om = self._omega_for_call()
        whole = whole_dataset(ds)
        if whole is not None:  # every row in one fused launch (same rows, same order)
            return self._engine.forward(*whole, logp=True, omega=om, build=False)["logp"][0]
        log_p_all_data = []
        for x_batch, y_batch in ds:
            out = self._engine.forward(x_batch, y_batch, logp=True, omega=om, build=False)
            log_p_all_data.append(out["logp"][0])
        return torch.cat(log_p_all_data, dim=0)
