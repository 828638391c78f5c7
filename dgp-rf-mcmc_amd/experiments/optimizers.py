"""Adam with the update rule of tf.keras.optimizers.Adam — the optimizer the reference's MCEM
notebooks hand to MCEM_Q_maximizer (experiments/train_classification.ipynb,
train_regression_EM_*.ipynb: `optimizer = optimizers.Adam(learning_rate=...)`).

The watched hyper-parameters are a few dozen floats living in the engine's packed `hyp` buffer
(their tensors are views of it), so the update runs in place on the device and the next
sgmcmc_update rebuilds Omega from them.
"""
import math

import torch


class Adam:
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, name="Adam"):
        self.learning_rate = float(learning_rate)
        self.beta_1 = float(beta_1)
        self.beta_2 = float(beta_2)
        self.epsilon = float(epsilon)
        self.name = name
        self.iterations = 0
        self._slots = {}  # id(var) -> (var, m, v)

    def apply_gradients(self, grads_and_vars):
        """t += 1;  lr_t = lr sqrt(1 - b2^t) / (1 - b1^t);  m <- b1 m + (1 - b1) g;
        v <- b2 v + (1 - b2) g^2;  var <- var - lr_t m / (sqrt(v) + eps)."""
        pairs = [(g, v) for g, v in grads_and_vars if g is not None]
        self.iterations += 1
        t = self.iterations
        lr_t = self.learning_rate * math.sqrt(1.0 - self.beta_2 ** t) / (1.0 - self.beta_1 ** t)
        with torch.no_grad():
            for g, var in pairs:
                key = id(var)
                if key not in self._slots:
                    self._slots[key] = (var, torch.zeros_like(var), torch.zeros_like(var))
                _, m, v = self._slots[key]
                g = torch.as_tensor(g, dtype=var.dtype, device=var.device).reshape(var.shape)
                m.mul_(self.beta_1).add_(g, alpha=1.0 - self.beta_1)
                v.mul_(self.beta_2).addcmul_(g, g, value=1.0 - self.beta_2)
                var.sub_(lr_t * m / (torch.sqrt(v) + self.epsilon))
        return t

    def get_slot(self, var, name):
        _, m, v = self._slots[id(var)]
        return {"m": m, "v": v}[name]
