"""Softmax likelihood — mirror of the reference's likelihoods/softmax.py:4-22."""
import torch

from dgprf.module import Module


class Softmax(Module):
    def __init__(self):
        super().__init__()

    def log_prob(self, F, Y):
        """-sparse_softmax_cross_entropy(labels=int32(Y[:, 0]), logits=F)."""
        F = torch.as_tensor(F, dtype=torch.float32)
        Y = torch.as_tensor(Y, device=F.device)
        labels = Y[:, 0].to(torch.int64)
        return -torch.nn.functional.cross_entropy(F, labels, reduction="none")

    def predict_full(self, F):
        return torch.softmax(torch.as_tensor(F, dtype=torch.float32), dim=-1)
