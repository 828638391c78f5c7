"""Synthetic workloads of BASELINE.json's configs.  No datasets are downloaded.

config1: 1-layer RBF n_rf=100, g=[1], D=1, mcycle-shaped N=133, SGLD, sigma^2=0.01 (full batch)
config2: 3-layer RBF n_rf=1024, g=[8,8,1], D=8, N=1e6, B=200, sigma^2=0.1, lr 0.01, beta 0.9, T=1
config3: 3-layer ARC n_rf=2048, g=[9,9,1], D=9, N=45,730 (protein-shaped), B=200
config4: 4-layer RBF n_rf=4096, g=[30,30,30,10], D=784, softmax, N=60,000, B=200
config5: 5-layer [RBF,ARC,RBF,ARC,RBF] n_rf=8192, g=[16,16,16,16,1], D=16, N=1e7, B=200
"""
import numpy as np
import torch

CONFIGS = {
    1: dict(kinds=["RBF"], n_rf=[100], n_gp=[1], d_in=1, d_out=1, n=133, n_test=100, batch=133,
            likelihood="gaussian", variance=0.01, lr=0.01, beta=0.0, T=1.0),
    2: dict(kinds=["RBF"] * 3, n_rf=[1024] * 3, n_gp=[8, 8, 1], d_in=8, d_out=1, n=1_000_000,
            n_test=100_000, batch=200, likelihood="gaussian", variance=0.1, lr=0.01, beta=0.9,
            T=1.0),
    3: dict(kinds=["ARC"] * 3, n_rf=[2048] * 3, n_gp=[9, 9, 1], d_in=9, d_out=1, n=45_730,
            n_test=4_573, batch=200, likelihood="gaussian", variance=0.1, lr=0.01, beta=0.9,
            T=1.0),
    4: dict(kinds=["RBF"] * 4, n_rf=[4096] * 4, n_gp=[30, 30, 30, 10], d_in=784, d_out=10,
            n=60_000, n_test=10_000, batch=200, likelihood="softmax", variance=None, lr=0.01,
            beta=0.9, T=1.0),
    5: dict(kinds=["RBF", "ARC", "RBF", "ARC", "RBF"], n_rf=[8192] * 5, n_gp=[16, 16, 16, 16, 1],
            d_in=16, d_out=1, n=10_000_000, n_test=1_000_000, batch=200, likelihood="gaussian",
            variance=0.1, lr=0.01, beta=0.9, T=1.0),
}


def regression_data(n, d, seed, device="cpu", a=None):
    """X ~ N(0, I); y = sin(X a) + 0.1 eps with a ~ N(0, I/d); y standardized."""
    g = torch.Generator(device=device).manual_seed(int(seed))
    X = torch.randn(n, d, generator=g, device=device, dtype=torch.float32)
    if a is None:
        ga = torch.Generator(device="cpu").manual_seed(12345)
        a = torch.randn(d, 1, generator=ga, dtype=torch.float32) / np.sqrt(d)
    a = a.to(device)
    y = torch.sin(X @ a) + 0.1 * torch.randn(n, 1, generator=g, device=device, dtype=torch.float32)
    y = (y - y.mean()) / y.std()
    return X, y, a


def classification_data(n, d, n_class, seed, device="cpu"):
    """X ~ U[-0.5, 0.5]^d (normalize_MNIST-like), labels uniform in {0..C-1} as float [n, 1]."""
    g = torch.Generator(device=device).manual_seed(int(seed))
    X = torch.rand(n, d, generator=g, device=device, dtype=torch.float32) - 0.5
    y = torch.randint(0, n_class, (n, 1), generator=g, device=device).to(torch.float32)
    return X, y


def mcycle_like(n=133, n_test=100, seed=0):
    """Synthetic motorcycle-shaped data (the real set comes from `pods`, absent here):
    x = sort(U(2.4, 57.6)), y = smooth + heteroscedastic noise, standardized."""
    rng = np.random.default_rng(seed)
    x = np.sort(rng.uniform(2.4, 57.6, n))
    smooth = np.where(x < 14, 0.0, -100 * np.sin((x - 14) / 9.0) * np.exp(-(x - 14) / 12.0))
    noise = rng.standard_normal(n) * (2.0 + 20.0 * (x > 14) * np.exp(-(x - 14) / 20.0))
    y = smooth + noise
    xm, xs = x.mean(), x.std()
    ym, ys = y.mean(), y.std()
    X = ((x - xm) / xs)[:, None].astype(np.float32)
    Y = ((y - ym) / ys)[:, None].astype(np.float32)
    Xt = ((np.linspace(-20.0, 80.0, n_test) - xm) / xs)[:, None].astype(np.float32)
    return X, Y, Xt, np.float32(ys)
