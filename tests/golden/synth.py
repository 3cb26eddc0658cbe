"""Synthetic inputs shared by the golden generators and the tests that
regenerate them from a seed (torch's CPU generator is deterministic for a
given torch build, the same image here and on the GPU box).  Test data."""
import torch


def make_x(kind, N, n, gen):
    """Synthetic activations following benchmarks.py:31-79 make_X recipes."""
    if kind == "gaussian":
        X = torch.randn(N, n, generator=gen)
    elif kind == "ar1":  # gaussian_corr, AR(1) rho=0.9 (benchmarks.py:18-28, :50-54)
        idx = torch.arange(n)
        Sigma = 0.9 ** (idx[None, :] - idx[:, None]).abs().double()
        L = torch.linalg.cholesky(Sigma + 1e-6 * torch.eye(n, dtype=torch.float64)).float()
        X = torch.randn(N, n, generator=gen) @ L.T
    elif kind == "lognormal":
        X = torch.exp(0.5 * torch.randn(N, n, generator=gen))
    else:
        raise ValueError(kind)
    return X.half()  # real hook inputs are fp16 (quantize.py:127-130)
