"""A6 -- the relative prediction error (gptq_utils.py:275-291).

CPU: the oracle's restatement reproduces the value the REFERENCE logged on
every fixture carrying R_x (tests/golden/a6_metric.json, written by
make_metric_golden.py from the reference's own log_quantization_error).
GPU: the native fused FP32 MFMA pass (tg_pred_error) reproduces the same
values and the same log line (the format extract_log.py:20 parses), also on a
4096 x 4096 layer against an FP64 torch reference of the same formula."""
import json
import logging
import os

import numpy as np
import pytest

from oracle import oracle as o

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
A6 = json.load(open(os.path.join(GOLD, "a6_metric.json")))


def _fixture(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


@pytest.mark.parametrize("name", sorted(A6))
def test_oracle_metric_matches_reference(name):
    z = _fixture(name)
    v = o.relative_prediction_error(z["W"], z["final_W"], z["Rx"], z["perm"])
    # the reference logs 6 decimals
    assert abs(v - A6[name]["value"]) <= 5e-7 + 1e-6 * v, (v, A6[name])


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(A6))
def test_native_metric_matches_reference(name, caplog):
    import torch
    import gptq_svd_amd.gptq_utils as g
    z = _fixture(name)
    dev = torch.device("cuda")
    with caplog.at_level(logging.INFO):
        v = g.log_quantization_error(torch.from_numpy(z["W"]).to(dev),
                                     torch.from_numpy(z["final_W"]).to(dev),
                                     torch.from_numpy(z["Rx"]).to(dev),
                                     torch.from_numpy(z["perm"]).to(dev))
    ref = o.relative_prediction_error(z["W"], z["final_W"], z["Rx"], z["perm"])
    assert abs(v - ref) <= 1e-5 * ref, (v, ref)
    lines = [r.getMessage() for r in caplog.records if "Relative prediction error" in r.getMessage()]
    assert lines and lines[-1] == A6[name]["line"], (lines, A6[name]["line"])


@pytest.mark.gpu
def test_native_metric_full_size():
    """4096 x 4096 layer, k = 3058 trapezoidal R_x, against FP64 torch."""
    import torch
    import gptq_svd_amd.gptq_utils as g
    dev = torch.device("cuda")
    gen = torch.Generator(device="cpu").manual_seed(7)
    m = n = 4096
    k = 3058
    W = torch.randn(m, n, generator=gen).to(dev)
    Wq = (W + 0.01 * torch.randn(m, n, generator=gen).to(dev))
    Rx = torch.triu(torch.randn(k, n, generator=gen, dtype=torch.float64)).to(dev)
    perm = torch.randperm(n, generator=gen).to(dev)
    v = g.log_quantization_error(W, Wq, Rx, perm)
    R = Rx.float().double()
    Wo = W[:, perm].double()
    ref = (torch.linalg.norm((Wo - Wq[:, perm].double()) @ R.T) / torch.linalg.norm(Wo @ R.T)).item()
    assert abs(v - ref) <= 1e-5 * ref, (v, ref)
