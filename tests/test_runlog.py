"""Run records in the reference's schema (runlog.py): ``quantization.log``
parses with the reference's log scraper patterns and ``results.json`` has the
reference's keys (quantize.py:62-66, :281-284; utils.py:12-28).

CPU only: the harness runs a tiny OPT with the oracle standing in for the
HIP solver (as tests/test_dist_harness.py), so what is checked is the
record-keeping, not the numerics.  The patterns are extract_log.py:19-21
restated."""
import json
import logging
import re

import numpy as np
import torch

from test_dist_harness import _patch, tiny_opt

RUN_PATTERN = re.compile(r"INFO:\s+Params:\s+(.+)")                       # extract_log.py:19
ERROR_PATTERN = re.compile(r"Relative prediction error:\s+([\d\.]+)")     # extract_log.py:20
MODULE_PATTERN = re.compile(r"INFO:\s+([\w\.]+)\s+\|\s+Rank:")           # extract_log.py:21


def scrape(path):
    """extract_log.parse_single_log's state machine (extract_log.py:11-57)."""
    rows, run_id, err = [], "Unknown_Run", None
    for line in open(path):
        line = line.strip()
        m = RUN_PATTERN.search(line)
        if m:
            run_id = m.group(1)
            continue
        m = ERROR_PATTERN.search(line)
        if m:
            err = float(m.group(1))
            continue
        m = MODULE_PATTERN.search(line)
        if m and err is not None:
            rows.append((run_id, m.group(1).split(".")[-1], err))
            err = None
    return rows


def test_run_records_parse_like_the_reference(tmp_path, monkeypatch):
    import gptq_svd_amd.harness as harness
    from oracle import oracle as o
    for nm in ("HessianAccumulator", "process_hessian_alt", "gptq_fwrd"):
        monkeypatch.setattr(harness, nm, getattr(harness, nm))  # restored after the test
    hs = []
    _patch(harness, hs)
    fwrd = harness.gptq_fwrd

    def fwrd_metric(W, R, q, perm, block_size=1024, use_triton=True, R_x=None):
        Wq, k = fwrd(W, R, q, perm, block_size, use_triton)
        if R_x is not None:   # gptq_utils.py:290-291's line, value from the oracle
            e = o.relative_prediction_error(W.float().numpy(), Wq.numpy(), R_x.numpy(),
                                            perm.numpy())
            logging.info(f"   [Metric] Relative prediction error: {e:.6f}")
        return Wq, k

    harness.gptq_fwrd = fwrd_metric
    gen = torch.Generator().manual_seed(3)
    ids = [torch.randint(0, 256, (1, 16), generator=gen) for _ in range(4)]
    model = tiny_opt(2)
    res = harness.quantize_model(model, ids, mode="eigh", w_bits=4, group_size=64, sym=False,
                                 eps=1e-3, threshold_method="energy", batch_size=2, device="cpu",
                                 save_path=str(tmp_path), run_config={"model_id": "tiny-opt"})
    log = tmp_path / "quantization.log"
    rows = scrape(log)
    # one (module, error) row per quantised linear: 2 layers x 6 OPT linears
    assert len(rows) == len(res["layer_stats"]) == 12
    assert {r[0] for r in rows} == {"Bits=4, Group=64, Eps=0.001"}
    assert [r[1] for r in rows[:6]] == ["q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"]
    assert all(0.0 <= r[2] < 1.0 for r in rows)
    text = log.read_text()
    assert re.search(r"^\[\d\d:\d\d:\d\d\] INFO: Model:  tiny-opt$", text, re.M)
    assert "==================== COMPLETED ====================" in text
    assert re.search(r"INFO: Total processing time: [\d.]+ minutes", text)
    rj = json.loads((tmp_path / "results.json").read_text())
    assert list(rj) == ["config", "layer_stats", "metrics"]
    cfg = rj["config"]
    assert list(cfg)[:19] == ["model_id", "device", "seed", "dataset", "n_samples", "seq_len",
                              "batch_size", "w_bits", "group_size", "sym", "eps", "sketch_ratio",
                              "mode", "threshold_method", "actorder", "damp_percent",
                              "adaptive_eps", "save_path", "no_save"]
    assert (cfg["model_id"], cfg["mode"], cfg["n_samples"], cfg["seq_len"]) == ("tiny-opt", "eigh",
                                                                               4, 16)
    assert (cfg["w_bits"], cfg["group_size"], cfg["eps"]) == (4, 64, 1e-3)
    assert rj["layer_stats"][0]["name"] == "layer_0.self_attn.q_proj"
    assert all(isinstance(s["rank"], int) and s["time"] >= 0 for s in rj["layer_stats"])
    assert set(rj["metrics"]) == {"total_time"} and rj["metrics"]["total_time"] > 0
    # the file handler is detached after the run
    assert not any(getattr(h, "baseFilename", "").endswith("quantization.log")
                   for h in logging.getLogger().handlers)


def test_results_with_ppl(tmp_path):
    from gptq_svd_amd import runlog
    cfg = runlog.reference_config(mode="eigh", w_bits=3, sym=True)
    with runlog.RunLog(str(tmp_path), cfg) as rl:
        rl.finish([{"name": "layer_0.mlp.down_proj", "rank": 12252, "time": 5.29}], 1534.27,
                  8.645248413085938)
    rj = json.loads((tmp_path / "results.json").read_text())
    assert rj["metrics"] == {"total_time": 1534.27, "quantized_ppl": 8.645248413085938}
    text = (tmp_path / "quantization.log").read_text()
    assert "INFO: Final Quantized PPL: 8.6452" in text
    assert "INFO: Params: Bits=3, Group=-1, Eps=0.01" in text
    assert np.isclose(float(re.search(r"Total processing time: ([\d.]+)", text).group(1)), 25.57)
