"""Run records in the reference's schema: ``quantization.log`` and
``results.json`` in a run's save directory, so the reference's own
post-processing (``extract_log.py``'s three patterns, ``run_benchmark.py``'s
results reader) consumes this build's runs unchanged.

Reference:
* log file and line format -- ``utils.py:12-28`` (``setup_logging``: root
  logger, ``[%(asctime)s] %(levelname)s: %(message)s``, ``%H:%M:%S``,
  ``<save_path>/quantization.log``);
* header / footer lines -- ``quantize.py:21-25, :51-56, :93, :254-256``;
* ``results.json`` -- ``quantize.py:62-66`` (``config`` = the argparse
  namespace, ``layer_stats``, ``metrics``), written at ``:281-284`` with
  ``metrics = {"total_time", "quantized_ppl"}`` (``total_time`` only when no
  evaluation ran, as after ``:257``).
"""
from __future__ import annotations

import json
import logging
import os
from typing import Any, Dict, List, Optional

__all__ = ["RunLog", "reference_config", "LOG_FORMAT", "LOG_DATEFMT"]

LOG_FORMAT = "[%(asctime)s] %(levelname)s: %(message)s"   # utils.py:25
LOG_DATEFMT = "%H:%M:%S"                                   # utils.py:26

# utils.py:31-125, in argparse order (the order ``vars(args)`` has)
_REF_DEFAULTS = dict(model_id="Qwen/Qwen3-8B", device="cuda", seed=42, dataset="wikitext2",
                     n_samples=128, seq_len=2048, batch_size=8, w_bits=4, group_size=-1,
                     sym=False, eps=1e-2, sketch_ratio=4.0, mode="svd",
                     threshold_method="mean_trimmed", actorder=False, damp_percent=0.01,
                     adaptive_eps=False, save_path="./output", no_save=False)


def reference_config(**kw) -> Dict[str, Any]:
    """The ``config`` block of results.json: the reference's argparse keys in
    their order with its defaults, overridden by ``kw`` (unknown keys are
    appended, so extra settings of this build stay visible)."""
    cfg = dict(_REF_DEFAULTS)
    cfg.update(kw)
    return cfg


def header(msg: str) -> None:          # quantize.py:21-22
    logging.info(f"\n{'=' * 20} {msg} {'=' * 20}")


def substep(msg: str) -> None:         # quantize.py:24-25
    logging.info(f"  [>] {msg}")


class RunLog:
    """Attach ``<save_path>/quantization.log`` to the root logger for the
    duration of a run and write ``results.json`` at its end.

        with RunLog(save_path, config) as rl:
            res = quantize_model(...)
            rl.finish(res["layer_stats"], res["total_time"], ppl)
    """

    def __init__(self, save_path: str, config: Dict[str, Any]):
        self.save_path = save_path
        self.config = config
        self._handler: Optional[logging.Handler] = None
        self._level = None

    def __enter__(self) -> "RunLog":
        os.makedirs(self.save_path, exist_ok=True)
        h = logging.FileHandler(os.path.join(self.save_path, "quantization.log"))
        h.setFormatter(logging.Formatter(LOG_FORMAT, datefmt=LOG_DATEFMT))
        root = logging.getLogger()
        self._level = root.level
        if root.level > logging.INFO or root.level == logging.NOTSET:
            root.setLevel(logging.INFO)
        root.addHandler(h)
        self._handler = h
        c = self.config
        header("INITIALIZING QUANTIZATION")                          # quantize.py:52-55
        logging.info(f"Model:  {c.get('model_id')}")
        logging.info(f"Mode:   {str(c.get('mode')).upper()}")
        logging.info(f"Params: Bits={c.get('w_bits')}, Group={c.get('group_size')}, "
                     f"Eps={c.get('eps')}")
        header(f"PIPELINE: {str(c.get('mode')).upper()}")            # quantize.py:93
        return self

    def finish(self, layer_stats: List[Dict[str, Any]], total_time: float,
               quantized_ppl: Optional[float] = None) -> Dict[str, Any]:
        header("COMPLETED")                                           # quantize.py:254-256
        logging.info(f"Total processing time: {total_time / 60:.2f} minutes")
        metrics: Dict[str, Any] = {"total_time": total_time}
        if quantized_ppl is not None:                                 # quantize.py:279-281
            logging.info(f"Final Quantized PPL: {quantized_ppl:.4f}")
            metrics["quantized_ppl"] = quantized_ppl
        log = {"config": self.config, "layer_stats": list(layer_stats), "metrics": metrics}
        with open(os.path.join(self.save_path, "results.json"), "w") as f:
            json.dump(log, f, indent=4)
        return log

    def __exit__(self, *exc) -> None:
        root = logging.getLogger()
        if self._handler is not None:
            root.removeHandler(self._handler)
            self._handler.close()
            self._handler = None
        if self._level is not None:
            root.setLevel(self._level)
