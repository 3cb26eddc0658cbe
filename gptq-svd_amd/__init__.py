"""gptq_svd_amd -- MI355X-native TruncGPTQ per-layer solver (HIP kernels behind a C ABI).

The reference-compatible API lives in ``gptq_svd_amd.gptq_utils``.
"""
from . import _lib  # noqa: F401  (fails loudly if libtruncgptq.so is missing)
from . import export, harness  # noqa: F401
from .gptq_utils import (HessianAccumulator, Quantizer, gptq_fwrd, log_quantization_error,  # noqa
                         next_power_of_2, pack_quantized, process_hessian, process_hessian_alt,
                         triton_process_block, truncated_spectral_factor)

__version__ = "0.1.0"
