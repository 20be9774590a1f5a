"""elephas_amd: MI355X-native distributed training of Keras-style models with
the Elephas API (SparkModel, SparkMLlibModel, ElephasEstimator/Transformer,
parameter servers, RDD/DataFrame adapters, Keras-HDF5 checkpoints).

Compute: hand-written CDNA4 (gfx950) HIP kernels driven by a native C++
executor with hipGraph replay; distribution: one process per GPU over
torch.distributed (RCCL over xGMI) plus a device-resident parameter server.
"""
__version__ = "0.1.0"

import os as _os

# Hardware queues per process (read by the HIP runtime once, when its library loads --
# so this only takes effect when elephas_amd is imported before torch). HIP's default
# of 4 maps the streams beyond the fourth onto shared queues, where they run one after
# another: the asynchronous / hogwild worker groups (one stream each) measured 7.5 M
# samples/s with 4 queues, 9.7 M with 8 and 15.8 M with 16 (8 groups, MNIST,
# profiles/README.md). Raised to ELEPHAS_AMD_HW_QUEUES (default 16) when lower; 0 leaves it.
_hwq = int(_os.environ.get("ELEPHAS_AMD_HW_QUEUES", "16") or 0)
if _hwq > 0 and int(_os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _hwq:
    import sys as _sys
    if "torch" in _sys.modules:
        # torch loaded the HIP runtime already: the setting below comes too late
        import warnings as _warnings
        _warnings.warn(
            f"elephas_amd was imported after torch: the HIP runtime already runs with "
            f"GPU_MAX_HW_QUEUES={_os.environ.get('GPU_MAX_HW_QUEUES', '4')}, so the asynchronous worker "
            f"groups' streams will share hardware queues (measured 7.5 M vs 16 M samples/s with 16). "
            f"Import elephas_amd before torch, or export GPU_MAX_HW_QUEUES={min(32, _hwq)}.",
            RuntimeWarning, stacklevel=2)
    _os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, _hwq))

from . import config  # noqa: F401
from .config import get_device, get_policy, set_device, set_engine, set_policy  # noqa: F401
