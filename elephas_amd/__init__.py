"""elephas_amd: MI355X-native distributed training of Keras-style models with
the Elephas API (SparkModel, SparkMLlibModel, ElephasEstimator/Transformer,
parameter servers, RDD/DataFrame adapters, Keras-HDF5 checkpoints).

Compute: hand-written CDNA4 (gfx950) HIP kernels driven by a native C++
executor with hipGraph replay; distribution: one process per GPU over
torch.distributed (RCCL over xGMI) plus a device-resident parameter server.
"""
__version__ = "0.1.0"

from . import config  # noqa: F401
from .config import get_device, get_policy, set_device, set_engine, set_policy  # noqa: F401
