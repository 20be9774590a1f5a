"""Keras-style mixed-precision policy switch (``set_global_policy('mixed_bfloat16')``).

'mixed_bfloat16': bf16 MFMA operands / activations, fp32 accumulation, fp32
master weights and optimizer state.  'float32': exact-f32 MFMA everywhere."""
from .. import config


def set_global_policy(policy: str) -> None:
    config.set_policy(policy)


def global_policy() -> str:
    return config.get_policy()
