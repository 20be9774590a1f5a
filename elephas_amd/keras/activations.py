"""``tensorflow.keras.activations``-shaped alias of ``elephas_amd.models.activations``."""
from ..models.activations import *  # noqa: F401,F403
