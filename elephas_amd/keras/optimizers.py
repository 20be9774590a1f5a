"""``tensorflow.keras.optimizers``-shaped alias of ``elephas_amd.models.optimizers``."""
from ..models.optimizers import *  # noqa: F401,F403
