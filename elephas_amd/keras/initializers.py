"""``tensorflow.keras.initializers``-shaped alias of ``elephas_amd.models.initializers``."""
from ..models.initializers import *  # noqa: F401,F403
