"""``tensorflow.keras.backend``-shaped alias of ``elephas_amd.models.backend``."""
from ..models.backend import *  # noqa: F401,F403
