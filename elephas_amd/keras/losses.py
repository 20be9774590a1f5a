"""``tensorflow.keras.losses``-shaped alias of ``elephas_amd.models.losses``."""
from ..models.losses import *  # noqa: F401,F403
