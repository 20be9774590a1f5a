"""``tensorflow.keras.metrics``-shaped alias of ``elephas_amd.models.metrics``."""
from ..models.metrics import *  # noqa: F401,F403
