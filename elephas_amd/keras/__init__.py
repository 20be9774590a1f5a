"""``tensorflow.keras``-shaped namespace so reference scripts port by changing
the import prefix: ``from elephas_amd.keras.models import Sequential`` etc."""
from ..models import Model, Sequential  # noqa: F401
from . import activations, backend, initializers, losses, metrics, optimizers  # noqa: F401
from . import layers, models, utils, datasets, mixed_precision  # noqa: F401
from ..models.layers import Input  # noqa: F401
