from ..models.layers import Activation, Dense, Dropout, Flatten, Input, InputLayer, Layer  # noqa: F401
