from ..models.utils import to_categorical  # noqa: F401
