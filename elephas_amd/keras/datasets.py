from ..models.datasets import boston_housing, mnist  # noqa: F401
