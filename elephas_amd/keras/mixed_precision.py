from ..models.mixed_precision import global_policy, set_global_policy  # noqa: F401
