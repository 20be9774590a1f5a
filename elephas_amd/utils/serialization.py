"""Model <-> dict (reference elephas/utils/serialization.py:6-25)."""
from typing import Any, Dict


def model_to_dict(model) -> Dict[str, Any]:
    return dict(model=model.to_json(), weights=model.get_weights())


def dict_to_model(_dict: Dict[str, Any], custom_objects: Dict[str, Any] = None):
    from ..models import model_from_json
    if custom_objects is None:
        custom_objects = {}
    model = model_from_json(_dict["model"], custom_objects)
    model.set_weights(_dict["weights"])
    return model
