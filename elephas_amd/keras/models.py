from ..models import Model, Sequential, clone_model, load_model, model_from_config, model_from_json, save_model  # noqa: F401
