from .adapter import *  # noqa: F401,F403
