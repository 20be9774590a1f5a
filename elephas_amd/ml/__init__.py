from .adapter import *  # noqa: F401,F403
from .params import *  # noqa: F401,F403
