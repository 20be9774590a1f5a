from .server import *  # noqa: F401,F403
from .client import *  # noqa: F401,F403
