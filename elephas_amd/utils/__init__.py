from .functional_utils import *  # noqa: F401,F403
from .rdd_utils import *  # noqa: F401,F403
from .serialization import *  # noqa: F401,F403
from .sockets import *  # noqa: F401,F403
from .rwlock import *  # noqa: F401,F403
