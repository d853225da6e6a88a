from .dataloader import *  # noqa: F401,F403
from .load_dataset import *  # noqa: F401,F403
from .synthetic import *  # noqa: F401,F403
from .prefetch import *  # noqa: F401,F403
