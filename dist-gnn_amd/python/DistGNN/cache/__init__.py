from .cache_value import *  # noqa: F401,F403
