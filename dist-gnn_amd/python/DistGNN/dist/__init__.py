from .communicator import *  # noqa: F401,F403
