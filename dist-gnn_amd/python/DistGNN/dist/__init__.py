from .communicator import *  # noqa: F401,F403
from .watchdog import SetupWatchdog  # noqa: F401
