"""DistGNN -- counterpart of the reference's Python package (python/DistGNN/__init__.py:1-4)
on top of the MI355X-native `dgs`."""
from . import cache
from . import dataloading
from . import dist
import dgs as capi  # noqa: F401
