"""dgs -- MI355X-native drop-in for the reference's pybind11 module `dgs`
(CommediaJW/Dist-GNN src/pybind.cc:17-77): submodules `classes` and `ops` with the same
names, backed by the HIP/C++ library libdgs_amd.so (include/dgs_amd.h)."""
import torch  # noqa: F401  (must precede the native library: it shares torch's HIP runtime)

from . import _lib  # noqa: F401  (raises ImportError when the native library is missing)
from . import classes, ops  # noqa: F401

__version__ = _lib.lib.dgs_version().decode()
LIB_PATH = _lib.LIB_PATH
