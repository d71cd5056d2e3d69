"""dirt_amd -- MI355X-native differentiable rasteriser with the op surface of dirt.rasterise_ops.

The reference package re-exports its op wrappers at top level (dirt/__init__.py:1-2); so does this one.
"""
from .rasterise_ops import *  # noqa: F401,F403
from .rasterise_ops import __all__  # noqa: F401
from . import rasterise_ops  # noqa: F401
from . import lighting, matrices  # noqa: F401,E402
