"""tropical -- MI355X-native drop-in for the ``tropical`` package of
seonghunn/tropical-nerf.pytorch (polyhedral complex derivation from
piecewise trilinear networks).

Surface kept from the reference: ``tropical.TropicalHashGrid``,
``tropical.subpoly.subpoly`` / ``subpoly_``, ``tropical.stanford.model.Net``
and ``python -m tropical.stanford.train``.  Compute runs in hand-written
gfx950 HIP kernels (libtropical_hip.so, C ABI include/tropical_hip.h).
"""
import functools
import warnings

from .tropical import TropicalHashGrid, compute_marks, level_meta  # noqa: F401

__version__ = "0.1.0"


def deprecated(reason=None):
    """The reference's decorator (tropical/__init__.py:12-34)."""
    def decorator(func):
        @functools.wraps(func)
        def wrapped(*args, **kwargs):
            msg = f"Function '{func.__name__}' is deprecated."
            if reason:
                msg += f" Reason: {reason}"
            warnings.warn(msg, category=DeprecationWarning, stacklevel=2)
            return func(*args, **kwargs)
        return wrapped
    if callable(reason):
        fn, reason = reason, None
        return decorator(fn)
    return decorator
