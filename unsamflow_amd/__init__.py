"""unsamflow_amd — MI355X-native (gfx950) cost-volume hot path of UnSAMFlow.

Drop-ins for the reference's hot-path operators:

* :class:`unsamflow_amd.correlation.Correlation` /
  :class:`unsamflow_amd.correlation.CorrelationFunction`
  (models/correlation_package/correlation.py)
* :class:`unsamflow_amd.correlation_native.Correlation`
  (models/correlation_native.py)
* :func:`unsamflow_amd.warp_utils.flow_warp` (utils/warp_utils.py)

all computed by hand-written HIP kernels in ``libunsamflow_hip.so`` (C ABI:
``include/unsamflow_hip.h``). The PWCLite model + unsupervised loss used by the
benchmark live in :mod:`unsamflow_amd.pwclite` and :mod:`unsamflow_amd.flow_loss`.
"""
from . import _lib  # noqa: F401
from .correlation import Correlation, CorrelationFunction  # noqa: F401
from .warp_utils import flow_warp  # noqa: F401

__all__ = ["Correlation", "CorrelationFunction", "flow_warp"]
