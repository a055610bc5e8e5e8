"""MI355X-native sparse bundle-adjustment core for InstantSfM (HIP kernels behind a C ABI, see include/insfm_ba.h)."""
from . import _capi  # noqa: F401
from .processors.bundle_adjustment import TorchBA  # noqa: F401
from .engine import BundleAdjuster  # noqa: F401

__all__ = ["TorchBA", "BundleAdjuster"]
