"""ssip — MI355X-native kernels and host runtime for the semi-supervised
ResNet image-classification path (train step, pseudo-labelling, evaluation,
embedding extraction) of Septimus4/semi-supervised-image-processing.

Compute runs in libssip_hip.so (hand-written gfx950 HIP kernels behind the
C ABI of include/ssip.h); this package is the host side.
"""
from . import ops  # noqa: F401
from ._lib import lib  # noqa: F401
from .resnet import DeviceImages, SSIPResNet, replace_fc  # noqa: F401

__all__ = ["ops", "lib", "SSIPResNet", "DeviceImages", "replace_fc"]
