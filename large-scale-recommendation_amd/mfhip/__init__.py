"""mfhip -- MI355X-native DSGD / online matrix factorisation (host mirror of the reference API).

The compute path is libmfhip.so (hand-written HIP for gfx950 behind a C ABI, include/mfhip.h);
this package is the Python equivalent of the Scala entry points that bind it.
"""
from . import _lib, jvm, synth
from ._lib import MFError, MFNoDeviceError, device_count, version
from .context import Context, block_update
from .core import (FactorInitializer, FactorInitializerDescriptor, Factors, FactorUpdater, FactorVector,
                   ItemUpdate, MockFactorUpdater, PseudoRandomFactorInitializer,
                   PseudoRandomFactorInitializerDescriptor, RandomFactorInitializer,
                   RandomFactorInitializerDescriptor, Rating, SGDUpdater, UserUpdate)
from .dsgd import DSGDforMF, LearningRateMethod
from .online import OnlineMF
from .ratings_io import read_ratings

__all__ = [
    "MFError", "MFNoDeviceError", "device_count", "version", "Context", "block_update", "DSGDforMF",
    "LearningRateMethod", "OnlineMF", "Rating", "FactorVector", "Factors", "FactorUpdater", "SGDUpdater",
    "MockFactorUpdater", "FactorInitializer", "FactorInitializerDescriptor", "PseudoRandomFactorInitializer",
    "PseudoRandomFactorInitializerDescriptor", "RandomFactorInitializer", "RandomFactorInitializerDescriptor",
    "UserUpdate", "ItemUpdate", "read_ratings",
]
