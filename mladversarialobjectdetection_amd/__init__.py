"""MI355X-native adversarial-patch optimisation (the inner step of tiiuae/MLAdversarialObjectDetection's
attacker_train.py) — HIP kernels for gfx950 behind the C ABI in include/phx.h.

Public API mirrors the reference: EfficientDetVictim (util.get_victim_model), PatchAttacker,
Patcher, BrightnessMatcher (attacker.py / brightness_matcher.py).
"""
from ._lib import PhxError, load as load_library  # noqa: F401

__all__ = ["PhxError", "load_library", "EfficientDetVictim", "PatchAttacker", "Patcher", "BrightnessMatcher"]


def __getattr__(name):
    if name in ("EfficientDetVictim", "PatchAttacker", "Patcher", "BrightnessMatcher", "ReduceLROnPlateau"):
        from . import attacker
        return getattr(attacker, name)
    raise AttributeError(name)
