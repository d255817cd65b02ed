"""MI355X-native multi-view-stereo depth engine (behaviour of kianoosh-j/CL_MultiView_Stereo).

Hot path: SLIC superpixels -> plane-sweep photo-consistency (reference SAD
superpixel sweep, per-pixel SAD parity sweep, build-defined per-pixel NCC cost
volume + WTA) -> superpixel-plane refinement -> cross-view consistency filter,
all as hand-written HIP kernels for gfx950 behind the C-ABI in include/mvs.h.
"""
from . import params, synth  # noqa: F401

__all__ = ["params", "synth"]
__version__ = "0.1.0"
