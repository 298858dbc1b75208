"""neural_polar_decoder_amd -- MI355X-native batch Polar/PAC decoding hot path.

Python mirror of the reference's PolarCode / PAC / RNN_decoder / convNet surfaces over a ctypes
C-ABI (include/npd.h, libnpd.so) of hand-written gfx950 HIP kernels.  See DESIGN.md.
"""
from ._lib import NpdError, load as load_library  # noqa: F401
from .codes import pac_info_positions, polar_info_positions  # noqa: F401
from .pac_code import PAC  # noqa: F401
from .polar import PolarCode, reference_polar_code  # noqa: F401
from .utils import errors_ber, errors_bler, snr_db2sigma  # noqa: F401

__all__ = ["PolarCode", "PAC", "reference_polar_code", "errors_ber", "errors_bler", "snr_db2sigma",
           "polar_info_positions", "pac_info_positions", "NpdError", "load_library"]
