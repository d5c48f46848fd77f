"""cim_quantization_amd -- MI355X-native CiM partial-sum-quantised convolution.

Hot path of UtkarshSaxena1/CiM_Quantization (models/_modules/lsq.py) on hand-written
gfx950 HIP kernels behind a C ABI (include/cimq.h, libcimq.so), with the reference's
PyTorch module / autograd surface on top:

    import cim_quantization_amd._modules as my_nn      # instead of models._modules
    conv = my_nn.Conv2dLSQCiM(16, 16, 3, 1, 1, bias=False, nbits_w=3, nbits_a=3,
                              nbits_alpha=8, wbitslice=1, abitslice=1, xbar=128, adcbits=1.5)
"""
from . import _lib  # noqa: F401
from .functional import cim_conv2d_lsq, get_cim_output_signed  # noqa: F401

__version__ = "0.1.0"


def native_library_path() -> str:
    return _lib.LIB_PATH
