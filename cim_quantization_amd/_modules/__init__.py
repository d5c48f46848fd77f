"""Drop-in for the reference's ``models._modules`` namespace
(``import cim_quantization_amd._modules as my_nn``)."""
from ._quan_base import *  # noqa: F401,F403
from .lsq import *  # noqa: F401,F403
from .lsq import get_cim_output_signed  # noqa: F401
