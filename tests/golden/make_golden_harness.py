"""Golden fixture for the training-harness parity test: the state_dict layout (key, shape,
dtype) of the reference's ResNet-20 after its ReplaceModuleTool swaps every conv for
Conv2dLSQCiM with the example prototxt's CiM settings (examples/classifier_cifar10/main_lsq.py,
utils/wrapper/replace_module.py), plus the nbits each replaced conv was built with.

Run in the build container only:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_harness.py
Writes tests/golden/harness_resnet20_cim_state.json (data only).
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF, _import_reference  # noqa: E402

KW = dict(nbits_w=3, nbits_a=3, nbits_alpha=8, wbitslice=1, abitslice=1, xbar=128, adcbits=1.5, signed_xbar=False,
          stochastic_quant=False)


def main():
    lsq = _import_reference()
    import models.cifar10 as cifar10  # noqa: E402  (the reference's, on sys.path from _import_reference)
    from utils.wrapper.replace_module import ReplaceModuleTool  # noqa: E402
    model = cifar10.__dict__["resnet20"](pretrained=False)
    tool = ReplaceModuleTool(model, {"Conv2d": [lsq.Conv2dLSQCiM]}, True, **KW)
    tool.replace()
    sd = model.state_dict()
    out = dict(kwargs=KW, state=[[k, list(v.shape), str(v.dtype)] for k, v in sd.items()],
               conv_bits=[[c.nbits_w, c.nbits_a] for c in tool.convs])
    with open(os.path.join(HERE, "harness_resnet20_cim_state.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", len(sd), "state_dict entries from", REF)


if __name__ == "__main__":
    main()
