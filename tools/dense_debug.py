"""Locate grad_x mismatches of the dense path (tests/test_gpu_parity.py RANDOM_CASES index)."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_gpu_parity as tp  # noqa: E402
from oracle import cim_oracle as co  # noqa: E402
import torch  # noqa: E402

idx = int(sys.argv[1])
cfg = tp.RANDOM_CASES[idx]
inp = tp._random_inputs(cfg, 7000 + idx)
st, pd = (cfg["s"], cfg["s"]), (cfg["p"], cfg["p"])
out, c = co.cim_forward(inp["x_q"], inp["w_q"], st, pd, (1, 1), cfg["ab"], cfg["abs"], cfg["wb"], cfg["wbs"],
                        cfg["adc"], cfg["xbar"], inp["binary_mask"], inp["alpha_q"], inp["sw"], inp["sa"],
                        False, inp["signed_act"], return_debug=True)
gx, gw, ga = co.cim_backward(c, inp["grad"])
res = tp.run_hip_function(torch.device("cuda:0"), cfg, inp)
d = np.abs(res["grad_x"] - gx).reshape(cfg["B"], cfg["C"])
bad = d > 1e-4 * (np.abs(gx).max())
print("bad rows", np.unique(np.nonzero(bad)[0])[:40], "count", bad.sum(), "of", bad.size)
print("bad cols", np.unique(np.nonzero(bad)[1])[:80])
dw = np.abs(res["grad_w"] - gw)
print("gw maxerr", dw.max(), "ref max", np.abs(gw).max())
print("ga maxerr", np.abs(res["grad_alpha"] - ga).max(), np.abs(ga).max())
