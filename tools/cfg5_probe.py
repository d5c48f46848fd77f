"""Per-kernel times of BASELINE cfg5 (QuantLinear 1024->1024 w4a4, B 4096) for each library in CIMQ_EXP_DIR
(tools/kernel_experiment.py builds): python tools/cfg5_probe.py <variant> ..."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from cim_quantization_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
for name in sys.argv[1:]:
    _lib._lib = _lib.load(os.path.join(os.environ.get("CIMQ_EXP_DIR", "exp"), f"libcimq_{name}.so"))
    r = bench.bench_cfg5(dev, 10, 2)
    k = r["kernel_roofs"]
    print(f"{name:16s} fwd_bwd {r['ms_fwd_bwd']:.4f} ms  fwd {r['ms_fwd']:.4f} ms  " +
          "  ".join(f"{n}={v['avg_launch_us']:.1f}us" for n, v in k.items()), flush=True)
