import json, os, sys, torch
sys.path.insert(0, os.getcwd())
import bench
dev = torch.device("cuda:0")
one = [("layer", 16, 16, 32, 1, 3)]
for adc in (4, 1.5):
    r = bench.bench_layers(dev, one, 4, 64, adc, 50, 5)
    print(os.environ.get("CIMQ_TUNE_GX_RB"), adc, round(r["ms_fwd_bwd_graph"], 4), round(r["ms_fwd_bwd"], 4), flush=True)
