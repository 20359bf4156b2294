#!/usr/bin/env python3
"""Launch-to-launch noise of the launch-order feedback (GPU box): renders the
1/8 C3 shard eight times and saves every launch's per-group cost table
(rtg_diag_group_list) to gpurun_out/cost_noise.npz."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import rtg_amd as R
from conftest import load_scene
g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
c = g["configs"]["c3"]
sph, lg = load_scene("c3", c["spheres"], c["lights"])
W, H, S = c["W"], c["H"], c["stack_size"]
ctx = R.Context(0)
ctx.set_scene(sph, lg)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
st = torch.cuda.current_stream().cuda_stream
costs = []
for k in range(8):
    ctx.render_device(W, H, out.data_ptr(), stack_size=S, row_block=8, shard=0, n_shards=8, stream=st)
    torch.cuda.synchronize()
    d = ctx.diag_group_list()
    costs.append(d["cost"].copy())
    if k == 7:
        lst = d["list"].copy()
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "cost_noise.npz"), costs=np.array(costs), lst=lst)
print("ok", len(costs), costs[-1].shape)
