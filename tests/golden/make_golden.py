"""Generate the committed golden fixtures from files the reference holds.

Run once in the build container (it reads /root/reference, which does not
exist on the GPU box):  python tests/golden/make_golden.py

Outputs (all data, no reference source):
  preds_0_true_stats.json  region / block statistics of preds/0_true.png
                           (the reference's own 500x500x100spp forward render
                           of scenes/0.txt, path_trace.cu:200-234)
  preds_0_true.png         the PNG itself (the createGraph target image,
                           ipt.py:138 / inv_scene.h:52-57)
  temp_pt_materials.npy    temp.pt (30x3 per-triangle Kd, loaded with
                           torch.load(weights_only=True))
"""
import json
import os
import shutil

import numpy as np
from PIL import Image

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

REGIONS = {
    "global": [0, 500, 0, 500],
    "light": [95, 135, 200, 300],
    "back_wall": [200, 280, 200, 300],
    "floor": [420, 480, 150, 350],
    "cube_top": [310, 318, 225, 275],
    "cube_front": [340, 380, 225, 275],
    "cyan_wall_left": [150, 350, 20, 120],
    "orange_wall_right": [150, 350, 380, 480],
    "ceiling": [20, 60, 150, 350],
}


def stats(img):
    img = img.astype(np.float64)
    out = {"regions": {}}
    for k, (r0, r1, c0, c1) in REGIONS.items():
        out["regions"][k] = img[r0:r1, c0:c1].reshape(-1, 3).mean(0).tolist()
    out["block10_means"] = img.reshape(50, 10, 50, 10, 3).mean(axis=(1, 3)).round(4).tolist()
    out["max"] = float(img.max())
    return out


def main():
    true = np.asarray(Image.open(os.path.join(REF, "preds/0_true.png")).convert("RGB"))
    pred = np.asarray(Image.open(os.path.join(REF, "preds/0_pred.png")).convert("RGB"))
    s = stats(true)
    s["noise_mean_abs_true_vs_pred"] = float(np.abs(true.astype(np.float64) - pred).mean())
    s["source"] = "reference preds/0_true.png: scenes/0.txt, 500x500, 100 spp, unbounded bounces, time-seeded"
    with open(os.path.join(HERE, "preds_0_true_stats.json"), "w") as f:
        json.dump(s, f)
    shutil.copyfile(os.path.join(REF, "preds/0_true.png"), os.path.join(HERE, "preds_0_true.png"))
    import torch

    t = torch.load(os.path.join(REF, "temp.pt"), weights_only=True)
    np.save(os.path.join(HERE, "temp_pt_materials.npy"), t.detach().cpu().numpy().astype(np.float32))


if __name__ == "__main__":
    main()
