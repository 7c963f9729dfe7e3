"""C1 golden vectors (SURVEY.md §8(c) "CPU-oracle golden vectors at C1"):
Cornell box (first object of scenes/0.txt), 128x128, 8 spp, max_bounces=2,
seed 0, rendered by the CPU oracle (oracle/ipt_oracle.c).  Stores the HDR
image (per-pixel mean in sample order), the u8 tonemap and the ray-cast count.

This pins the oracle against regressions and gives the GPU path a fixed
bitwise target; reference parity of the oracle itself is pinned statistically
by preds_0_true_stats.json.

    python tests/golden/make_c1_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib  # noqa: E402
from conftest import CORNELL  # noqa: E402

W, H, SPP, MB, SEED = 128, 128, 8, 2, 0


def render():
    sc = oracle_lib.OracleScene(CORNELL)
    s, casts = sc.render_samples(W, H, SPP, MB, SEED)
    hdr, ldr = oracle_lib.pixel_mean(s, W * H, SPP)
    return hdr.reshape(H, W, 3), ldr.reshape(H, W, 3), casts


if __name__ == "__main__":
    hdr, ldr, casts = render()
    np.savez_compressed(os.path.join(HERE, "c1_cornell_128x128x8_b2_seed0.npz"), hdr=hdr, ldr=ldr,
                        casts=np.int64(casts))
    print("casts/sample", casts / (W * H * SPP), "mean", hdr.mean())
