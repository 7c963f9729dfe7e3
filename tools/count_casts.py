"""Counts C-bar = ray casts per sample (camera/continuation + shadow) with the
CPU oracle over the FULL benchmark configurations.  The
printed constants are committed in bench.py (CASTS_PER_SAMPLE)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402
from conftest import ASSETS, CORNELL, SCENE0  # noqa: E402

# scenes/0.txt with the Phong cube (assets/phong/scene0_phong.txt, bench.py c3_phong)
SCENE0_PHONG = CORNELL + [((0, -1.5, 4), (0, 0, 0), (1, 1, 1), os.path.join(ASSETS, "phong", "cube_phong.obj"),
                           os.path.join(ASSETS, "phong", "cube_phong.mtl"))]
CONFIGS = {
    "C2_cornell_512x512x64_b4": (CORNELL, 512, 512, 64, 4, 0),
    "C3_scene0_512x512x64_b4": (SCENE0, 512, 512, 64, 4, 0),
    "C3_phong_512x512x64_b4": (SCENE0_PHONG, 512, 512, 64, 4, 0),
}
# tools/count_casts.py NAME ...: only those configurations, merged into the committed file
only = sys.argv[1:]
path = os.path.join(ROOT, "profiles", "casts_per_sample.json")
out = json.load(open(path)) if only and os.path.exists(path) else {}
for name, (recs, W, H, spp, mb, seed) in CONFIGS.items():
    if only and name not in only:
        continue
    sc = O.OracleScene(recs)
    total, n, t0 = 0, 0, time.time()
    step = 32  # rows per chunk (bounded memory)
    for r in range(0, H, step):
        s, c = sc.render_samples(W, H, spp, mb, seed, r * W * spp, min(H, r + step) * W * spp)
        total += c
        n += len(s)
    out[name] = {"casts_per_sample": total / n, "samples": n, "nT": sc.nT, "seconds": round(time.time() - t0, 1)}
    print(name, out[name], flush=True)
# createGraph at the reference's own configuration (scene.h:8-11: 500x500,
# 100 spp, no bounce cap; scenes/0.txt): its integrator draws isSpecular at
# every vertex, so its paths differ from the forward's -- counted separately
if not only:
    sc = O.OracleScene(SCENE0)
    t0 = time.time()
    c = sc.graph_casts(500, 500, 100, None, 0)
    out["graph_scene0_500x500x100_unbounded"] = {"casts_per_sample": c / (500 * 500 * 100), "samples": 500 * 500 * 100,
                                                 "nT": sc.nT, "seconds": round(time.time() - t0, 1)}
    print("graph", out["graph_scene0_500x500x100_unbounded"], flush=True)
with open(path, "w") as f:
    json.dump(out, f, indent=1)
