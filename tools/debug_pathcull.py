"""Debug: rays where the culled path cast differs from the full pair loop
(saved to gpurun_out/pathcull_mismatch.npz)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import CORNELL, SCENE0, product_scene  # noqa: E402
import test_gpu as TG  # noqa: E402

for which, recs in (("cornell", CORNELL), ("scene0", SCENE0)):
    P = product_scene(recs)
    tris = P.triangles()
    rng = np.random.RandomState(31)
    n = 300000
    v = tris[:, 0:9].reshape(-1, 3, 3)
    src = rng.randint(0, P.nT, n)
    a, b = rng.uniform(0, 1, (2, n))
    flip = a + b > 1
    a[flip], b[flip] = 1 - a[flip], 1 - b[flip]
    O = v[src, 0] + a[:, None] * (v[src, 1] - v[src, 0]) + b[:, None] * (v[src, 2] - v[src, 0])
    D = rng.normal(size=(n, 3))
    nrm = np.cross(v[src, 1] - v[src, 0], v[src, 2] - v[src, 0])
    graze = rng.uniform(0, 1, n) < 0.2
    Dg = D - (np.sum(D * nrm, 1) / np.sum(nrm * nrm, 1))[:, None] * nrm
    D[graze] = Dg[graze] + rng.normal(0, 1e-3, (int(graze.sum()), 3))
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    Oa, Da = TG._rays(P, 20000, 60000, 5)
    O = np.concatenate([O.astype(np.float32), Oa])
    D = np.concatenate([D.astype(np.float32), Da])
    kind = np.concatenate([np.where(graze, 1, 0), np.full(20000, 2), np.full(60000, 3)])
    tg = np.full(len(O), -1, np.int32)
    tc, ic = P.closest_hit(O, D, targets=tg)
    tf, i_f = P.closest_hit(O, D)
    bad = (ic != i_f) | (tc.view(np.uint32) != tf.view(np.uint32))
    print(which, "mismatches", int(bad.sum()), "of", len(O), "by kind", np.bincount(kind[bad], minlength=4))
    np.savez(os.path.join(ROOT, "gpurun_out", "pathcull_mismatch_%s.npz" % which), O=O[bad], D=D[bad], ic=ic[bad],
             i_f=i_f[bad], tc=tc[bad], tf=tf[bad], kind=kind[bad])
    # index order sanity: same rays through the probe in reverse order
    print(which, "first mismatches", list(zip(ic[bad][:10], i_f[bad][:10], tc[bad][:10], tf[bad][:10])))
