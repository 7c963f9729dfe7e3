"""First-contact GPU diagnostics: parity of every kernel against the CPU
oracle on small seeded cases + a first C2 timing.  Prints, never asserts."""
import os
import sys
import time

import numpy as np
import torch  # load torch's HIP runtime first (shared with libipt_amd.so)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402
from inverse_path_tracer_amd import Scene  # noqa: E402
from inverse_path_tracer_amd import _native as N  # noqa: E402
import ctypes as C  # noqa: E402

A = os.path.join(ROOT, "assets")
CORNELL = [((0, 0, 4), (0, 0, 0), (2, 2, 2), A + "/CornellBox/CornellBox-Empty-CO.obj", A + "/CornellBox/CornellBox-Empty-CO.mtl")]
SCENE0 = CORNELL + [((0, -1.5, 4), (0, 0, 0), (1, 1, 1), A + "/shapes/cube.obj",
                     "*Kd 0.9041462985304743 0.5854651848798454 0.007022117649276849*")]
from inverse_path_tracer_amd.scene import ObjectSpec  # noqa: E402


def prod(objs):
    return Scene([ObjectSpec(o[3], o[4], o[0], o[1], o[2]) for o in objs])


def cmp(name, a, b):
    a = np.asarray(a); b = np.asarray(b)
    eq = (a.view(np.uint32) == b.view(np.uint32)) if a.dtype == np.float32 else (a == b)
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    print(f"[{name}] bit-equal {eq.mean()*100:.4f}%  max|d| {d.max():.3e}  mean|a| {np.abs(a).mean():.4e}", flush=True)


print("devices", N.device_count(), torch.cuda.get_device_name(0), flush=True)
for nm, objs in [("cornell", CORNELL), ("scene0", SCENE0)]:
    P, Q = prod(objs), O.OracleScene(objs)
    cmp(nm + " triangles", P.triangles(), Q.triangles())
    cmp(nm + " camera", P.camera(), Q.camera())

P, Q = prod(CORNELL), O.OracleScene(CORNELL)
t0 = time.time(); s_p = P.render_samples(128, 128, 8, 2, 0); t1 = time.time()
s_q, casts = Q.render_samples(128, 128, 8, 2, 0)
print("C1 gpu host-call time", t1 - t0, "casts/sample", casts / (128 * 128 * 8))
cmp("C1 samples", s_p, s_q)
bad = np.where(np.any(s_p.view(np.uint32) != s_q.view(np.uint32), axis=1))[0]
print("C1 mismatching samples", len(bad), bad[:10])
if len(bad):
    for i in bad[:5]:
        print("  ", i, s_p[i], s_q[i])

P0, Q0 = prod(SCENE0), O.OracleScene(SCENE0)
s_p = P0.render_samples(64, 64, 16, None, 7)
s_q, _ = Q0.render_samples(64, 64, 16, None, 7)
cmp("scene0 unbounded samples", s_p, s_q)
hdr = P0.render(64, 64, 16, None, 7)
hq, _ = O.pixel_mean(s_q, 64 * 64, 16)
cmp("scene0 hdr", hdr.reshape(-1, 3), hq)

adj = np.random.RandomState(1).uniform(-1, 1, (64, 64, 3)).astype(np.float32)
gp = P0.adjoint(adj, 64, 64, 8, 4, 3)
gq = Q0.adjoint(64, 64, 8, 4, 3, adj)
print("adjoint rel err", np.abs(gp - gq).max() / np.abs(gq).max(), "float-equal", (gp.astype(np.float32) == gq.astype(np.float32)).mean())
tgt = np.random.RandomState(2).randint(0, 256, (64, 64, 3)).astype(np.uint8)
ap, dp_ = P0.graph(tgt, 64, 64, 8, None, 5)
aq, dq = Q0.graph(64, 64, 8, None, 5, tgt)
print("graph acc rel err", np.abs(ap - aq).max() / np.abs(aq).max(), "data max|d|", np.abs(dp_ - dq).max())

# ---- timing C2 through the device API on torch's stream
dev = torch.device("cuda:0")
for nm, objs, mb in [("C2 cornell 512x512x64 b4", CORNELL, 4), ("scene0 512x512x64 b4", SCENE0, 4)]:
    S = prod(objs)
    p = N.make_params(512, 512, 64, mb, 0)
    hdr_t = torch.empty((512, 512, 3), device=dev)
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        N.check(N.lib().ipt_render_dev(S.handle, C.byref(p), None, hdr_t.data_ptr(), None, st))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        N.check(N.lib().ipt_render_dev(S.handle, C.byref(p), None, hdr_t.data_ptr(), None, st))
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(f"{nm}: {ms:.3f} ms/frame  {512*512*64/ms/1e3:.1f} Msamples/s", flush=True)
    adjt = torch.ones((512, 512, 3), device=dev)
    g = torch.zeros((S.nT, 3), dtype=torch.float64, device=dev)
    N.check(N.lib().ipt_adjoint_dev(S.handle, C.byref(p), None, adjt.data_ptr(), g.data_ptr(), st))
    torch.cuda.synchronize()
    e0.record()
    for _ in range(3):
        N.check(N.lib().ipt_adjoint_dev(S.handle, C.byref(p), None, adjt.data_ptr(), g.data_ptr(), st))
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    print(f"{nm} adjoint: {ms:.3f} ms  {512*512*64/ms/1e3:.1f} grad-Msamples/s", flush=True)
