import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from inverse_path_tracer_amd import torch_ops
from inverse_path_tracer_amd.optimize import build_tasks, optimize
torch.cuda.set_device(0)
A = os.path.join(ROOT, "assets", "scenes")
for (W, spp, steps, lr) in [(64, 16, 60, 2e-2), (64, 16, 150, 2e-2), (128, 32, 100, 3e-2)]:
    tasks = build_tasks([os.path.join(A, "0.txt")], W, W, 256, 4, 0.5, torch.device("cuda"))
    t = tasks[0]
    img = torch_ops.render(t.scene, t.kd, W, W, 64, 4, seed=5)
    ((img - t.target) ** 2).mean().backward()
    g = t.kd.grad.abs().sum(1)
    t.kd.grad = None
    optimize(tasks, W, W, spp, 4, steps=steps, lr=lr)
    print("cfg", W, spp, steps, lr, "loss", t.history[0], t.history[-1])
    for i in range(t.kd.shape[0]):
        print(i, ["%.3f" % x for x in t.truth[i].tolist()], ["%.3f" % x for x in t.kd[i].tolist()], "%.3g" % float(g[i]))
