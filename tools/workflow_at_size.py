"""The reference's workflow at its own size, once, on one GPU, with stage
timings.

  1. pipeline (ipt.py:86-140 + ipt_cuda.py:115-165) at the legacy render
     configuration (500x500, 100 spp, unbounded): generate_files for 100
     scenes (scene text + createImage PNG), generate_data (createGraph against
     each image + getMaterials), the GCN (--epochs) and the 100 predicted
     renders;
  2. optimize (BASELINE configs[4] on one GPU): all 100 scenes/*.txt as ONE
     scene batch, 256x256, 32 spp, 4 bounces, Adam on the per-triangle Kd,
     targets rendered at 1024 spp.

Writes one JSON record (--out).  The dataset goes to a scratch directory
(--root, default /tmp/ipt_workflow), not into the repository."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def now_sync():
    import torch

    torch.cuda.synchronize()
    return time.time()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default="/tmp/ipt_workflow")
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--epochs", type=int, default=300)
    ap.add_argument("--opt-steps", type=int, default=200)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    import numpy as np
    import torch

    from inverse_path_tracer_amd import optimize as O
    from inverse_path_tracer_amd import pipeline as P

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    rec = {"gpu": torch.cuda.get_device_name(0), "n_scenes": a.n}
    idx = list(range(a.n))
    cfg = dict(width=500, height=500, spp=100, max_bounces=None, seed=0)
    os.makedirs(a.root, exist_ok=True)

    def save():
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)

    # ------------------------------------------------------------------ 1. pipeline
    t0 = now_sync()
    P.generate_files(a.root, idx, **cfg)
    t1 = now_sync()
    rec["generate_files"] = {"s": round(t1 - t0, 2), "per_scene_ms": round((t1 - t0) / a.n * 1e3, 2),
                             "what": "scenes/{i}.txt + createImage imgs/{i}.png (500x500x100, unbounded)"}
    print("files", rec["generate_files"], flush=True)
    save()
    P.generate_data(a.root, idx, **cfg)
    t2 = now_sync()
    rec["generate_data"] = {"s": round(t2 - t1, 2), "per_scene_ms": round((t2 - t1) / a.n * 1e3, 2),
                            "what": "createGraph vs imgs/{i}.png (500x500x100, unbounded) + compress + npz"}
    print("data", rec["generate_data"], flush=True)
    save()
    _, errs = P.train_and_predict(a.root, idx, a.epochs, lr=1e-4, device="cuda", split=int(0.8 * a.n),
                                  log_every=max(1, a.epochs // 5), **cfg)
    t3 = now_sync()
    rec["train_and_predict"] = {"s": round(t3 - t2, 2), "epochs": a.epochs, "train_scenes": int(0.8 * a.n),
                                "mean_l1_material_error": round(float(np.mean(errs)), 5),
                                "heldout_l1_material_error": round(float(np.mean(errs[int(0.8 * a.n):])), 5),
                                "what": "GCN (gcn.py, ipt.py:104-124) + preds/{i}_pred.png renders"}
    print("train", rec["train_and_predict"], flush=True)
    rec["pipeline_total_s"] = round(t3 - t0, 2)
    save()

    # ------------------------------------------------------------------ 2. optimize
    files = O._scene_files(os.path.join(ROOT, "assets", "scenes"), a.n)
    t4 = now_sync()
    tasks = O.build_tasks(files, 256, 256, 1024, 4, 0.5, dev)
    t5 = now_sync()
    m = O.MaterialOptimizer(tasks, 256, 256, 32, 4, 1e-2, None, 0, 16, True)
    m.step()  # warm-up (first-launch costs)
    t6 = now_sync()
    m.run(a.opt_steps - 1)
    t7 = now_sync()
    err0 = 0.5
    err = [float((t.kd.detach() - t.truth).abs()[18:].mean()) for t in tasks]
    rec["optimize"] = {"scenes": len(tasks), "targets_s": round(t5 - t4, 2), "steps": a.opt_steps,
                       "ms_per_step": round((t7 - t6) / max(1, a.opt_steps - 1) * 1e3, 3),
                       "scene_iterations_per_s": round(len(tasks) * (a.opt_steps - 1) / (t7 - t6), 1),
                       "fwd_plus_adj_Msamples_s": round(2 * len(tasks) * 256 * 256 * 32 * (a.opt_steps - 1) /
                                                        (t7 - t6) / 1e6, 1),
                       "mean_abs_cube_kd_err_after": round(float(np.mean(err)), 5),
                       "init": err0,
                       "what": "all scenes as one batch: batched forward + batched adjoint + L2 + Adam per step"}
    print("optimize", rec["optimize"], flush=True)
    save()


if __name__ == "__main__":
    main()
