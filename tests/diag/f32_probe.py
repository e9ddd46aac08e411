"""Diagnostics: the CH_PREC_F32 step against the fp64 oracle -- error statistics per output."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import oracle as O  # noqa: E402
from cattleherd._lib import spawn_table  # noqa: E402
from cattleherd.env import HerdBatch  # noqa: E402
from helpers import stack  # noqa: E402


def main():
    n, m, E = 4, 16, 256
    table = spawn_table(m)
    rng = np.random.default_rng(3)
    envs, states = [], []
    for e in range(E):
        env = O.Env(0, n, m, table, start_level=7, env_id=e)
        env.reset()
        for _ in range(int(rng.integers(0, 120))):
            env.step(rng.uniform(-1, 1, (n, 4)).astype(np.float32), autoreset=True)
        envs.append(env)
        states.append(env.get_state())
    acts = np.random.default_rng(1).uniform(-1, 1, (E, n, 4)).astype(np.float32)
    ref = None
    for prec in ("f64", "f32"):
        b = HerdBatch(E, n, m, curriculum_level=7, precision=prec)
        b.reset()
        b.set_state(stack([{k: v for k, v in s.items() if k != "episode"} for s in states]))
        obs, rew, te, tr = b.step(torch.tensor(acts, device=b.device), autoreset=False)
        torch.cuda.synchronize()
        if ref is None:
            ref = [env.step(acts[e], autoreset=False) for e, env in enumerate(envs)]
        ro = np.stack([r[0] for r in ref]).astype(np.float64)
        go = obs.cpu().numpy().astype(np.float64)
        rr = np.array([r[1][0] for r in ref])
        gr = rew.cpu().numpy()[:, 0].astype(np.float64)
        b.close()
        rel = np.abs(gr - rr) / np.maximum(np.abs(rr), 1e-30)
        big = np.abs(ro) > 1e-3
        print(f"[{prec}] obs: max rel (|ref| > 1e-3) {np.max(np.abs(go - ro)[big] / np.abs(ro)[big]):.3e}, "
              f"max abs {np.max(np.abs(go - ro)):.3e}")
        groups = {"z": [0], "rpy": [1, 2, 3], "vel": [4, 5, 6], "angvel": [7, 8, 9], "nbr": [10, 11, 12, 13],
                  "cattle": list(range(86 - 2 * m, 86))}
        for name, cols in groups.items():
            d, r_ = np.abs(go - ro)[..., cols], np.abs(ro)[..., cols]
            bg = r_ > 1e-3
            mr = np.max(d[bg] / r_[bg]) if bg.any() else 0.0
            print(f"   {name:7s} max abs {d.max():.3e}  max rel (|ref| > 1e-3) {mr:.3e}  "
                  f"q99.9 rel {np.quantile(d[bg] / r_[bg], 0.999) if bg.any() else 0.0:.3e}")
        for rt, at in ((1e-4, 1e-6), (1e-4, 1e-7), (1e-4, 1e-8), (5e-5, 1e-8)):
            okc = np.isclose(go[..., 7:10], ro[..., 7:10], rtol=rt, atol=at)
            print(f"   angvel isclose(rtol {rt:g}, atol {at:g}) fails {int((~okc).sum())} of {okc.size}")
        relo = np.where(big, np.abs(go - ro) / np.maximum(np.abs(ro), 1e-30), 0)
        for idx in np.argsort(relo.ravel())[-5:][::-1]:
            e, r, c = np.unravel_index(idx, relo.shape)
            print(f"   worst env {e} row {r} col {c}: gpu {go[e, r, c]:.9g} ref {ro[e, r, c]:.9g}")
        print(f"[{prec}] reward: max rel {rel.max():.3e} (env {rel.argmax()}: gpu {gr[rel.argmax()]:.9g} "
              f"ref {rr[rel.argmax()]:.9g}), q99 {np.quantile(rel, 0.99):.3e}, median {np.median(rel):.3e}, "
              f"max abs {np.max(np.abs(gr - rr)):.3e}")
        trr = np.array([r[3][0] for r in ref])
        ter = np.array([r[2][0] for r in ref])
        print(f"[{prec}] truncated mismatches {int(np.sum(tr.cpu().numpy()[:, 0] != trr))}, terminated mismatches "
              f"{int(np.sum(te.cpu().numpy()[:, 0] != ter))} of {E}")

if __name__ == "__main__":
    main()
