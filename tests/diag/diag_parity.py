"""GPU diagnostic: per-region errors of the HIP step vs golden rollout fixtures and the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rl-cattle-herding_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import torch  # noqa: E402
from helpers import load, stack, state_at  # noqa: E402
from cattleherd.env import HerdBatch  # noqa: E402


def main(fname="ctde_roll_n4_m16_l7.npz"):
    d = load(fname)
    mode = 0 if fname.startswith("ctde") else 1
    T = len(d["action"])
    states = [state_at(d, "state_", t) for t in range(T)]
    n, m, lvl = int(states[0]["n"]), int(states[0]["m"]), int(states[0]["ctor_level"])
    b = HerdBatch(T, n, m, mode="ctde" if mode == 0 else "marl", curriculum_level=lvl)
    b.reset()
    s = stack(states)
    s = {k: v for k, v in s.items() if k not in ("m", "ctor_level", "episode_len")}
    b.set_state(s)
    g0 = b.get_state()
    for k in ("drone_pos", "drone_quat", "drone_vel", "drone_angv", "pid_int_rpy"):
        print("injected", k, np.max(np.abs(g0[k][:, :n] - s[k][:, :n])))
    print("injected cow", np.max(np.abs(g0["cow_pos"] - s["cow_pos"][:, :m])), np.max(np.abs(g0["cow_vel"] - s["cow_vel"][:, :m])))
    for k in ("n", "step_counter", "step_counter_A", "level", "tally", "has_prev", "spawn_index"):
        print("injected", k, np.array_equal(g0[k], s[k]))
    obs, rew, te, tr = b.step(torch.tensor(d["action"], device=b.device), autoreset=False)
    torch.cuda.synchronize()
    obs = obs.cpu().numpy()
    err = np.abs(obs.astype(np.float64) - d["obs"])
    print("obs max err per column (first 20):", np.round(err.max(axis=(0, 1))[:20], 9))
    print("obs max err cols 20-66:", err.max(axis=(0, 1))[20:66].max(), "rows>=n:", err[:, n:].max())
    bad = np.argwhere(err > 1e-6 + 1e-6 * np.abs(d["obs"]))
    print("n bad elems", len(bad), "first", bad[:10].tolist())
    for t, r, c in bad[:5]:
        print(t, r, c, obs[t, r, c], d["obs"][t, r, c])
    print("reward err", np.nanmax(np.abs(rew.cpu().numpy()[:, 0] - d["reward"])) if mode == 0 else "")
    g = b.get_state()
    idx = [t for t in range(T - 1) if t not in set(d["reset_at"].tolist())]
    nxt = stack([states[t + 1] for t in idx])
    for k in ("drone_pos", "drone_quat", "drone_vel", "drone_angv", "pid_int_rpy", "pid_int_pos", "pid_last_rpy"):
        e = np.abs(g[k][idx, :n] - nxt[k][:, :n])
        print("next", k, e.max(), "argmax", np.unravel_index(e.argmax(), e.shape))
    print("next cow_pos", np.abs(g["cow_pos"][idx] - nxt["cow_pos"][:, :m]).max(),
          "cow_vel", np.abs(g["cow_vel"][idx] - nxt["cow_vel"][:, :m]).max())




def pid_debug(fname="ctde_roll_n4_m16_l7.npz"):
    """Compare per-drone PID intermediates (device debug buffer) with the oracle's PID on the same inputs."""
    import ctypes
    import oracle as O
    from cattleherd import _lib
    d = load(fname)
    T = len(d["action"])
    states = [state_at(d, "state_", t) for t in range(T)]
    n, m, lvl = int(states[0]["n"]), int(states[0]["m"]), int(states[0]["ctor_level"])
    b = HerdBatch(T, n, m, mode="ctde", curriculum_level=lvl)
    b.reset()
    s = stack(states)
    b.set_state({k: v for k, v in s.items() if k not in ("m", "ctor_level", "episode_len")})
    dbg = torch.zeros((T, n, 16), dtype=torch.float64, device=b.device)
    _lib.lib().ch__set_debug(b.handle, ctypes.c_void_p(dbg.data_ptr()))
    b.step(torch.tensor(d["action"], device=b.device), autoreset=False)
    torch.cuda.synchronize()
    g = dbg.cpu().numpy()
    worst = {}
    for t in range(T):
        st = states[t]
        for k in range(n):
            a = d["action"][t][k].astype(np.float32)
            hn = np.sqrt(np.float32(a[0] * a[0] + a[1] * a[1]), dtype=np.float32)
            sc = np.float32(np.float32(2.5000000000000004) * np.abs(a[3]))
            ux = a[0] / hn if hn != 0 else np.float32(0)
            uy = a[1] / hn if hn != 0 else np.float32(0)
            tv = np.array([float(ux) * float(sc), float(uy) * float(sc), 0.0])
            rpy = O.euler_from_quat(st["drone_quat"][k])
            rpm, _, _, _ = O.pid_vel(st["drone_pos"][k], st["drone_quat"][k], st["drone_vel"][k],
                                     np.array([st["drone_pos"][k][0], st["drone_pos"][k][1], 0.45]),
                                     np.array([0, 0, rpy[2]]), tv, 1 / 60, st["pid_last_rpy"][k], st["pid_int_pos"][k],
                                     st["pid_int_rpy"][k])
            for name, gv, ov in (("tv", g[t, k, 0:3], tv), ("rpm", g[t, k, 10:14], rpm), ("hn", g[t, k, 14], hn),
                                 ("sc", g[t, k, 15], sc)):
                e = float(np.max(np.abs(np.asarray(gv, np.float64) - np.asarray(ov, np.float64))))
                if e > worst.get(name, (0,))[0]:
                    worst[name] = (e, t, k)
    print("PID intermediates, worst |gpu - oracle|:", worst)


if __name__ == "__main__":
    {"main": main, "pid": pid_debug}[sys.argv[1]](*sys.argv[2:])
