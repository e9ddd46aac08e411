"""Diagnostics: ch_step_n (k_step2_multi) time per step over workgroup geometries (envs per workgroup, block size) --
e.g. two co-resident 8-env workgroups per CU against one 16-env workgroup.
  python tools/multi_geom.py ctde 4096 4 16 16x768 8x256 8x512"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
import torch  # noqa: E402
from cattleherd import _lib  # noqa: E402
from cattleherd.env import HerdBatch  # noqa: E402


def main():
    mode, E, n, m = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    L = _lib.lib()
    for geo in sys.argv[5:]:
        G, B = (int(x) for x in geo.split("x"))
        b = HerdBatch(E, n, m, mode=mode)
        rc = L.ch__set_geometry(b.handle, ctypes.c_int32(G), ctypes.c_int32(B))
        if rc != 0:
            print(geo, "unsupported", rc, flush=True)
            b.close()
            continue
        b.reset()
        for _ in range(300):
            b.step(random_actions=True, autoreset=True, terminal_obs=False)
        b.step_n(100, random_actions=True)
        torch.cuda.synchronize()
        m0 = L.ch__multi_steps(b.handle)
        t0 = time.perf_counter()
        b.step_n(2000, random_actions=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        t1 = time.perf_counter()
        for _ in range(500):
            b.step(random_actions=True, autoreset=True, terminal_obs=False)
        torch.cuda.synchronize()
        d1 = time.perf_counter() - t1
        print(f"{geo}: ch_step_n {E * 2000 / dt / 1e6:.1f} M env-steps/s ({dt / 2000 * 1e6:.2f} us/step, multi "
              f"{L.ch__multi_steps(b.handle) - m0}) | ch_step {E * 500 / d1 / 1e6:.1f} M ({d1 / 500 * 1e6:.2f} us)",
              flush=True)
        b.close()


if __name__ == "__main__":
    main()
