"""Diagnostics: per-launch time of the v2 step kernel over workgroup geometries (envs per workgroup G,
block size), against the v1 team-per-env kernel, for the BASELINE configs."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
import torch  # noqa: E402
from cattleherd import _lib  # noqa: E402
from cattleherd.env import HerdBatch  # noqa: E402


def time_launches(b, k=200):
    for _ in range(20):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(k):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / k * 1000.0


def main():
    L = _lib.lib()
    configs = [("ctde", 4096, 4, 16), ("ctde", 4096, 2, 8), ("ctde", 1024, 2, 8), ("marl", 4096, 4, 32),
               ("ctde", 4096, 12, 16)]
    precs = sys.argv[1:] or ["f64"]
    if len(sys.argv) >= 5:   # one config: mode E n m [prec]
        configs = [(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]))]
        precs = sys.argv[5:] or ["f64"]
    for prec in precs:
        for mode, E, n, m in configs:
            b = HerdBatch(E, n, m, mode=mode, precision=prec)
            g, blk, lds, kv = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int32()
            L.ch__geometry(b.handle, ctypes.byref(g), ctypes.byref(blk), ctypes.byref(lds), ctypes.byref(kv))
            b.reset()
            row = [f"default(G={g.value},B={blk.value},v{kv.value})={time_launches(b):.1f}"]
            L.ch__set_kernel(b.handle, ctypes.c_int32(1))
            row.append(f"v1={time_launches(b):.1f}")
            L.ch__set_kernel(b.handle, ctypes.c_int32(2))
            for G in ([int(x) for x in os.environ["CH_SWEEP_G"].split(",")] if os.environ.get("CH_SWEEP_G") else (1, 2, 3, 4, 8, 16, 32)):
                for B in (128, 192, 256, 320, 384, 512, 576, 640, 704, 768):
                    if L.ch__set_geometry(b.handle, ctypes.c_int32(G), ctypes.c_int32(B)) != 0:
                        continue
                    row.append(f"G{G}/B{B}={time_launches(b):.1f}")
            print(prec, mode, E, n, m, "us:", " ".join(row), flush=True)
            b.close()


if __name__ == "__main__":
    main()
