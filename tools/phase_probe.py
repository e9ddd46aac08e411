"""Diagnostics: per-launch time of the step kernel with phases skipped (ch__set_phase_mask: 1 drones,
2 flock, 4 task, 8 obs), per kernel version and geometry, for one config: mode E n m [prec]."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from geom_sweep import time_launches  # noqa: E402
from cattleherd import _lib  # noqa: E402
from cattleherd.env import HerdBatch  # noqa: E402


def main():
    mode, E, n, m = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    prec = sys.argv[5] if len(sys.argv) > 5 else "f64"
    geoms = [tuple(int(x) for x in g.split("/")) for g in sys.argv[6:]] or [None]
    L = _lib.lib()
    b = HerdBatch(E, n, m, mode=mode, precision=prec)
    b.reset()
    for kv in (1, 2):
        for geom in (geoms if kv == 2 else [None]):
            L.ch__set_kernel(b.handle, ctypes.c_int32(kv))
            if geom is not None:
                if L.ch__set_geometry(b.handle, ctypes.c_int32(geom[0]), ctypes.c_int32(geom[1])) != 0:
                    print("bad geometry", geom)
                    continue
            row = []
            for mask in (0, 2, 4, 8, 1, 6, 14, 15):
                L.ch__set_phase_mask(b.handle, ctypes.c_int32(mask))
                row.append(f"m{mask}={time_launches(b, 100):.1f}")
            L.ch__set_phase_mask(b.handle, ctypes.c_int32(0))
            print(f"{prec} {mode} E={E} N={n} M={m} v{kv} geom={geom}:", " ".join(row), flush=True)
    b.close()


if __name__ == "__main__":
    main()
