"""f32 throughput at the saturated size for the shared-table geometries (16 envs per workgroup, 512 or 768
threads), one process, timed with HIP events around back-to-back steps."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
import torch  # noqa: E402
from cattleherd import _lib  # noqa: E402
from cattleherd.env import HerdBatch  # noqa: E402

L = _lib.lib()
for prec in ("f32", "f64"):
    for E in (4096, 262144):
        for blk in (None, 512, 768):
            b = HerdBatch(E, 4, 16, precision=prec)
            if blk is not None:
                assert L.ch__set_geometry(b.handle, ctypes.c_int32(16), ctypes.c_int32(blk)) == 0
            b.reset()
            k = 200 if E == 4096 else 40
            for _ in range(20):
                b.step(random_actions=True, autoreset=True, terminal_obs=False)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(k):
                b.step(random_actions=True, autoreset=True, terminal_obs=False)
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / k * 1000
            print(f"{prec} E={E} block={blk or 'default'}: {us:.2f} us/step, {E / us:.1f} M env-steps/s", flush=True)
            b.close()
