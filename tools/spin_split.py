"""Diagnostics: how much of k_step2's SQ_INSTS_SALU is hand-off spinning.

Two halves:
  * static (CPU): the instructions of one sleep iteration of the hand-off waits (ch_step.hip lds_wait: s_sleep 1, an
    LDS load of the flag, the compare, the loop control), read from configs[3]'s k_step2 in ch_step.hip's gfx950
    device assembly compiled with the library's flags (`--asm`, made once and cached);
  * dynamic (GPU): a diagnostic build (-DCH_COUNT_SPINS, `--build` writes cattleherd/libcattleherd_spins.so) sums the
    sleep iterations of every hand-off wait per wave kind (drone wave, cow waves) over plain ch_step launches of
    configs[3] after the bench's burn-in; iterations x SALU per iteration is the spin share of the SALU count.

  python tools/spin_split.py --build                       # CPU: the counting library
  python tools/spin_split.py --static-only --asm X.s        # CPU: the loop cost (writes X.s when absent)
  python tools/spin_split.py --asm X.s|X.json [--json out]  # GPU: counts per launch + the loop cost
"""
import argparse
import collections
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "rl-cattle-herding_amd")
SPIN_LIB = os.path.join(PKG, "cattleherd", "libcattleherd_spins.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

KERNEL = "_ZN2ch7k_step2IdLi0ELi16ELi4ELi16ELb0ELb0ELb0EEEvNS_10StepParamsIT_EE"   # configs[3]'s k_step2
NON_ALU = ("s_sleep", "s_waitcnt", "s_cbranch", "s_branch", "s_barrier", "s_nop", "s_setprio")


def device_asm(path):
    """ch_step.hip's device assembly with the library's flags (about 3 minutes; cached at `path`)."""
    if not os.path.exists(path):
        subprocess.run([HIPCC, "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", "-I" + os.path.join(ROOT, "include"), os.path.join(PKG, "csrc", "ch_step.hip"), "-o",
                        path], check=True, stderr=subprocess.DEVNULL)
    return open(path).read()


def loop_cost(asm):
    """One sleep iteration of the hand-off waits in configs[3]'s kernel: the instructions after each `s_sleep` up to
    the loop's branch, at every sleep site (the waits are unrolled, so one iteration sits between two sleeps); the
    most common window is the iteration of an inlined lds_wait."""
    body = asm.split(KERNEL + ":", 1)[1].split(".Lfunc_end", 1)[0]
    ins = [ln.strip().split()[0] for ln in body.splitlines()
           if ln.strip() and not ln.strip().startswith((".", ";")) and not ln.strip().endswith(":")]
    wins = collections.Counter()
    for i, m in enumerate(ins):
        if m == "s_sleep":
            w = ["s_sleep"]
            for x in ins[i + 1:i + 12]:
                w.append(x)
                if x.startswith(("s_cbranch", "s_branch")) or x == "s_sleep":
                    break
            wins[tuple(w)] += 1
    win, n = wins.most_common(1)[0]
    salu = [x for x in win if x.startswith("s_") and not x.startswith(NON_ALU)]
    return {"body": list(win), "sites": n, "sleep_sites": ins.count("s_sleep"), "kernel_static_instructions": len(ins),
            "salu": len(salu), "scalar_all": sum(x.startswith("s_") for x in win),
            "valu": sum(x.startswith("v_") for x in win), "lds": sum(x.startswith("ds_") for x in win)}


def build():
    sys.path.insert(0, PKG)
    from cattleherd import _build
    print(_build.build(extra_flags=("-DCH_COUNT_SPINS",), out=SPIN_LIB))


def measure(steps):
    os.environ["CH_LIB_PATH"] = SPIN_LIB   # (read at import by cattleherd._lib)
    sys.path.insert(0, PKG)
    import torch
    from cattleherd import _lib
    from cattleherd.env import HerdBatch
    L = _lib.lib()
    fn = L.ch__spin_counts
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    fn.restype = ctypes.c_int
    b = HerdBatch(4096, 4, 16, mode="ctde")
    b.reset()
    for _ in range(1200):   # bench.py's burn-in: envs spread over their episodes
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    out = (ctypes.c_ulonglong * 4)()
    assert fn(out) == 0
    for _ in range(steps):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    assert fn(out) == 0
    b.close()
    grid = 4096 // 16
    return {"launches": steps, "grid": grid,
            "drone_sleeps_per_launch": out[0] / steps, "cow_sleeps_per_launch": out[1] / steps,
            "drone_waits_per_launch": out[2] / steps, "cow_waits_per_launch": out[3] / steps,
            "drone_sleeps_per_wave": out[0] / steps / grid, "cow_sleeps_per_wave": out[1] / steps / grid / 11}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--salu-per-launch", type=float, default=None,
                    help="SQ_INSTS_SALU per launch of the shipped library (profiles/counters/c4_f64.json)")
    ap.add_argument("--json", default=None)
    ap.add_argument("--asm", default="/tmp/ch_step_dev.s", help="ch_step.hip device assembly (made when absent)")
    ap.add_argument("--static-only", action="store_true")
    args = ap.parse_args()
    if args.build:
        build()
        return
    if args.asm.endswith(".json"):   # the static half, computed beforehand (--static-only > X.json)
        lc = json.load(open(args.asm))
    else:
        lc = loop_cost(device_asm(args.asm))
    if args.static_only:
        print(json.dumps(lc))
        return
    print("wait loop, one iteration:", " ".join(lc["body"]), flush=True)
    r = measure(args.steps)
    salu = args.salu_per_launch
    if salu is None:
        rec = os.path.join(ROOT, "profiles", "counters", "c4_f64.json")
        salu = json.load(open(rec))["sq_insts_salu"] if os.path.exists(rec) else None
    iters = r["drone_sleeps_per_launch"] + r["cow_sleeps_per_launch"]
    spin_salu = iters * lc["salu"]
    r.update({"loop_salu_per_iteration": lc["salu"], "loop_scalar_all_per_iteration": lc["scalar_all"],
              "loop_valu_per_iteration": lc["valu"], "loop_lds_per_iteration": lc["lds"], "loop_body": lc["body"],
              "spin_scalar_all_per_launch": iters * lc["scalar_all"], "spin_valu_per_launch": iters * lc["valu"],
              "spin_salu_per_launch": spin_salu, "salu_per_launch": salu,
              "spin_share_of_salu": spin_salu / salu if salu else None})
    for k, v in r.items():
        if k != "loop_body":
            print(f"{k}: {v}")
    if args.json:
        with open(args.json, "w") as f:
            json.dump(r, f, indent=1)


if __name__ == "__main__":
    main()
