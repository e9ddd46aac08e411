"""Diagnostics: fp64 VALU instructions per evaluated alpha pair, from the gfx950 ISA.

Compiles probe kernels that run exactly one piece of the flock's alpha pair evaluation (ch_step.hip alpha_full_pw ->
ch_device.h pair_terms_n; flockUtils.py:237-258, 327-337) on one value per lane, with the library's flags, and counts
the instructions of each kernel body minus a load/store skeleton.  The pieces: the pair norm's sqrt, IEEE divisions
(zx / den, zy / den, sigma_1's z / sqrt), divc (correctly rounded division by a constant), the bump's cos on [0, pi],
and the whole pair as alpha_full_pw evaluates it.  Static counts: every branch of the bump is counted (its b = 0 / 1
arms are a few instructions; a queued pair inside the lattice range takes the cos arm).

  python tools/alpha_pair_isa.py [--json out.json]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rl-cattle-herding_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

PROBE = r'''
#include "ch_device.h"
using namespace ch;
#define K(name, expr) extern "C" __global__ void name(const double* __restrict__ a, const double* __restrict__ b, \
                                                       double* __restrict__ o) { \
    const int i = threadIdx.x; const double x = a[i], y = b[i]; o[i] = (expr); }
K(k_skeleton, x + y)
K(k_sqrt, sqrt(x * x + y * y))
K(k_div, x / y)
K(k_divc, divc(x, 0.1))
K(k_sigma1, sigma_1(x))
K(k_cos, cos_0pi(x))
K(k_bump, bump(x))
extern "C" __global__ void k_pair(const double* __restrict__ a, const double* __restrict__ b, double* __restrict__ o) {
    // alpha_full_pw's evaluation of one queued pair: offset in, (gx, gy, b) out
    const int i = threadIdx.x;
    const double zx = a[i], zy = b[i];
    const double ra = sigma_norm_n(1.2), da = ra;
    const double nrm = sqrt(zx * zx + zy * zy);
    double gx = 0, gy = 0, cx = 0, cy = 0;
    const double bb = pair_terms_n(nrm, zx, zy, 0.0, 0.0, 0.0, 0.0, ra, da, gx, gy, cx, cy);
    o[i] = gx; o[64 + i] = gy; o[128 + i] = bb;
}
extern "C" __global__ void k_pair_skeleton(const double* __restrict__ a, const double* __restrict__ b,
                                           double* __restrict__ o) {
    const int i = threadIdx.x;
    o[i] = a[i]; o[64 + i] = b[i]; o[128 + i] = a[i] + b[i];
}
'''

FLOP_MODEL = 34   # SURVEY 8(d)'s full alpha pair (DESIGN.md Roofline), sqrt and cos counted as one FLOP each


def classify(m):
    if m.startswith("v_"):
        return "valu_f64" if ("f64" in m or m in ("v_div_fmas_f64", "v_div_fixup_f64")) else "valu_other"
    if m.startswith("s_"):
        return "salu"
    if m.startswith(("global_", "buffer_", "flat_", "ds_")):
        return "mem"
    return "other"


def count(asm):
    out = {}
    cur = None
    for line in asm.splitlines():
        mt = re.match(r"^(k_\w+):", line)
        if mt:
            cur = mt.group(1)
            out[cur] = collections.Counter()
            continue
        if cur and line.startswith(".Lfunc_end"):
            cur = None
            continue
        if cur:
            s = line.strip()
            if not s or s.startswith((".", ";", "//")) or s.endswith(":"):
                continue
            m = s.split()[0]
            out[cur][classify(m)] += 1
            out[cur]["all"] += 1
            out[cur]["op:" + m] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "probe.hip")
        with open(src, "w") as f:
            f.write(PROBE)
        asm = os.path.join(td, "probe.s")
        subprocess.run([HIPCC, "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", "-I" + CSRC, "-I" + os.path.join(ROOT, "include"), src, "-o", asm], check=True)
        c = count(open(asm).read())
    rows = {}
    for k, skel in (("k_sqrt", "k_skeleton"), ("k_div", "k_skeleton"), ("k_divc", "k_skeleton"),
                    ("k_sigma1", "k_skeleton"), ("k_cos", "k_skeleton"), ("k_bump", "k_skeleton"),
                    ("k_pair", "k_pair_skeleton")):
        rows[k[2:]] = {key: c[k][key] - c[skel][key] for key in ("all", "valu_f64", "valu_other", "salu")}
    pair_ops = {key[3:]: v for key, v in sorted(c["k_pair"].items()) if key.startswith("op:v_")}
    for name, r in rows.items():
        print(f"{name:8s} all {r['all']:4d}  fp64 VALU {r['valu_f64']:4d}  other VALU {r['valu_other']:4d}  "
              f"SALU {r['salu']:3d}")
    p = rows["pair"]
    print(f"pair: {p['valu_f64']} fp64 VALU for the {FLOP_MODEL}-FLOP model = {p['valu_f64'] / FLOP_MODEL:.2f} per FLOP; "
          f"{p['valu_f64'] + p['valu_other']} VALU in all")
    print("pair VALU mix:", ", ".join(f"{k} {v}" for k, v in sorted(pair_ops.items(), key=lambda t: -t[1])))
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"pieces": rows, "pair_valu_ops": pair_ops, "flop_model": FLOP_MODEL}, f, indent=1)


if __name__ == "__main__":
    main()
