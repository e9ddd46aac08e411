"""Diagnostics: per-workgroup phase timestamps of the v2 step kernel (ch__set_tstamp).

For a few consecutive steps: kernel span on the 100 MHz wall clock, spread of workgroup start times
(dispatch), per-workgroup duration, and mean shader cycles per phase."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rl-cattle-herding_amd"))
import torch  # noqa: E402
from cattleherd import _lib  # noqa: E402
from cattleherd.env import HerdBatch  # noqa: E402


def trace(mode, E, n, m, prec, G=None, B=None, steps=4, summary=None):
    """Print the phase table of `steps` launches; `summary` (a list) receives one dict per launch with the numbers
    bench.py's latency roofline quotes (drone chain and workgroup cycles)."""
    L = _lib.lib()
    b = HerdBatch(E, n, m, mode=mode, precision=prec)
    if G is not None:
        assert L.ch__set_geometry(b.handle, ctypes.c_int32(G), ctypes.c_int32(B)) == 0
    g, blk, lds, kv = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int32()
    L.ch__geometry(b.handle, ctypes.byref(g), ctypes.byref(blk), ctypes.byref(lds), ctypes.byref(kv))
    grid = (E + g.value - 1) // g.value
    ts = torch.zeros((grid, 128), dtype=torch.int64, device=b.device)
    b.reset()
    for _ in range(0 if os.environ.get("CH_TRACE_NOBURN") else 250):   # steady state: resets have desynchronised the flocking parity
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    L.ch__set_tstamp(b.handle, ctypes.c_void_p(ts.data_ptr()))
    if os.environ.get("CH_PHASE_MASK"):
        L.ch__set_phase_mask(b.handle, ctypes.c_int32(int(os.environ["CH_PHASE_MASK"])))
    print(f"== {prec} {mode} E={E} N={n} M={m} G={g.value} block={blk.value} lds={lds.value} grid={grid}")
    multi = bool(os.environ.get("CH_TRACE_MULTI"))   # ch_step_n's k_step2_multi: the stamps of a launch's third step
    for s in range(steps):
        ts.zero_()
        torch.cuda.synchronize()
        if multi:
            b.step_n(3, random_actions=True)
        else:
            b.step(random_actions=True, autoreset=True, terminal_obs=False)
        torch.cuda.synchronize()
        t = ts.cpu().numpy()
        w0, w1 = t[:, 0], t[:, 1]
        span_us = (w1.max() - w0.min()) / 100.0
        start = (w0 - w0.min()) / 100.0
        dur = (w1 - w0) / 100.0
        cyc = t[:, 14] - t[:, 2]
        clk = (cyc / np.maximum(dur, 1e-3)).mean() / 1e3
        cus = len(np.unique(t[:, 12]))
        rel = lambda k: (t[:, k] - t[:, 2]).mean()  # noqa: E731
        print(f" step {s}: span {span_us:.1f}us | WG start q50/q90/max {np.percentile(start, 50):.1f}/"
              f"{np.percentile(start, 90):.1f}/{start.max():.1f}us | WG dur mean/max {dur.mean():.1f}/{dur.max():.1f}us"
              f" | ~{clk:.2f} GHz | CUs {cus}")
        print(f"   drone wave (cycles from start): B0 {rel(3):.0f} chain {rel(4):.0f} terms {rel(5):.0f} "
              f"H {rel(6):.0f} resets-published {rel(15):.0f} book {rel(7):.0f} | cow waves: alpha {rel(8):.0f} D {rel(9):.0f} flock {rel(10):.0f} "
              f"copy {rel(11):.0f} | B1 {rel(13):.0f} end {rel(14):.0f}")
        print(f"   drone wave end {rel(35):.0f} | cow waves: final pass start (wave 1) {rel(37):.0f}, Euler math done "
              f"{(t[t[:, 62] > 0, 62] - t[t[:, 62] > 0, 2]).mean() if (t[:, 62] > 0).any() else float('nan'):.0f}, "
              f"last cow wave end {rel(63):.0f}")
        if os.environ.get("CH_TRACE_SLOTS"):   # every phase slot the launch wrote: mean cycles from workgroup start
            sl = {k: round(float((t[t[:, k] > 0, k] - t[t[:, k] > 0, 2]).mean())) for k in range(3, 64)
                  if k != 12 and (t[:, k] > 0).any() and k not in range(22, 26)}
            print("   slots " + " ".join(f"{k}:{v}" for k, v in sorted(sl.items(), key=lambda kv: kv[1])))
        print(f"   cow waves (latest of the workgroup's waves): flock done {rel(57):.0f}, reset list seen {rel(56):.0f}, "
              f"Euler stores done {rel(58):.0f}, final pass done {rel(60):.0f}, end {rel(63):.0f}")
        nfv = t[:, 31]
        for sel, name in ((nfv >= 0, "all"), (nfv <= 2, "nf<=2"), (nfv >= 7, "nf>=7")):
            if not sel.any():
                continue
            r2 = lambda k: (t[sel, k] - t[sel, 2]).mean()  # noqa: E731
            print(f"   cow waves [{name}, {int(sel.sum())} WGs]: E {r2(11):.0f} pairs {r2(18):.0f} A {r2(20):.0f} rows+sync {r2(21):.0f} "
                  f"D {r2(9):.0f} H(drone) {r2(6):.0f} delta {r2(16):.0f} Q {r2(17):.0f} flock {r2(10):.0f} "
                  f"| cow waves done (mean per wave) {' '.join(f'{(t[sel, 40 + w] - t[sel, 2]).mean():.0f}' for w in range(1, blk.value // 64))} "
                  f"| drone book {r2(7):.0f} B1 {r2(13):.0f} end {r2(14):.0f}")
        print(f"   at the last barrier: drone wave {rel(35):.0f} cow wave 1 {rel(36):.0f} (F_R seen {rel(37):.0f})")
        nw = blk.value // 64
        ws = np.where(t[:, 52:52 + nw] > 0, t[:, 52:52 + nw] - t[:, 2:3], 0)
        rs = t[:, 30] > 0
        if rs.any():
            r3 = lambda k: (t[rs, k] - t[rs, 2]).mean()  # noqa: E731
            print(f"   resetting WGs ({int(rs.sum())}), cow wave 1: reset list seen {r3(52):.0f} bodies computed {r3(55):.0f} "
                  f"sync passed {r3(53):.0f} stores issued {r3(54):.0f} | drone book {r3(7):.0f} | cow waves done (max per WG) "
                  f"{(t[rs, 41:41 + blk.value // 64 - 1].max(axis=1) - t[rs, 2]).mean():.0f} vs non-resetting "
                  f"{(t[~rs, 41:41 + blk.value // 64 - 1].max(axis=1) - t[~rs, 2]).mean():.0f}")
        print(f"   wave start (cycles after wave 0's): mean {' '.join(f'{ws[:, w].mean():.0f}' for w in range(nw))} | "
              f"last wave q50/max {np.percentile(ws.max(axis=1), 50):.0f}/{ws.max():.0f} | first barrier passed {rel(3):.0f}")
        print(f"   alpha passes (cow wave 1): cheap done {rel(38):.0f} all cheap (F_C) {rel(39):.0f} full done {rel(18):.0f}"
              f" | queued pairs per WG {t[:, 29].mean():.1f} (per flocking env {(t[:, 29] / np.maximum(t[:, 31], 1)).mean():.1f})")
        print(f"   bookkeeping: scalars+centroid {rel(32):.0f} marl-prep {rel(33):.0f} env.step dicts {rel(34):.0f}")
        print(f"   drone wave after H: dtaskB {rel(26):.0f} pre-fence {rel(27):.0f} published {rel(15):.0f} "
              f"reward {rel(19):.0f} metrics stored {rel(28):.0f} book {rel(7):.0f}")
        simd = (t[:, 22:26] >> 4) & 3
        same = 0
        pairs = 0
        for cu in np.unique(t[:, 12]):
            ks = np.nonzero(t[:, 12] == cu)[0]
            for a in range(len(ks)):
                for c in range(a + 1, len(ks)):
                    pairs += 1
                    same += int(simd[ks[a], 0] == simd[ks[c], 0])
        from collections import Counter
        pat = Counter()
        for cu in np.unique(t[:, 12]):
            ks = np.nonzero(t[:, 12] == cu)[0]
            if len(ks) == 2:
                a, b2 = ks
                pat[(tuple(simd[a].tolist()), tuple(simd[b2].tolist()))] += 1
        # per cow wave: chunks and cycles per loop; the wave that shares its SIMD with the co-resident
        # workgroup's drone wave: wave 1 in the grid's first half, wave 3 in the second
        names = ("pairs", "cows", "rows", "delta", "flock")
        half = len(t) // 2
        for w in range(1, min(7, blk.value // 64)):
            sh = np.array([(w == 1) if k < half else (w == 3) for k in range(len(t))])
            for lab, sel in (("shared", sh), ("free", ~sh)):
                if not sel.any():
                    continue
                base = 64 + 10 * (w - 1)
                parts = []
                for li, nm in enumerate(names):
                    c = t[sel, base + 2 * li].astype(np.float64)
                    cy = t[sel, base + 2 * li + 1].astype(np.float64)
                    parts.append(f"{nm} {c.mean():.2f}x{(cy.sum() / max(c.sum(), 1)):.0f}")
                print(f"   cow wave {w} [{lab}, {int(sel.sum())}]: " + " | ".join(parts))
        print("   co-resident wave->SIMD patterns (first WG, second WG):", pat.most_common(6))
        split = sum(1 for cu in np.unique(t[:, 12]) for ks in [np.nonzero(t[:, 12] == cu)[0]]
                    if len(ks) == 2 and ks[0] < len(t) // 2 <= ks[1])
        print(f"   CUs whose first WG is in the lower half of the grid and second in the upper: {split}")
        print(f"   SIMD of wave 0: counts {np.bincount(simd[:, 0], minlength=4).tolist()} | wave order sample "
              f"{simd[:3].tolist()} | co-resident WG pairs {pairs}, drone waves on the same SIMD {same}")
        tail = (t[:, 14] - t[:, 13]).astype(np.float64)
        chain = (t[:, 4] - t[:, 3]).astype(np.float64)
        res = t[:, 30] > 0   # workgroups that rebuilt auto-reset envs this step
        print(f"   spread: WG cycles q50/q90/max {np.percentile(cyc, 50):.0f}/{np.percentile(cyc, 90):.0f}/{cyc.max():.0f}"
              f" | resetting WGs {int(res.sum())}: cycles mean {cyc[res].mean() if res.any() else 0:.0f} vs "
              f"{cyc[~res].mean():.0f} | chain q50/q90/max {np.percentile(chain, 50):.0f}/{np.percentile(chain, 90):.0f}/"
              f"{chain.max():.0f}")
        if summary is not None:
            summary.append({"wg_cycles_q50": float(np.percentile(cyc, 50)), "wg_cycles_q90": float(np.percentile(cyc, 90)),
                            "wg_cycles_max": float(cyc.max()), "chain_cycles_q50": float(np.percentile(chain, 50)),
                            "chain_start": float(rel(3)), "chain_done": float(rel(4)), "drone_terms_done": float(rel(5)),
                            "h_received": float(rel(6)), "reset_list": float(rel(15)), "reward_done": float(rel(19)),
                            "drone_wave_end": float(rel(35)), "span_us": float(span_us), "clock_ghz": float(clk),
                            "flocking_envs_per_wg": float(nfv.mean()), "resetting_wgs": int(res.sum())})
        slow = np.argsort(cyc)[-5:]
        nfv = t[:, 31]
        print(f"   flocking envs per WG: mean {nfv.mean():.2f} | slow WGs' nf {nfv[slow].tolist()} | cycles by nf: " +
              " ".join(f"{v}:{cyc[nfv == v].mean():.0f}" for v in np.unique(nfv)))
        for k in slow:
            print(f"     slow WG {k}: flock end per cow wave {[int(t[k, 40 + w] - t[k, 2]) for w in range(1, blk.value // 64)]}")
        for k in slow:
            print(f"     slow WG {k}: cyc {cyc[k]:.0f} chain {chain[k]:.0f} tail {tail[k]:.0f} B0 {t[k, 3] - t[k, 2]} "
                  f"terms {t[k, 5] - t[k, 4]} H {t[k, 6] - t[k, 5]} book {t[k, 7] - t[k, 6]} B1 {t[k, 13] - t[k, 7]} "
                  f"cu {t[k, 12]}")
    b.close()


def main():
    if len(sys.argv) >= 2 and sys.argv[1] == "--json":   # --json mode E n m: 8 launches, then one JSON summary line
        a = sys.argv[2:]
        rows = []
        trace(a[0], int(a[1]), int(a[2]), int(a[3]), "f64", steps=8, summary=rows)
        out = {k: float(np.mean([r[k] for r in rows])) for k in rows[0]}
        out["launches"] = len(rows)
        out["chain_over_wg"] = out["chain_cycles_q50"] / out["wg_cycles_q50"]
        out["post_chain_cycles"] = out["drone_wave_end"] - out["chain_done"]
        import json
        print(json.dumps(out), flush=True)
        return
    if len(sys.argv) >= 5:   # one config: mode E n m [G B]
        a = sys.argv[1:]
        geom = (int(a[4]), int(a[5])) if len(a) >= 6 else (None, None)
        trace(a[0], int(a[1]), int(a[2]), int(a[3]), "f64", *geom)
        return
    precs = sys.argv[1:] or ["f64"]
    for prec in precs:
        trace("ctde", 4096, 4, 16, prec)
        trace("ctde", 4096, 4, 16, prec, 4, 128)
        trace("ctde", 4096, 4, 16, prec, 8, 256)
        trace("ctde", 4096, 4, 16, prec, 4, 256)
        trace("ctde", 4096, 2, 8, prec, 4, 128)



def host_rate(mode="ctde", E=4096, n=4, m=16, prec="f64", k=500):
    """Host submission cost per step (loop without sync) vs. the synchronised per-step time."""
    import time
    b = HerdBatch(E, n, m, mode=mode, precision=prec)
    b.reset()
    for _ in range(50):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host submit {1e6 * (t1 - t0) / k:.1f} us/step, synchronised {1e6 * (t2 - t0) / k:.1f} us/step")
    b.close()



def back_to_back(mode="ctde", E=4096, n=4, m=16, prec="f64", k=12):
    """Timestamps of k back-to-back launches: per-kernel span and the gap to the previous kernel."""
    L = _lib.lib()
    b = HerdBatch(E, n, m, mode=mode, precision=prec)
    g, blk, lds, kv = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int32()
    L.ch__geometry(b.handle, ctypes.byref(g), ctypes.byref(blk), ctypes.byref(lds), ctypes.byref(kv))
    grid = (E + g.value - 1) // g.value
    ts = torch.zeros((k, grid, 128), dtype=torch.int64, device=b.device)
    b.reset()
    for _ in range(250):
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    for i in range(k):
        L.ch__set_tstamp(b.handle, ctypes.c_void_p(ts[i].data_ptr()))
        b.step(random_actions=True, autoreset=True, terminal_obs=False)
    torch.cuda.synchronize()
    L.ch__set_tstamp(b.handle, None)
    t = ts.cpu().numpy()
    prev_end = None
    for i in range(k):
        w0, w1 = t[i, :, 0].min(), t[i, :, 1].max()
        gap = "" if prev_end is None else f" gap {(w0 - prev_end) / 100.0:.1f}us"
        nres = int((t[i, :, 6] != 0).sum())
        print(f" kernel {i}: span {(w1 - w0) / 100.0:.1f}us{gap} | WG dur max {(t[i, :, 1] - t[i, :, 0]).max() / 100.0:.1f}us")
        prev_end = w1
    b.close()


if __name__ == "__main__":
    host_rate()
    back_to_back()
    if len(sys.argv) > 1:
        main()
