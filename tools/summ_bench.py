"""One line per bench log: step rate, policy rollout rate, forward time and the PPO legs (rate, us per step)."""
import glob
import json
import sys

for pat in sys.argv[1:]:
    for f in sorted(glob.glob(pat)):
        for line in open(f):
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            p = d.get("policy_rollout") or {}
            s = f"{f}: step {d['value'] / 1e6:.1f} M ({d['ms_per_step'] * 1e3:.2f} us, kernel {d['roofline']['kernel_us']:.2f})"
            if p:
                s += f" | policy {p['env_steps_per_s'] / 1e6:.1f} M fwd {p['forward_us']:.2f} us"
                for k, v in p.items():
                    if k.startswith("ppo"):
                        s += f" | {k} {v['env_steps_per_s'] / 1e6:.1f} M {v['ms_per_step'] * 1e3:.1f} us"
            print(s)
