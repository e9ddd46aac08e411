"""Host-side evaluation logger for single-env evaluation runs (reference: utils/evaluation.py:5-94,
BaseAviary.update_evaluation_metrics / evaluation_episode_trigger, sb3_envs/BaseAviary.py:1406-1450).

Records per-step drone/cattle poses and velocities, effectiveness and episode time, and writes the
reference's ``evaluation_data.pkl`` schema.  Two deliberate differences, both documented in
DESIGN.md: per-step rows are copies (the reference appends aliases of arrays it keeps mutating), and
recording only happens while ``is_evaluating`` is set by the caller (the reference appends on every
training step without bound).
"""
import os
import pickle

import numpy as np


def herding_effectiveness(cattle_xy, drone_xy):
    """evaluate_herding_effectiveness (evaluation.py:100-138): % of cows with non-zero winding number
    w.r.t. the polygon of drone positions in index order."""
    c = np.asarray(cattle_xy, np.float64).reshape(-1, 2)
    p = np.asarray(drone_xy, np.float64).reshape(-1, 2)
    if len(c) == 0:
        return 0
    q = np.roll(p, -1, axis=0)
    x1, y1, x2, y2 = p[:, 0][None], p[:, 1][None], q[:, 0][None], q[:, 1][None]
    px, py = c[:, 0][:, None], c[:, 1][:, None]
    il = (x2 - x1) * (py - y1) - (px - x1) * (y2 - y1)
    up = (y1 <= py) & (y2 > py) & (il > 0)
    down = (y1 > py) & (y2 <= py) & (il < 0)
    wn = up.sum(1) - down.sum(1)
    return np.count_nonzero(wn) / len(c) * 100


class Evaluator:
    def __init__(self):
        self.active = True
        for k in ("total_drone_distances", "total_time_taken", "total_effectiveness", "total_number_of_drones",
                  "drone_distances_per_step", "effectiveness_per_step", "time_per_step", "drone_poses_per_step",
                  "cattle_poses_per_step", "drone_vel_per_step", "cattle_vel_per_step"):
            setattr(self, k, [])
        self._clear_current()
        self._last_pos = None
        self._dist = None
        self._prev_cattle_vel = None

    def _clear_current(self):
        self.curr = {k: [] for k in ("drone_poses", "cattle_poses", "drone_vel", "cattle_vel", "drone_distances",
                                     "effectiveness", "time")}

    def start_episode(self, s, n):
        # _housekeeping initialises the distance accumulators to the start positions and reset()
        # zeroes last_drones_pos (BaseAviary.py:317, 683-688)
        self._dist = [np.array(s["drone_pos"][0, i, :2], np.float64) for i in range(n)]
        self._last_pos = [np.zeros(2) for _ in range(n)]
        self._prev_cattle_vel = np.array(s["cow_vel"][0], np.float64)

    def record_step(self, s, n, m, ctrl_freq, counter_inc=4):
        if self._dist is None:
            self.start_episode(s, n)
        dp = np.array(s["drone_pos"][0, :n, :2], np.float64)
        for i in range(n):
            self._dist[i] = self._dist[i] + np.linalg.norm(self._last_pos[i] - dp[i]) * 1.7
            self._last_pos[i] = dp[i].copy()
        cp = np.array(s["cow_pos"][0, :m], np.float64)
        # update_evaluation_metrics runs before the step counter advances (BaseAviary.py:462-464)
        t = (int(s["step_counter"][0]) - counter_inc) / ctrl_freq
        row = {"drone_poses": dp, "cattle_poses": cp, "drone_vel": np.array(s["drone_vel"][0, :n, :2]),
               "cattle_vel": self._prev_cattle_vel[:m].copy(), "drone_distances": [d.copy() for d in self._dist],
               "effectiveness": herding_effectiveness(cp, dp), "time": t}
        self._prev_cattle_vel = np.array(s["cow_vel"][0], np.float64)
        for k, v in row.items():
            self.curr[k].append(v)

    def end_episode(self, n, ep_time):
        """evaluation_episode_trigger fires once per _computeTruncated call — twice per step
        (CattleAviary.py:315 and BaseAviary.py:460) — hence an empty second episode, as in the
        reference's own evaluation_data.pkl."""
        for _ in range(2):
            eff = self.curr["effectiveness"][-1] if self.curr["effectiveness"] else 0
            self.total_drone_distances.append([d.copy() for d in (self._dist or [])])
            self.total_number_of_drones.append(n)
            self.total_time_taken.append(ep_time)
            self.total_effectiveness.append(eff)
            self.drone_poses_per_step.append(self.curr["drone_poses"])
            self.cattle_poses_per_step.append(self.curr["cattle_poses"])
            self.drone_vel_per_step.append(self.curr["drone_vel"])
            self.cattle_vel_per_step.append(self.curr["cattle_vel"])
            self.drone_distances_per_step.append(self.curr["drone_distances"])
            self.time_per_step.append(self.curr["time"])
            self.effectiveness_per_step.append(self.curr["effectiveness"])
            self._clear_current()

    def save_evaluation_data(self, save_path="evaluation_data.pkl"):
        data = {"distances": self.total_drone_distances, "num_drones": self.total_number_of_drones,
                "time_taken": self.total_time_taken, "effectiveness": self.total_effectiveness,
                "distances_per_step": self.drone_distances_per_step, "time_per_step": self.time_per_step,
                "effectiveness_per_step": self.effectiveness_per_step,
                "drone_poses_per_step": self.drone_poses_per_step, "cattle_poses_per_step": self.cattle_poses_per_step,
                "drone_vel_per_step": self.drone_vel_per_step, "cattle_vel_per_step": self.cattle_vel_per_step}
        with open(save_path, "wb") as f:
            pickle.dump(data, f)
        print(f"Evaluation data saved to {os.path.abspath(save_path)}")
