"""Evaluation logging of the reference (utils/evaluation.py:5-94 ``evaluator``; BaseAviary
``update_evaluation_metrics`` / ``evaluation_episode_trigger``, sb3_envs/BaseAviary.py:1406-1450) over
the device batch.

``Evaluator`` keeps the reference's attributes and methods, so ``save_evaluation_data`` writes the same
``evaluation_data.pkl`` schema.  ``EvalTracker`` is the env-side half of BaseAviary: the per-episode list
``episode_drone_distances`` and the two call sites.  The per-drone distance itself is accumulated on the
device by the step kernel every step (ch_config.eval_metrics, ``HerdBatch.eval_distances``), so only
logging needs host data.

The reference's data flow is reproduced as it is, because it is what its pickle holds:
* the distance "2-vector" of a drone starts at (0, 0) -- ``_housekeeping`` zeroes ``self.pos`` before it
  copies it (BaseAviary.py:567, 683-688) -- and both components receive the same additions;
* every logged distance row is the env's list object itself, mutated in place afterwards, so all rows of
  an episode show its final distances (and an episode's first row is the previous episode's list, see
  below);
* ``evaluation_episode_trigger`` fires from ``_computeTruncated`` at the time limit, which ``step`` runs
  twice -- inside ``_computeReward`` and after it (CattleAviary.py:314-315, BaseAviary.py:458-460) -- both
  before ``update_evaluation_metrics`` (462): two episode entries per time-out, the second empty, and the
  time-out step itself logged into the next episode's rows.
One deliberate difference: rows are appended only while ``is_evaluating`` is set (the reference appends
on every training step, without bound); distances are accumulated on every step regardless.
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


def failure_truncation(state, e, n, target_alt=0.45, max_alt_error=0.27, collision=0.2, max_formation=8.0,
                       mission_boundary=15.0):
    """Conditions 1-4 of CattleAviary._computeTruncated (CattleAviary.py:513-542) on env ``e`` of a state
    dict (``HerdBatch.get_state``) with ``n`` live drones: altitude loss, a drone pair closer than the
    collision threshold, a drone isolated from all others, the formation too far from the herd."""
    pos = np.asarray(state["drone_pos"][e, :n], np.float64)
    if np.any(np.abs(pos[:, 2] - target_alt) > max_alt_error):
        return True
    xy = pos[:, :2]
    d = np.linalg.norm(xy[:, None, :] - xy[None, :, :], axis=-1)
    iu = np.triu_indices(n, 1)
    if np.any(d[iu] < collision):
        return True
    np.fill_diagonal(d, np.inf)
    if np.any(np.all(d > max_formation, axis=1)):
        return True
    herd = np.asarray(state["cow_pos"][e], np.float64).mean(axis=0)
    return bool(np.linalg.norm(xy.mean(axis=0) - herd) > mission_boundary)


class Evaluator:
    """utils/evaluation.py:5-94 (``evaluator``): episode-level and per-step lists."""

    def __init__(self):
        self.total_drone_distances = []
        self.total_time_taken = []
        self.total_effectiveness = []
        self.total_number_of_drones = []
        self.drone_distances_per_step = []
        self.effectiveness_per_step = []
        self.time_per_step = []
        self.drone_poses_per_step = []
        self.cattle_poses_per_step = []
        self.drone_vel_per_step = []
        self.cattle_vel_per_step = []
        self._clear_current()

    def _clear_current(self):
        self.curr_drone_poses, self.curr_cattle_poses, self.curr_drone_vel, self.curr_cattle_vel = [], [], [], []
        self.curr_drone_distances, self.curr_effectiveness, self.curr_time = [], [], []

    def append_timestep_data(self, drone_distances, timestep_time, effectiveness, drone_poses, cattle_poses, drone_vel,
                             cattle_vel):
        self.curr_drone_distances.append(drone_distances)
        self.curr_time.append(timestep_time)
        self.curr_effectiveness.append(effectiveness)
        self.curr_drone_poses.append(drone_poses)
        self.curr_cattle_poses.append(cattle_poses)
        self.curr_drone_vel.append(drone_vel)
        self.curr_cattle_vel.append(cattle_vel)

    def append_episode_data(self, drone_distances, num_drones, time, effectiveness):
        self.total_drone_distances.append(drone_distances)
        self.total_number_of_drones.append(num_drones)
        self.total_time_taken.append(time)
        self.total_effectiveness.append(effectiveness)
        self.drone_poses_per_step.append(self.curr_drone_poses)
        self.cattle_poses_per_step.append(self.curr_cattle_poses)
        self.drone_vel_per_step.append(self.curr_drone_vel)
        self.cattle_vel_per_step.append(self.curr_cattle_vel)
        self.drone_distances_per_step.append(self.curr_drone_distances)
        self.time_per_step.append(self.curr_time)
        self.effectiveness_per_step.append(self.curr_effectiveness)
        self._clear_current()

    def evaluation_data(self):
        """The dict save_evaluation_data pickles (evaluation.py:73-90)."""
        return {"distances": self.total_drone_distances, "num_drones": self.total_number_of_drones,
                "time_taken": self.total_time_taken, "effectiveness": self.total_effectiveness,
                "distances_per_step": self.drone_distances_per_step, "time_per_step": self.time_per_step,
                "effectiveness_per_step": self.effectiveness_per_step,
                "drone_poses_per_step": self.drone_poses_per_step, "cattle_poses_per_step": self.cattle_poses_per_step,
                "drone_vel_per_step": self.drone_vel_per_step, "cattle_vel_per_step": self.cattle_vel_per_step}

    def save_evaluation_data(self, save_path="evaluation_data.pkl"):
        with open(save_path, "wb") as f:
            pickle.dump(self.evaluation_data(), f)
        print(f"Evaluation data saved to {os.path.abspath(save_path)}")


class EvalTracker:
    """BaseAviary's side of the logging for env ``e`` of a batch: ``episode_drone_distances`` (one list per
    episode, its arrays updated in place from the device accumulator) and the two call sites."""

    def __init__(self, evaluator, env_index=0):
        self.evaluator = evaluator
        self.e = env_index
        self.episode_drone_distances = []
        self._prev_cattle_vel = None

    def on_reset(self, state, n):
        """_housekeeping (BaseAviary.py:683-688): a new list, every entry (0, 0)."""
        self.episode_drone_distances = [np.zeros(2) for _ in range(n)]
        self._prev_cattle_vel = np.array(state["cow_vel"][self.e], np.float64)

    def set_step_start(self, state):
        """The cattle velocities at the start of a step: what the read-back of that step returns (the
        flock update of the step only reaches Bullet afterwards, BaseAviary.py:452-455, 1398-1400)."""
        self._prev_cattle_vel = np.array(state["cow_vel"][self.e], np.float64)

    def _sync_distances(self, dist_row):
        for i, d in enumerate(self.episode_drone_distances):
            d[:] = dist_row[i]   # in place: rows logged earlier in the episode see it (the reference's aliasing)

    def _poses(self, state, n, m):
        e = self.e
        return (np.array(state["drone_pos"][e, :n, :2], np.float64), np.array(state["cow_pos"][e, :m], np.float64))

    def after_step(self, state, dist_row, n, m, step_counter_before, ctrl_freq, episode_len_sec):
        """One env.step's logging, in the reference's order: the time-out triggers of the two
        _computeTruncated calls (CattleAviary.py:545-548), then update_evaluation_metrics (BaseAviary.py:462)."""
        self._sync_distances(dist_row)
        drone_poses, cattle_poses = self._poses(state, n, m)
        ep_time = step_counter_before / ctrl_freq
        eff = herding_effectiveness(cattle_poses, drone_poses)
        # _computeTruncated returns at the first failure condition (CattleAviary.py:513-542); the time-out
        # branch with its trigger (545-548) is reached only when none of them holds
        if ep_time > episode_len_sec and not failure_truncation(state, self.e, n):
            for _ in range(2):   # evaluation_episode_trigger (BaseAviary.py:1439-1450)
                self.evaluator.append_episode_data(self.episode_drone_distances, n, ep_time, eff)
        drone_vel = np.array(state["drone_vel"][self.e, :n, :2], np.float64)
        cattle_vel = self._prev_cattle_vel[:m].copy() if self._prev_cattle_vel is not None else np.zeros((m, 2))
        self.evaluator.append_timestep_data(self.episode_drone_distances, ep_time, eff, drone_poses, cattle_poses,
                                            drone_vel, cattle_vel)
        self.set_step_start(state)
