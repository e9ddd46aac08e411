"""``Logger``, the flight log ``CTDECattleHerder.py:40`` imports (its use there is commented out, :193-215).

Restates the reference's ``utils/Logger.py:9-205``: per-drone timestamps, 16 state rows and 12 control rows,
``log`` with the reference's column reordering, ``save`` (``.npy``-named ``np.savez``) and ``save_as_csv``
(one ``t, value`` file per quantity).  The plotting is outside the hot path; ``plot`` draws the
same 10 × 2 grid of state rows with matplotlib, imported only when called.
"""
import os
from datetime import datetime

import numpy as np

# save_as_csv: file stem -> state row (reference Logger.py:146-201); the *r files are finite differences
_CSV_ROWS = (("x", 0), ("y", 1), ("z", 2), ("r", 6), ("p", 7), ("ya", 8), ("vx", 3), ("vy", 4), ("vz", 5),
             ("wx", 9), ("wy", 10), ("wz", 11))
_CSV_RATES = (("rr", 6), ("pr", 7), ("yar", 8))


class Logger(object):
    """Stores, saves and plots the kinematics and RPMs of one or more drones."""

    def __init__(self, logging_freq_hz: int, output_folder: str = "results", num_drones: int = 1,
                 duration_sec: int = 0, colab: bool = False):
        self.COLAB = colab
        self.OUTPUT_FOLDER = output_folder
        if not os.path.exists(self.OUTPUT_FOLDER):
            os.mkdir(self.OUTPUT_FOLDER)
        self.LOGGING_FREQ_HZ = logging_freq_hz
        self.NUM_DRONES = num_drones
        self.PREALLOCATED_ARRAYS = duration_sec != 0
        cols = duration_sec * self.LOGGING_FREQ_HZ
        self.counters = np.zeros(num_drones)
        self.timestamps = np.zeros((num_drones, cols))
        # rows: pos xyz, vel xyz, roll pitch yaw, ang vel xyz, rpm0-3
        self.states = np.zeros((num_drones, 16, cols))
        # rows: target pos xyz, vel xyz, rpy, ang vel xyz
        self.controls = np.zeros((num_drones, 12, cols))

    def log(self, drone: int, timestamp, state, control=np.zeros(12)):
        """Log one step of one drone; ``state`` is the (20,) kinematic vector (pos, quat, rpy, vel, ang vel,
        rpm) and is reordered into the 16 state rows (reference ``Logger.py:83-119``)."""
        if drone < 0 or drone >= self.NUM_DRONES or timestamp < 0 or len(state) != 20 or len(control) != 12:
            print("[ERROR] in Logger.log(), invalid data")
        k = int(self.counters[drone])
        if k >= self.timestamps.shape[1]:
            self.timestamps = np.concatenate((self.timestamps, np.zeros((self.NUM_DRONES, 1))), axis=1)
            self.states = np.concatenate((self.states, np.zeros((self.NUM_DRONES, 16, 1))), axis=2)
            self.controls = np.concatenate((self.controls, np.zeros((self.NUM_DRONES, 12, 1))), axis=2)
        elif not self.PREALLOCATED_ARRAYS and self.timestamps.shape[1] > k:
            k = self.timestamps.shape[1] - 1
        self.timestamps[drone, k] = timestamp
        self.states[drone, :, k] = np.hstack([state[0:3], state[10:13], state[7:10], state[13:20]])
        self.controls[drone, :, k] = control
        self.counters[drone] = k + 1

    def _stamp(self):
        return datetime.now().strftime("%m.%d.%Y_%H.%M.%S")

    def save(self):
        """``np.savez`` of timestamps, states and controls into ``save-flight-<date>.npy``."""
        with open(os.path.join(self.OUTPUT_FOLDER, "save-flight-" + self._stamp() + ".npy"), "wb") as f:
            np.savez(f, timestamps=self.timestamps, states=self.states, controls=self.controls)

    def save_as_csv(self, comment: str = ""):
        """One ``t, value`` CSV per logged quantity and drone, in ``save-flight-<comment>-<date>/``."""
        d = os.path.join(self.OUTPUT_FOLDER, "save-flight-" + comment + "-" + self._stamp())
        os.makedirs(d, exist_ok=True)
        t = np.arange(0, self.timestamps.shape[1] / self.LOGGING_FREQ_HZ, 1 / self.LOGGING_FREQ_HZ)

        def put(name, values):
            with open(os.path.join(d, name + ".csv"), "wb") as f:
                np.savetxt(f, np.transpose(np.vstack([t, values])), delimiter=",")

        for i in range(self.NUM_DRONES):
            s = self.states[i]
            for stem, row in _CSV_ROWS:
                put(stem + str(i), s[row, :])
            for stem, row in _CSV_RATES:
                put(stem + str(i), np.hstack([0, (s[row, 1:] - s[row, :-1]) * self.LOGGING_FREQ_HZ]))
            for m in range(4):
                put("rpm%d-%d" % (m, i), s[12 + m, :])
            for m in range(4):
                put("pwm%d-%d" % (m, i), (s[12 + m, :] - 4070.3) / 0.2685)

    def plot(self, pwm=False):
        """Plot every state row against time, one panel per quantity, one line per drone."""
        import matplotlib.pyplot as plt
        t = np.arange(0, self.timestamps.shape[1] / self.LOGGING_FREQ_HZ, 1 / self.LOGGING_FREQ_HZ)
        labels = ("x", "y", "z", "vx", "vy", "vz", "r", "p", "y", "wx", "wy", "wz",
                  "PWM0" if pwm else "RPM0", "PWM1" if pwm else "RPM1", "PWM2" if pwm else "RPM2",
                  "PWM3" if pwm else "RPM3")
        fig, axs = plt.subplots(8, 2)
        for k, lab in enumerate(labels):
            ax = axs[k % 8, k // 8]
            for j in range(self.NUM_DRONES):
                v = self.states[j, k, :]
                if pwm and k >= 12:
                    v = (v - 4070.3) / 0.2685
                ax.plot(t, v, label="drone_" + str(j))
            ax.set_xlabel("time")
            ax.set_ylabel(lab)
            ax.grid(True)
        fig.subplots_adjust(left=.06, bottom=.05, right=.99, top=.98, wspace=.15, hspace=.0)
        if self.COLAB:
            plt.savefig(os.path.join("results", "output_figure.png"))
        else:
            plt.show()
