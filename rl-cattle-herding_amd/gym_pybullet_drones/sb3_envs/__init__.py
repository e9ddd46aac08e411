from gym_pybullet_drones.sb3_envs.CattleAviary import CattleAviary  # noqa: F401
