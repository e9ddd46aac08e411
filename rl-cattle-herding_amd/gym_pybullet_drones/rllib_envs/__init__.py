from gym_pybullet_drones.rllib_envs.MARLCattleAviary import MARLCattleAviary  # noqa: F401
